"""Federation on the fused HIP engine (one GPU, several clients in-process)."""
import numpy as np
import pytest
import torch

from gfedntm_amd.data.synthetic import generate_synthetic
from gfedntm_amd.federation.data import ClientCorpus
from gfedntm_amd.federation.runner import LocalFederation
from gfedntm_amd.utils.config import load_config

pytestmark = pytest.mark.gpu


def _params(**kw):
    p = dict(load_config().training_params)
    p.update(num_epochs=2, batch_size=32, hidden_sizes=(50, 50), n_components=10)
    p.update(kw)
    return p


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_fused_federation_round_is_fedavg(model_type):
    sc = generate_synthetic(vocab_size=400, n_topics=10, n_docs=60, n_nodes=3, frozen_topics=2,
                            nwords=(30, 60), seed=4)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(3)]
    fed = LocalFederation(corpora, _params(model_type=model_type), max_iters=1, device="cuda",
                          backend="fused", seed=1, graph=False)
    assert all(c.tm.backend == "fused" for c in fed.clients)
    w = fed.weights
    # one round by hand: local steps, then the expected sum of pre-scaled states
    for c in fed.clients:
        c.local_step(0)
    torch.cuda.synchronize()
    pre = [c.shared.clone() for c in fed.clients]        # already scaled by w_i in-kernel
    fed.agg.average_([c.shared for c in fed.clients], prescaled=True)
    expect = sum(pre)
    for c in fed.clients:
        torch.testing.assert_close(c.shared, expect, rtol=0, atol=0)
    # the in-kernel pre-scale is w_i times the local state: undo it on one client
    # and check that its unscaled state is finite and non-trivial
    un = pre[0] / w[0]
    assert torch.isfinite(un).all() and un.abs().max() > 0


def test_fused_federation_trains():
    sc = generate_synthetic(vocab_size=500, n_topics=10, n_docs=200, n_nodes=2, frozen_topics=2,
                            nwords=(40, 80), seed=5)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    fed = LocalFederation(corpora, _params(num_epochs=30), max_iters=300, device="cuda",
                          backend="fused", seed=2, graph=True)
    fed.run()
    for c in fed.clients:
        h = c.loss_history()[:300]
        assert np.isfinite(h).all()
        assert h[-30:].mean() < 0.9 * h[:30].mean()
    a, b = (c.shared for c in fed.clients)
    torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_fused_checkpoint_resume_is_bitwise(tmp_path, model_type):
    """Fused engine + round-graph replay: checkpoint at round 7, resume in a fresh
    federation, finish at round 15 -- the flat state (parameters, BN buffers), the
    optimizer moments and the loss history equal an uninterrupted run bit for bit
    (Philox draws keyed by (seed, step); the device beta^t products travel verbatim)."""
    sc = generate_synthetic(vocab_size=500, n_topics=10, n_docs=90, n_nodes=2, frozen_topics=2,
                            nwords=(40, 80), seed=6)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    kw = dict(device="cuda", backend="fused", seed=3, graph=True)
    full = LocalFederation(corpora, _params(model_type=model_type), max_iters=15, **kw)
    full.run()
    a = LocalFederation(corpora, _params(model_type=model_type), max_iters=7,
                        checkpoint_dir=str(tmp_path), checkpoint_every=7, **kw)
    a.run()
    b = LocalFederation(corpora, _params(model_type=model_type), max_iters=15,
                        checkpoint_dir=str(tmp_path), checkpoint_every=100, **kw)
    assert b.round == 7 and b.round_graph
    b.run()
    for cf, cb in zip(full.clients, b.clients):
        ef, eb = cf.tm.engine, cb.tm.engine
        assert torch.equal(cb.tm.flat.buffer, cf.tm.flat.buffer)
        assert torch.equal(eb.exp_avg, ef.exp_avg) and torch.equal(eb.exp_avg_sq, ef.exp_avg_sq)
        assert torch.equal(eb.loss_hist[:15], ef.loss_hist[:15])
        assert cb.current_epoch == cf.current_epoch and cb.samples_processed == cf.samples_processed
        assert int(eb.adam_t.item()) == int(ef.adam_t.item()) == 15
