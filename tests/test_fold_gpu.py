"""The batched round's FedAvg inside the update kernels' epilogues (round 6).

csrc/prodlda.hip gfk_bwd_fold_k and csrc/update.hip gfk_win_fold_k take one tile for ALL the
batched clients, in client order, and write the client-order sum of their pre-scaled Adam
results once; the golden is the same batched steps followed by the fold kernel
(csrc/comm.hip gfk_local_fedavg, GFEDNTM_FOLD=0).  Reference round: server.py:477-521.
"""
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
    p.update(num_epochs=2, batch_size=64, hidden_sizes=(50, 50), n_components=50)
    p.update(kw)
    return p


def _corpora(n, vocab=5000, docs=None, seed=21):
    # uneven shards: different FedAvg weights and different partial last batches
    sc = generate_synthetic(vocab_size=vocab, n_topics=50, n_docs=docs or 150 * n, n_nodes=n,
                            frozen_topics=5, nwords=(150, 250), seed=seed)
    return [ClientCorpus(synthetic=sc, node=i) for i in range(n)]


def _run(monkeypatch, corpora, fold: str, iters: int, **kw):
    monkeypatch.setenv("GFEDNTM_FOLD", fold)
    fed = LocalFederation(corpora, _params(**kw), max_iters=iters, device="cuda",
                          backend="fused", seed=7, round_batched=True)
    fed.run()
    torch.cuda.synchronize()
    return fed


def _state(fed):
    out = []
    for c in fed.clients:
        e = c.tm.engine
        out += [c.tm.flat.buffer.clone(), e.exp_avg.clone(), e.exp_avg_sq.clone(),
                e.loss_hist.clone()]
    return out


def _assert_same(a, b):
    """Bitwise equality of two runs' states; on a mismatch, name the client, buffer and
    flat-layout slot of the first differing element."""
    sa, sb = _state(a), _state(b)
    for i, (x, y) in enumerate(zip(sa, sb)):
        if torch.equal(x, y):
            continue
        c, kind = divmod(i, 4)
        j = int(torch.nonzero(x != y)[0])
        slot = None
        if kind < 3:
            for k, s in a.clients[c].tm.flat.slots.items():
                if s.offset <= j < s.offset + s.numel:
                    slot = (k, j - s.offset)
        n = int((x != y).sum())
        raise AssertionError(f"client {c} {['param', 'exp_avg', 'exp_avg_sq', 'loss'][kind]}: "
                             f"{n} elements differ, first {j} {slot}: {float(x[j])!r} vs {float(y[j])!r}")


@pytest.mark.parametrize("n_clients,iters", [(8, 40), (3, 25)])
def test_fold_in_epilogue_is_bitwise_fold_kernel(monkeypatch, n_clients, iters):
    """Several epochs (partial last batches, uneven weights): the in-epilogue FedAvg gives
    the batched steps + fold kernel's parameters, Adam moments and losses bit for bit --
    8 clients (one per XCD) and 3 (no power of two)."""
    corpora = _corpora(n_clients, docs=(1100 if n_clients == 8 else 500))
    a = _run(monkeypatch, corpora, "1", iters)
    b = _run(monkeypatch, corpora, "0", iters)
    assert a.fold_plan == "in-epilogue" and b.fold_plan == "fold kernel"
    _assert_same(a, b)
    s0 = a.clients[0].shared
    for c in a.clients[1:]:
        assert torch.equal(c.shared, s0)
    assert np.isfinite(a.clients[0].loss_history()[:iters]).all()


def test_fold_learn_priors_and_leftover_pieces(monkeypatch):
    """Learned priors (vector jobs without a source: the gradient slot) and a vocabulary
    whose batch-norm buffers span several leftover pieces."""
    corpora = _corpora(4, vocab=3000, docs=600, seed=5)
    a = _run(monkeypatch, corpora, "1", 12, learn_priors=True)
    b = _run(monkeypatch, corpora, "0", 12, learn_priors=True)
    assert a.fold_plan == "in-epilogue"
    assert a._batched._fold.n_left >= 3
    _assert_same(a, b)


def test_fold_reason_refuses_other_plans():
    """Configurations outside the fold kernels' plan keep the fold kernel, with a reason."""
    from gfedntm_amd.ops.engine import BatchedSteps
    corpora = _corpora(2, vocab=800, docs=200, seed=3)
    fed = LocalFederation(corpora, _params(batch_size=32, n_components=20), max_iters=1,
                          device="cuda", backend="fused", seed=7, round_batched=True)
    bs = BatchedSteps([c.tm.engine for c in fed.clients])
    bs.prepare()
    assert "batch 64" in bs.fold_reason()
    with pytest.raises(ValueError):
        from gfedntm_amd.ops import kernel_abi as abi
        bs.set_fold(abi.FOLD_ALL)
