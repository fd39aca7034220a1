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


def test_grpc_two_fused_gpu_clients_in_one_process(tmp_path):
    """Two fused-engine clients served from ONE process over the reference gRPC protocol:
    their graph captures and device synchronisations must not overlap (the process-wide
    device lock and thread-local capture mode in utils.misc.graph_capture); each client
    ends holding the server's aggregate of the last round."""
    import socket
    import threading
    from gfedntm_amd.federation.grpc_transport import FederationServicer, run_client, serve
    params = _params(num_epochs=100, batch_size=32, hidden_sizes=(32, 32), n_components=10)
    sc = generate_synthetic(vocab_size=400, n_topics=10, n_docs=120, n_nodes=2, frozen_topics=3,
                            nwords=(30, 60), seed=4)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    base = None
    for b in range(47000, 60000, 41):
        try:
            for p in range(b, b + 3):
                with socket.socket() as s:
                    s.bind(("127.0.0.1", p))
            base = b
            break
        except OSError:
            continue
    iters = 6
    svc = FederationServicer(params, "avitm", 2, iters, client_host="127.0.0.1", base_port=base,
                             save_server=str(tmp_path / "server" / ""), wait_timeout=60)
    server = serve(svc, base)
    clients, errors = {}, []

    def run(i):
        try:
            clients[i] = run_client(corpora[i - 1], i, f"127.0.0.1:{base}", base + i,
                                    backend="fused", device="cuda", seed=0,
                                    save_client=str(tmp_path / "client"), timeout=60,
                                    max_iters=iters)
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)

    ts = [threading.Thread(target=run, args=(i,)) for i in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(100)
    assert svc.done.wait(10)
    server.stop(0)
    assert not errors, errors
    assert svc.error is None and svc.rounds == iters
    for c in clients.values():
        sd = c.tm.model.state_dict()
        for k, v in svc.aggregated.items():
            np.testing.assert_allclose(sd[k].cpu().numpy(), v, rtol=0, atol=1e-6, err_msg=k)


def _ctx_corpora(n_nodes, C, seed=7, labels=0):
    sc = generate_synthetic(vocab_size=400, n_topics=10, n_docs=80, n_nodes=n_nodes,
                            frozen_topics=2, nwords=(30, 60), seed=seed)
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n_nodes):
        emb = rng.standard_normal((sc.counts[i].shape[0], C)).astype(np.float32)
        out.append(ClientCorpus(synthetic=sc, node=i, embeddings=emb))
    return out


@pytest.mark.parametrize("model_type,C", [("ctm", 64), ("zeroshot", 64), ("ctm", 30)])
def test_round_graph_matches_per_client_graphs(model_type, C):
    """CombinedTM / ZeroShotTM federations: the one-graph-per-round path equals the
    per-client step graphs + eager FedAvg kernel bit for bit.  C = 30 (C % 4 != 0) puts
    CombinedTM on the host-GEMM fallback, which must stay out of the round graph."""
    corpora = _ctx_corpora(3, C)
    p = _params(contextual_size=C)
    kw = dict(model_type=model_type, max_iters=6, device="cuda", backend="fused", seed=5)
    rg = LocalFederation(corpora, p, round_graph=True, round_batched=False, **kw)
    ref = LocalFederation(corpora, p, round_graph=False, **kw)
    fallback = any(c.tm.engine.host_gemm_fallback for c in rg.clients)
    assert fallback == (C % 4 != 0)
    assert rg.round_graph == (not fallback) and not ref.round_graph
    rg.run()
    ref.run()
    for a, b in zip(rg.clients, ref.clients):
        assert torch.equal(a.tm.flat.buffer, b.tm.flat.buffer)
        assert torch.equal(a.tm.engine.loss_hist[:6], b.tm.engine.loss_hist[:6])


def test_round_graph_recaptures_after_engine_change():
    """An engine reconfigured between run() calls (here: a new learning rate, which
    rebuilds the optimizer tables and invalidates the engine's graph) must not be
    replayed through a stale round graph."""
    sc = generate_synthetic(vocab_size=400, n_topics=10, n_docs=90, n_nodes=2, frozen_topics=2,
                            nwords=(30, 60), seed=8)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    kw = dict(device="cuda", backend="fused", seed=9)
    a = LocalFederation(corpora, _params(), max_iters=9, round_graph=True, round_batched=False, **kw)
    b = LocalFederation(corpora, _params(), max_iters=9, round_graph=False, **kw)
    for fed in (a, b):
        fed.max_iters = 4           # (the clients' batch plans cover 9 rounds)
        fed.run()
        for c in fed.clients:
            c.tm.engine.set_lr(5e-3)
        fed.max_iters = 9
        fed.run()
    assert a.round == b.round == 9
    for x, y in zip(a.clients, b.clients):
        assert torch.equal(x.tm.flat.buffer, y.tm.flat.buffer)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_batched_round_matches_branch_round(model_type):
    """One launch per phase for all clients (grid z = client, the kernels' batched
    instances) == one graph branch per client (the by-value instances): after one round
    within fp32 rounding (the two instances are compiled separately, so FMA contraction
    may differ), and two batched runs are bitwise equal."""
    sc = generate_synthetic(vocab_size=500, n_topics=10, n_docs=70, n_nodes=4, frozen_topics=2,
                            nwords=(30, 60), seed=12)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(4)]
    kw = dict(device="cuda", backend="fused", seed=4)
    p = _params(model_type=model_type)
    a = LocalFederation(corpora, p, max_iters=1, round_batched=True, **kw)
    b = LocalFederation(corpora, p, max_iters=1, round_batched=False, **kw)
    a.run()
    b.run()
    assert a._batched is not None and b._batched is None
    # Adam's first step moves every element by ~lr * sign(g): where the true gradient is
    # ~0 (rounding noise) the two instances may step in opposite directions (<= 2 lr)
    lr = a.clients[0].tm.engine.lr
    for x, y in zip(a.clients, b.clients):
        diff = (x.tm.flat.buffer - y.tm.flat.buffer).abs()
        assert float(diff.max()) <= 2.5 * lr
        assert int((diff > 1e-5).sum()) <= 0.01 * diff.numel()
        torch.testing.assert_close(x.tm.engine.loss_hist[:1], y.tm.engine.loss_hist[:1],
                                   rtol=1e-6, atol=1e-3)
    c = LocalFederation(corpora, p, max_iters=12, round_batched=True, **kw)
    d = LocalFederation(corpora, p, max_iters=12, round_batched=True, **kw)
    c.run()
    d.run()
    for x, y in zip(c.clients, d.clients):
        assert torch.equal(x.tm.flat.buffer, y.tm.flat.buffer)


@pytest.mark.parametrize("strip", ["fill", "keep"])
def test_batched_large_round_variants_match_branch_round(monkeypatch, strip):
    """8 clients at the headline's vocabulary (~74 tiles each): the batched launch switches
    the strip forward to 3-4 tiles per 16-wave workgroup ("fill", the default; "keep": the
    engines' one-tile-per-workgroup grids in rounds of the CUs), post_bwd to two rows per workgroup with its batch-level
    workgroup in row_bwd (bit 20), and win_update to its 8-wave tile shape (bit 9: all
    clients' tiles exceed two rounds of 16-wave workgroups), all in the fused update mode.
    The round must still agree with the per-client branch round within fp32 rounding."""
    from gfedntm_amd.ops.engine import (STAGE_FWD_STRIP, STAGE_POST_ROWS2, STAGE_WIN_BATCH8,
                                        UPDATE_FUSED)
    monkeypatch.setenv("GFEDNTM_BATCH_STRIP", strip)
    sc = generate_synthetic(vocab_size=5000, n_topics=50, n_docs=1000, n_nodes=8, frozen_topics=5,
                            nwords=(150, 250), seed=13)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(8)]
    kw = dict(device="cuda", backend="fused", seed=4)
    p = _params(batch_size=64, n_components=50)
    a = LocalFederation(corpora, p, max_iters=1, round_batched=True, **kw)
    b = LocalFederation(corpora, p, max_iters=1, round_batched=False, **kw)
    a.run()
    b.run()
    assert a._batched is not None
    host = a._batched._host
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    assert 8 * (host.n_tiles + 8) > 2 * cu and host.stage_flags & STAGE_WIN_BATCH8, host.n_tiles
    from gfedntm_amd.ops import kernel_abi as abi
    from gfedntm_amd.ops.engine import STAGE_FWD_POSTFOLD
    # the strip forward with the posterior folded in (post_fwd not launched)
    assert host.stage_flags & STAGE_FWD_STRIP
    assert host.stage_flags & STAGE_FWD_POSTFOLD and abi.PH_POST_FWD not in a._batched._phases
    if strip == "fill":
        # (the fewest tiles per workgroup whose 8 clients' workgroups fit one round)
        t = next(t for t in (1, 2, 3, 4) if 8 * -(-host.n_tiles // t) <= cu)
        assert host.dec_grid == -(-host.n_tiles // t)
    else:
        assert host.dec_grid == host.n_tiles and 8 * host.dec_grid > cu
    assert host.stage_flags & STAGE_POST_ROWS2 and host.n_dpart == host.n_tiles
    assert all(c.tm.engine.update_mode == UPDATE_FUSED for c in a.clients)
    lr = a.clients[0].tm.engine.lr
    for x, y in zip(a.clients, b.clients):
        diff = (x.tm.flat.buffer - y.tm.flat.buffer).abs()
        assert float(diff.max()) <= 2.5 * lr
        assert int((diff > 1e-5).sum()) <= 0.01 * diff.numel()
        torch.testing.assert_close(x.tm.engine.loss_hist[:1], y.tm.engine.loss_hist[:1],
                                   rtol=1e-6, atol=1e-3)


def test_batched_ctm_takes_the_large_vocabulary_plan():
    """CombinedTM, 8 clients at V ~ 5-10k (> 64 tiles each): the batched launch's 8 x n_tiles
    vocabulary tiles exceed two rounds of the CUs, so it runs the large-vocabulary shapes
    (stage bits 5 and 12: the forward with all batch rows per tile, the persistent
    pipelined backward) that one client of this size does not use.  The round must agree
    with the per-client branch round (the engines' own plan) within fp32 rounding."""
    from gfedntm_amd.ops.engine import STAGE_CTX_BWDPP, STAGE_CTX_FULL, STAGE_CTX_RS
    C = 64
    sc = generate_synthetic(vocab_size=10000, n_topics=50, n_docs=1000, n_nodes=8, frozen_topics=2,
                            nwords=(150, 250), seed=17)
    rng = np.random.default_rng(17)
    corpora = [ClientCorpus(synthetic=sc, node=i,
                            embeddings=rng.standard_normal((sc.counts[i].shape[0], C)).astype(np.float32))
               for i in range(8)]
    kw = dict(model_type="ctm", device="cuda", backend="fused", seed=4)
    p = _params(batch_size=64, n_components=20, contextual_size=C)
    a = LocalFederation(corpora, p, max_iters=1, round_batched=True, **kw)
    b = LocalFederation(corpora, p, max_iters=1, round_batched=False, **kw)
    e = b.clients[0].tm.engine
    assert not e._m.stage_flags & (STAGE_CTX_FULL | STAGE_CTX_BWDPP)    # one client's plan
    a.run()
    b.run()
    host = a._batched._host
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    assert 8 * host.n_tiles > 2 * cu, host.n_tiles
    assert host.stage_flags & STAGE_CTX_FULL and host.stage_flags & STAGE_CTX_BWDPP
    assert not host.stage_flags & STAGE_CTX_RS and host.ctx_bgrid == cu
    lr = a.clients[0].tm.engine.lr
    for x, y in zip(a.clients, b.clients):
        diff = (x.tm.flat.buffer - y.tm.flat.buffer).abs()
        assert float(diff.max()) <= 2.5 * lr
        assert int((diff > 1e-5).sum()) <= 0.01 * diff.numel()
        torch.testing.assert_close(x.tm.engine.loss_hist[:1], y.tm.engine.loss_hist[:1],
                                   rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("strip", ["fill", "keep"])
def test_batched_lda_decoder_grid_fill(monkeypatch, strip):
    """NeuralLDA, 8 clients at the headline's vocabulary: the batched launch gives each
    decoder workgroup T tiles so the 8 clients' workgroups fit one round of the CUs ("fill",
    the default; "keep": the engines' own grids).  Either way the round agrees with the
    per-client branch round within fp32 rounding."""
    monkeypatch.setenv("GFEDNTM_BATCH_STRIP", strip)
    sc = generate_synthetic(vocab_size=5000, n_topics=50, n_docs=1000, n_nodes=8, frozen_topics=5,
                            nwords=(150, 250), seed=13)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(8)]
    kw = dict(device="cuda", backend="fused", seed=4)
    p = _params(model_type="LDA", batch_size=64, n_components=50)
    a = LocalFederation(corpora, p, max_iters=1, round_batched=True, **kw)
    b = LocalFederation(corpora, p, max_iters=1, round_batched=False, **kw)
    a.run()
    b.run()
    host = a._batched._host
    own = b.clients[0].tm.engine._m.dec_grid
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    if strip == "fill" and 8 * own > cu:
        t = next((t for t in (1, 2, 3, 4) if 8 * -(-host.n_tiles // t) <= cu), None)
        assert host.dec_grid == (-(-host.n_tiles // t) if t else max(1, cu // 8))
    else:
        assert host.dec_grid == own
    lr = a.clients[0].tm.engine.lr
    for x, y in zip(a.clients, b.clients):
        diff = (x.tm.flat.buffer - y.tm.flat.buffer).abs()
        assert float(diff.max()) <= 2.5 * lr
        assert int((diff > 1e-5).sum()) <= 0.01 * diff.numel()
        torch.testing.assert_close(x.tm.engine.loss_hist[:1], y.tm.engine.loss_hist[:1],
                                   rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("batched", [True, False])
def test_multi_round_replays_are_bitwise_one_round_replays(monkeypatch, batched):
    """GFEDNTM_ROUNDS_PER_GRAPH: k rounds captured back to back in one graph (runs ending at
    the epoch ends, power-of-two lengths, every graph captured before the first round) give
    the same state and losses, bit for bit, as one replay per round -- and the engine's
    k-step graph (FusedEngine.step_k) the same as k step() calls."""
    sc = generate_synthetic(vocab_size=600, n_topics=10, n_docs=200, n_nodes=4, frozen_topics=2,
                            nwords=(40, 80), seed=9)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(4)]
    out = {}
    for k in ("1", "16"):
        monkeypatch.setenv("GFEDNTM_ROUNDS_PER_GRAPH", k)
        fed = LocalFederation(corpora, _params(num_epochs=3), max_iters=37, device="cuda",
                              backend="fused", seed=3, graph=True, round_batched=batched)
        assert fed.rounds_per_replay() == int(k)
        fed.run()
        torch.cuda.synchronize()
        out[k] = ([c.shared.clone() for c in fed.clients],
                  [c.tm.engine.loss_hist[:37].clone() for c in fed.clients])
        if k == "16":
            assert 16 in fed._rgk and 1 in fed._rgk
    for a, b in zip(out["1"][0] + out["1"][1], out["16"][0] + out["16"][1]):
        assert torch.equal(a, b)


def test_engine_step_k_is_bitwise_k_steps():
    from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
    from gfedntm_amd.models import AVITM
    from tests.helpers import random_csr
    X = random_csr(400, 2000, 40, seed=2)
    res = []
    for mode in ("step", "step_k"):
        torch.manual_seed(0)
        tm = AVITM(backend="fused", input_size=2000, n_components=20, hidden_sizes=(50, 50),
                   batch_size=64, verbose=False, device="cuda")
        e = tm.engine
        e.bind_data(DeviceCSR(X, "cuda"), BatchPlan.build(400, 64, 24, seed=0))
        e.enable_graph(True)
        if mode == "step":
            for s in range(24):
                e.step(s)
        else:
            e.step_k(0, 8)
            e.step_k(8, 16)
        torch.cuda.synchronize()
        res.append((tm.flat.buffer.clone(), e.loss_hist[:24].clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_batched_bf16_large_vocab_keeps_ring_forward():
    """bf16 strip forward at a vocabulary past 4 tiles per workgroup (V > 64 x CUs): the
    batched plan shares one round of the CUs between the clients' grids (round 5 switched to
    an fp32-only variant here, which the launcher refused: CombinedTM K=100 V=99k bf16, 8
    clients).  Agrees with the per-client branch round."""
    from gfedntm_amd.ops.engine import STAGE_FWD_STRIP
    sc = generate_synthetic(vocab_size=60000, n_topics=20, n_docs=1200, n_nodes=2, frozen_topics=2,
                            nwords=(150, 250), seed=17)
    corpora = [ClientCorpus(synthetic=sc, node=i) for i in range(2)]
    kw = dict(device="cuda", backend="fused", seed=4)
    p = _params(batch_size=64, n_components=20, matmul_dtype="bf16")
    a = LocalFederation(corpora, p, max_iters=3, round_batched=True, **kw)
    b = LocalFederation(corpora, p, max_iters=3, round_batched=False, **kw)
    a.run()
    b.run()
    host = a._batched._host
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    assert host.n_tiles > cu and host.mm_bf16
    assert host.stage_flags & STAGE_FWD_STRIP
    assert 2 * host.dec_grid <= cu
    for x, y in zip(a.clients, b.clients):
        assert torch.isfinite(x.tm.flat.buffer).all()
        torch.testing.assert_close(x.tm.engine.loss_hist[:3], y.tm.engine.loss_hist[:3],
                                   rtol=1e-5, atol=1e-2)
