"""The production one-process-per-client runner (``run_distributed``) with the fused
engine and the in-step xGMI all-reduce, rehearsed on the one GPU of the test box
(every rank on cuda:0 over gloo; the IPC peer-memory protocol is the one used
across xGMI).

Reference round: src/federation/server.py:436-521 + client.py:135-183.

* unequal shards, so each client reaches ``num_epochs`` (and saves its results:
  full-shard inference + npz write, host work while the peers could be spinning
  in the next round's all-reduce) at a different round, plus one rank stalled on
  the host for 1.5 s before a round: the final shared state must be bit-identical
  to the in-process :class:`LocalFederation` golden (client-order sum), with the
  all-reduce's error word 0;
* a spin bound far below the injected stall: every rank must fail with
  ``CommError`` instead of producing a model.
"""
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = (100, 70, 45)           # docs per client: num_epochs=2 reached at rounds 7, 5, 3
ROUNDS = 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpora():
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    sc = generate_synthetic(vocab_size=600, n_topics=10, n_docs=max(SIZES), n_nodes=len(SIZES),
                            frozen_topics=2, nwords=(30, 60), seed=3)
    return [ClientCorpus(texts=sc.texts(i)[:n]) for i, n in enumerate(SIZES)]


def _params():
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(num_epochs=2, batch_size=32, hidden_sizes=(32, 32), n_components=10)
    return p


LARGE_SIZES = (260, 220, 180)


def _corpora_large():
    """K = 200 class at large V: a 150k-word generator vocabulary, ~70k words in the union
    (more strips than waves, the persistent pipelined backward, in-place xGMI parts)."""
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    sc = generate_synthetic(vocab_size=150000, n_topics=200, n_docs=max(LARGE_SIZES),
                            n_nodes=len(LARGE_SIZES), frozen_topics=5, nwords=(150, 250), seed=7)
    return [ClientCorpus(texts=sc.texts(i)[:n]) for i, n in enumerate(LARGE_SIZES)]


def _params_large():
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(num_epochs=1, batch_size=64, hidden_sizes=(50, 50), n_components=200)
    return p


def _worker(rank, world, port, tmp, stall, spin, q, poll=None, rounds=ROUNDS, epochs=2, large=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if spin is not None:
        os.environ["GFEDNTM_XGMI_SPIN"] = str(spin)
    if poll is not None:
        os.environ["GFEDNTM_COMM_POLL"] = str(poll)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        from gfedntm_amd.federation.runner import CommError, run_distributed

        def hook(it):
            if rank == 1 and it == 5:
                time.sleep(stall)

        try:
            params = dict(_params_large() if large else _params(), num_epochs=epochs)
            corpus = (_corpora_large() if large else _corpora())[rank]
            out = run_distributed(corpus, params, max_iters=rounds, backend="fused",
                                  seed=5, save_client=os.path.join(tmp, "client"),
                                  stamp="20240101", rehearse_1gpu=True, round_hook=hook,
                                  keep_round=True)
        except CommError as e:
            q.put((rank, "comm_error", str(e)))
            return
        c = out["client"]
        q.put((rank, out["allreduce"], c.shared.detach().cpu().numpy().copy(),
               c.tm.engine.fedavg_error(), c.results_saved, c.current_epoch))
        c.tm.engine.detach_fedavg()
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "exception", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _run(tmp, stall, spin=None, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = len(SIZES)
    ps = [ctx.Process(target=_worker, args=(r, world, port, str(tmp), stall, spin, q), kwargs=kw)
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    return res


def test_run_distributed_xgmi_matches_local_golden(tmp_path):
    res = _run(tmp_path, stall=1.5)
    for r in res:
        assert r[1] not in ("exception", "comm_error"), r
    # golden: the same federation in one process (client-order sum, fused engine)
    from gfedntm_amd.federation.runner import LocalFederation
    # (per-client kernels, as the one-client ranks run: the batched instances of the
    # kernels are compiled separately and need not round identically)
    fed = LocalFederation(_corpora(), _params(), max_iters=ROUNDS, device="cuda",
                          backend="fused", seed=5, round_batched=False)
    assert fed.round_graph
    fed.run()
    gold = fed.clients[0].shared.detach().cpu().numpy()
    for rank, used, shared, err, saved, epoch in res:
        assert used.startswith("xgmi"), used
        assert err == 0
        assert saved and epoch >= 2
        np.testing.assert_array_equal(shared, gold)
    for i in range(1, len(SIZES) + 1):
        assert os.path.exists(tmp_path / f"client{i}" / f"model_{i}_20240101.npz")


def test_run_distributed_large_v_matches_local_golden(tmp_path):
    """K = 200 at V ~ 70k over 3 ranks: the production large-state path (in-place xGMI
    parts, beta's share overlapped with the encoder backward, the pipelined backward,
    multi-strip forward) leaves the shared state bit-identical to LocalFederation."""
    rounds = 6
    res = _run(tmp_path, stall=0.0, rounds=rounds, epochs=1, large=True)
    for r in res:
        assert r[1] not in ("exception", "comm_error"), r
    from gfedntm_amd.federation.runner import LocalFederation
    fed = LocalFederation(_corpora_large(), _params_large(), max_iters=rounds, device="cuda",
                          backend="fused", seed=5, round_batched=False)
    fed.run()
    gold = fed.clients[0].shared.detach().cpu().numpy()
    e = fed.clients[0].tm.engine
    assert e._m.bwd_pre == 3 and e._m.n_tiles * 4 > 4096
    assert 4 * gold.size > (8 << 20)              # above the in-place threshold
    for rank, used, shared, err, saved, epoch in res:
        assert used.startswith("xgmi"), used
        assert err == 0
        np.testing.assert_array_equal(shared, gold)


def test_run_distributed_fails_loudly_on_a_timed_out_wait(tmp_path):
    res = _run(tmp_path, stall=2.0, spin=2000)
    for r in res:
        assert r[1] == "comm_error", r[:2]


def test_timed_out_wait_is_caught_between_aligned_rounds(tmp_path):
    """No host-heavy round before the end (num_epochs never reached, no checkpoints, no
    metrics): the periodic error-word poll still stops every rank within a few rounds of
    the timeout (the host may run ahead of the device by the enqueued rounds) instead of
    training on to max_iters on invalid shared state."""
    res = _run(tmp_path, stall=2.0, spin=2000, poll=4, rounds=400, epochs=10 ** 6)
    for r in res:
        assert r[1] == "comm_error", r[:2]
        before = int(r[2].split("before round ")[1].split()[0])
        assert before < 400, r[2]         # stopped before max_iters


N_MULTI = 8                      # clients, over 2 ranks: 4 per rank


CTM_C = 48                       # contextual size of the CombinedTM rehearsals


def _multi_corpora(n=N_MULTI, ctm=False):
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    sc = generate_synthetic(vocab_size=500, n_topics=10, n_docs=60, n_nodes=n,
                            frozen_topics=2, nwords=(30, 60), seed=9)
    if not ctm:
        return [ClientCorpus(synthetic=sc, node=i) for i in range(n)]
    proj = np.random.default_rng(3).standard_normal((10, CTM_C)).astype(np.float32)
    out = []
    for i in range(n):      # synthetic embeddings: a projection of the topic mixture + noise
        dt = np.asarray(sc.doc_topics[i], dtype=np.float32)
        emb = dt @ proj + 0.1 * np.random.default_rng(11 + i).standard_normal(
            (dt.shape[0], CTM_C)).astype(np.float32)
        out.append(ClientCorpus(synthetic=sc, node=i, embeddings=emb))
    return out


def _ctm_params():
    return dict(_params(), contextual_size=CTM_C)


def _multi_worker(rank, world, port, tmp, q, n_clients=N_MULTI, env=None, stall=None,
                  rounds=ROUNDS, epochs=2, ctm=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        from gfedntm_amd.federation.hierarchical import assign_clients, run_distributed_multi
        from gfedntm_amd.federation.runner import CommError
        ids = assign_clients(n_clients, world)[rank]
        corpora = _multi_corpora(n_clients, ctm=ctm)

        def hook(it):
            if stall and rank == 1 and it == 5:
                time.sleep(stall)

        try:
            out = run_distributed_multi([corpora[i - 1] for i in ids], ids,
                                        dict(_ctm_params() if ctm else _params(), num_epochs=epochs),
                                        model_type="ctm" if ctm else "avitm", max_iters=rounds,
                                        backend="fused", seed=5, rehearse_1gpu=True,
                                        save_client=os.path.join(tmp, "client"), stamp="20240101",
                                        round_hook=hook)
        except CommError as e:
            q.put((rank, "comm_error", str(e), None, None))
            return
        rr = out["round"]
        q.put((rank, out["allreduce"], [c.shared.detach().cpu().numpy().copy() for c in out["clients"]],
               [c.id for c in out["clients"]], (out["attach"] or {}).get("inplace")))
        rr.close()
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "exception", traceback.format_exc(), None, None))
    finally:
        dist.destroy_process_group()


def _run_multi(tmp, **kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_multi_worker, args=(r, 2, port, str(tmp), q), kwargs=kw)
          for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    return res


@pytest.mark.parametrize("n_clients,inplace_mb", [(N_MULTI, None), (40, "0")])
def test_more_clients_than_ranks_xgmi_matches_grouped_golden(tmp_path, n_clients, inplace_mb):
    """8 clients on 2 ranks (4 per rank, one GPU): every rank's round graph holds its 4
    clients' steps (one launch per phase), the in-rank fold, the xGMI all-reduce of the
    partial sums and the broadcast -- beta's share forked onto a side stream after the
    decoder backward; the final state of all clients equals the in-process federation
    with the same grouping bit for bit, and every client saves its results.  40 clients
    (20 per rank, past the old 16-buffer fold) with both parts all-reduced in place
    (GFEDNTM_XGMI_INPLACE_MB=0: two in-place parts of one allocation, one shared mapping)."""
    env = {} if inplace_mb is None else {"GFEDNTM_XGMI_INPLACE_MB": inplace_mb}
    res = _run_multi(tmp_path, n_clients=n_clients, env=env)
    for r in res:
        assert r[1] not in ("exception", "comm_error"), r[2]
        assert r[1] == "xgmi+overlap", r[1]
        if inplace_mb == "0":
            assert r[4] == {"rest": True, "beta": True}, r[4]
    assert [i for r in res for i in r[3]] == list(range(1, n_clients + 1))
    from gfedntm_amd.federation.runner import LocalFederation
    half = n_clients // 2
    fed = LocalFederation(_multi_corpora(n_clients), _params(), max_iters=ROUNDS, device="cuda",
                          backend="fused", seed=5, groups=[half, half])
    assert fed.round_graph
    fed.run()
    gold = fed.clients[0].shared.detach().cpu().numpy()
    for r in res:
        for sh in r[2]:
            np.testing.assert_array_equal(sh, gold)
    for i in range(1, n_clients + 1):
        assert os.path.exists(tmp_path / f"client{i}" / f"model_{i}_20240101.npz")


@pytest.mark.parametrize("n_clients", [2, 6])
def test_combined_tm_adapt_bert_overlap_matches_golden(tmp_path, n_clients):
    """CombinedTM over 2 ranks (one client each, or 3 per rank): the shared state's three
    parts -- beta forked after the decoder backward, adapt_bert after ctx_bwd (both on the
    side stream, overlapping the encoder backward / win_update), the rest after the step --
    leave every client's state bit-identical to the in-process federation."""
    res = _run_multi(tmp_path, n_clients=n_clients, ctm=True)
    for r in res:
        assert r[1] not in ("exception", "comm_error"), r[2]
        assert r[1] == "xgmi+overlap", r[1]
    from gfedntm_amd.federation.runner import LocalFederation
    half = n_clients // 2
    fed = LocalFederation(_multi_corpora(n_clients, ctm=True), _ctm_params(), model_type="ctm",
                          max_iters=ROUNDS, device="cuda", backend="fused", seed=5,
                          **({"groups": [half, half]} if half > 1 else {"round_batched": False}))
    fed.run()
    e = fed.clients[0].tm.engine
    assert set(e.fedavg_parts()) == {"rest", "wa", "beta"}
    gold = fed.clients[0].shared.detach().cpu().numpy()
    for r in res:
        for sh in r[2]:
            np.testing.assert_array_equal(sh, gold)


def test_more_clients_than_ranks_timed_out_wait_is_polled(tmp_path):
    """The multi-client runner inherits the periodic error-word poll: a host stall longer
    than the xGMI spin bound, with no host-heavy round before the end, stops every rank
    with CommError within a few rounds instead of training on to max_iters."""
    res = _run_multi(tmp_path, env={"GFEDNTM_XGMI_SPIN": "2000", "GFEDNTM_COMM_POLL": "4"},
                     stall=2.0, rounds=400, epochs=10 ** 6)
    for r in res:
        assert r[1] == "comm_error", r[:3]
        before = int(r[2].split("before round ")[1].split()[0])
        assert before < 400, r[2]


@pytest.mark.parametrize("clients,inject", [("2", "GFEDNTM_INJECT_STALL=1:8:2.0"),
                                             ("8", "GFEDNTM_INJECT_STALL=1:8:2.0"),
                                             ("2", "GFEDNTM_INJECT_CORRUPT=1:3")])
def test_bench_falls_back_to_rccl_when_xgmi_times_out(tmp_path, clients, inject):
    """bench.py (2 ranks on the one GPU; one client per rank, or the default 8 clients as 4
    per rank): an injected host stall longer than the xGMI spin bound -- or a replica that
    diverges (GFEDNTM_INJECT_CORRUPT: the digest check) -- makes every rank raise
    CommError in the timed region; with the data plane on auto-selection the bench
    re-measures the same federation over RCCL and records why, instead of printing no
    number."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    k, v = inject.split("=")
    env = dict(os.environ, GFEDNTM_REHEARSE_1GPU="1", GFEDNTM_XGMI_SPIN="2000",
               GFEDNTM_DIGEST_EVERY="4", **{k: v})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "20",
                        "--warmup", "5", "--no-npmi", "--clients", clients], cwd=root, env=env,
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert "xGMI all-reduce failed" in rec["allreduce_fallback"]
    assert rec["value"] > 0 and rec["ranks"] == 2
    # the injected stall belongs to the failed attempt only: the RCCL re-measure's rounds
    # are plain (a 2 s stall over 20 rounds would be >= 100 ms per round)
    assert rec["ms_per_step"] < 50, rec["ms_per_step"]
