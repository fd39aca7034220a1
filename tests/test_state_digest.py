"""Cross-rank digest of the shared state (parallel/digest.py, csrc/comm.hip gfk_digest_*):
the data plane's self-check.  After every FedAvg round all replicas must be bit-identical
(reference: one average pushed to every client, src/federation/server.py:477-521); the
round loop compares digests periodically and at aligned rounds, and a divergence stops
every rank with CommError.

* the numpy digest equals a plain-integer re-statement of its definition and does not
  depend on how the work is chunked;
* gloo CPU ranks: a clean federation checks digests (W0, periodic, end) and finishes; a
  persistent one-word corruption on one rank (GFEDNTM_INJECT_CORRUPT) stops EVERY rank with
  CommError within one digest interval of the first digest round after it;
* GPU: the device kernels equal the numpy digest (odd sizes: the partial last float4);
  the one-GPU xGMI rehearsal detects the injected corruption on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch

from gfedntm_amd.parallel.digest import compare, digest_numpy


def _ref_digest(words):
    m = (1 << 64) - 1
    tot = 0
    for i, w in enumerate(np.asarray(words).reshape(-1).view(np.uint32).tolist()):
        z = ((i << 32) | w) & m
        z = (z + 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        z = z ^ (z >> 31)
        tot = (tot + z) & m
    return tot


def test_digest_definition_and_chunking():
    x = np.random.default_rng(0).standard_normal(1003).astype(np.float32)
    d = digest_numpy(x)
    assert d == _ref_digest(x)
    assert d == digest_numpy(x, chunk=7) == digest_numpy(x.view(np.uint32))
    y = x.copy()
    y.view(np.uint32)[501] ^= 1                  # one flipped bit
    assert digest_numpy(y) != d
    z = x.copy()
    z[[3, 4]] = z[[4, 3]]                        # two words swapped: position-sensitive
    assert digest_numpy(z) != d


def test_compare_reports_the_divergent_rank():
    assert compare([(7, [5, 5]), (7, [5, 5])], 0) is None
    why = compare([(7, [5]), (7, [6])], 0)
    assert "rank 1" in why and "round 7" in why
    assert "different rounds" in compare([(7, [5]), (8, [5])], 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpora(n):
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    sc = generate_synthetic(vocab_size=120, n_topics=5, n_docs=40, n_nodes=n, frozen_topics=2,
                            nwords=(15, 30), seed=1)
    return [ClientCorpus(synthetic=sc, node=i) for i in range(n)]


def _params():
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(num_epochs=10 ** 6, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    return p


def _worker(rank, world, port, env, rounds, q, gpu=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfedntm_amd.federation.runner import CommError, run_distributed
        kw = dict(backend="fused", rehearse_1gpu=True) if gpu else dict(backend="torch")
        if gpu:
            torch.cuda.set_device(0)
        try:
            out = run_distributed(_corpora(world)[rank], _params(), max_iters=rounds, seed=0, **kw)
        except CommError as e:
            q.put((rank, "comm_error", str(e)))
            return
        q.put((rank, "ok", out["digests"], out["allreduce"]))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "exception", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _run(world, env, rounds, gpu=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, env, rounds, q, gpu))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    return res


def test_gloo_clean_run_checks_digests():
    res = _run(2, {"GFEDNTM_DIGEST_EVERY": "4"}, rounds=18)
    for r in res:
        assert r[1] == "ok", r
        # W0, the periodic ones (rounds 3, 7, 11; resolved one interval later), the end
        assert r[2]["checked"] >= 4 and r[2]["every"] == 4, r[2]
        assert r[2]["last"][0] == 17
    assert res[0][2]["last"] == res[1][2]["last"]


def test_gloo_injected_corruption_stops_every_rank():
    res = _run(2, {"GFEDNTM_DIGEST_EVERY": "4", "GFEDNTM_INJECT_CORRUPT": "1:5"}, rounds=60)
    for r in res:
        assert r[1] == "comm_error", r
        assert "diverged" in r[2] and "rank 1" in r[2], r[2]
        # digested after round 7 (the first digest round from the injection on), caught
        # at the next interval: long before max_iters
        assert "after round 7" in r[2], r[2]


@pytest.mark.gpu
def test_device_digest_matches_numpy():
    from gfedntm_amd.parallel.digest import DigestProbe
    rng = np.random.default_rng(1)
    bufs = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)).cuda()
            for n in (1, 5, 4096, 1_000_003)]
    probe = DigestProbe(bufs)
    probe.take(3)
    rnd, ds = probe.result()
    assert rnd == 3
    assert ds == [digest_numpy(b.cpu().numpy()) for b in bufs]


@pytest.mark.gpu
def test_rehearsal_injected_corruption_stops_every_rank():
    """3 ranks on the one GPU over the in-step xGMI kernel: a clean run agrees on every
    digest; a persistent flip on rank 2 stops all three with CommError."""
    res = _run(3, {"GFEDNTM_DIGEST_EVERY": "4"}, rounds=18, gpu=True)
    for r in res:
        assert r[1] == "ok", r
        assert r[3].startswith("xgmi"), r[3]
        assert r[2]["checked"] >= 4
    res = _run(3, {"GFEDNTM_DIGEST_EVERY": "4", "GFEDNTM_INJECT_CORRUPT": "2:5"}, rounds=60,
               gpu=True)
    for r in res:
        assert r[1] == "comm_error", r
        assert "diverged" in r[2] and "after round 7" in r[2], r[2]
