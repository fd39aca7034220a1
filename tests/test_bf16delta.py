"""Opt-in reduced-byte FedAvg (``--fedavg_wire bf16delta``): every rank sends its pre-scaled
post-step state's departure from the last averaged state in bf16 and the departures are
summed in fp32 (parallel/aggregator.py; csrc/comm.hip gfk_xgmi_allreduce_bf16d over xGMI).
The default stays the reference's fp32 averaging (src/federation/server.py:477-487).

* the in-process golden (LocalAggregator) restates the kernel's arithmetic exactly;
* gloo CPU ranks: replicas bit-identical, equal to the in-process golden, and the final
  state stays within a small bound of the fp32 FedAvg over 200 rounds;
* GPU: the xGMI bf16-delta kernel validates against its torch restatement and a 3-rank
  one-GPU rehearsal reproduces the golden bit for bit, twice.
"""
import os
import socket

import numpy as np
import pytest
import torch

from gfedntm_amd.parallel.aggregator import LocalAggregator


def test_local_delta_restates_the_kernel_arithmetic():
    torch.manual_seed(0)
    n = [30, 50, 20]
    agg = LocalAggregator(n, wire="bf16delta")
    ref = torch.randn(1001)
    agg.set_reference(ref)
    w = agg.w
    states = [ref * wi + 1e-3 * torch.randn(1001) * wi for wi in w]   # pre-scaled post-step
    flats = [s.clone() for s in states]
    agg.average_(flats, prescaled=True)
    s = None
    for wi, f in zip(w, states):
        d = (f - ref * torch.tensor(float(np.float32(wi)))).to(torch.bfloat16).float()
        s = d if s is None else s + d
    exp = ref + s.to(torch.bfloat16).float()
    for f in flats:
        assert torch.equal(f, exp)
    assert torch.equal(agg.ref, exp)
    # the average it approximates: sum_i f_i (fp32), within bf16 rounding of the departures
    fp = sum(states)
    assert float((flats[0] - fp).abs().max()) < 1e-4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _corpora(n):
    from gfedntm_amd.data.synthetic import generate_synthetic
    from gfedntm_amd.federation.data import ClientCorpus
    sc = generate_synthetic(vocab_size=150, n_topics=5, n_docs=60, n_nodes=n, frozen_topics=2,
                            nwords=(15, 30), seed=5)
    return [ClientCorpus(synthetic=sc, node=i) for i in range(n)]


def _params():
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(num_epochs=10 ** 6, batch_size=16, hidden_sizes=(16, 16), n_components=5)
    return p


def _worker(rank, world, port, rounds, wire, q, gpu=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gfedntm_amd.federation.runner import run_distributed
        kw = dict(backend="fused", rehearse_1gpu=True) if gpu else dict(backend="torch")
        if gpu:
            torch.cuda.set_device(0)
        out = run_distributed(_corpora(world)[rank], _params(), max_iters=rounds, seed=1,
                              fedavg_wire=wire, **kw)
        q.put((rank, out["client"].shared.detach().cpu().numpy().copy(), out["allreduce"],
               (out["attach"] or {}).get("plane")))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc(), None, None))
    finally:
        dist.destroy_process_group()


def _run(world, rounds, wire, gpu=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, rounds, wire, q, gpu)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    for r in res:
        assert not isinstance(r[1], str), r[1]
    return res


def _golden(world, rounds, wire, device="cpu", backend="torch", perturb=0.0, full=False):
    from gfedntm_amd.federation.runner import LocalFederation
    fed = LocalFederation(_corpora(world), _params(), max_iters=rounds, device=device,
                          backend=backend, seed=1, fedavg_wire=wire,
                          **({"round_batched": False} if device != "cpu" else {}))
    w0 = fed.clients[0].shared.detach().cpu().numpy().copy()
    if perturb:
        with torch.no_grad():
            for c in fed.clients:
                c.shared.mul_(1.0 + perturb)
    fed.run()
    sh = fed.clients[0].shared.detach().cpu().numpy()
    if not full:
        return sh
    loss = float(np.mean([c.tm.engine.loss_hist[rounds - 50:rounds].mean().item()
                          for c in fed.clients]))
    return w0, sh, loss


def test_gloo_bf16delta_matches_golden_and_tracks_fp32():
    res = _run(2, 200, "bf16delta")
    np.testing.assert_array_equal(res[0][1], res[1][1])          # replicas bit-identical
    w0, gold, l_bf = _golden(2, 200, "bf16delta", full=True)
    np.testing.assert_array_equal(res[0][1], gold)
    assert np.isfinite(gold).all()
    # deviation from the fp32 FedAvg after 200 rounds, relative to how far training moved
    # the state: at the level of the training dynamics' own sensitivity (an fp32 run whose
    # W0 is scaled by 1 + 1e-7 departs by about as much), and the loss is unchanged
    _, fp32, l_fp = _golden(2, 200, "fp32", full=True)
    _, pert, _ = _golden(2, 200, "fp32", perturb=1e-7, full=True)
    moved = np.linalg.norm(fp32 - w0)
    dev, noise = np.linalg.norm(gold - fp32) / moved, np.linalg.norm(pert - fp32) / moved
    assert dev < 0.1 and dev < 3 * noise, (dev, noise)
    assert abs(l_bf - l_fp) / l_fp < 1e-3, (l_bf, l_fp)


def test_gloo_bf16delta_three_ranks_is_bitwise_golden():
    """3 ranks: the torch.distributed path sums the bf16 departures in fp32 in
    rank order and rounds once (all_gather of the bf16 words), as the xGMI kernel and the
    golden do -- a native bf16 all-reduce would round after every add, which 2 ranks cannot
    tell apart from this arithmetic but 3 can."""
    res = _run(3, 25, "bf16delta")
    for r in res[1:]:
        np.testing.assert_array_equal(res[0][1], r[1])
    np.testing.assert_array_equal(res[0][1], _golden(3, 25, "bf16delta"))


@pytest.mark.gpu
def test_xgmi_bf16delta_rehearsal_is_bitwise_and_reproducible():
    res1 = _run(3, 12, "bf16delta", gpu=True)
    res2 = _run(3, 12, "bf16delta", gpu=True)
    for r in res1:
        assert r[2].startswith("xgmi"), r[2]
        assert all(p.get("wire") == "bf16delta" for p in r[3].values()), r[3]
    for a, b in zip(res1, res2):
        np.testing.assert_array_equal(a[1], b[1])                # reproducible
    for r in res1[1:]:
        np.testing.assert_array_equal(r[1], res1[0][1])          # replicas bit-identical
    gold = _golden(3, 12, "bf16delta", device="cuda", backend="fused")
    np.testing.assert_array_equal(res1[0][1], gold)
