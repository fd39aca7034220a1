"""Custom xGMI all-reduce (csrc/comm.hip): exactness against the rank-ordered fp32
sum, sizes that are not multiples of 4, hipGraph capture + replay, and the
aggregator's validated selection.  Several ranks share the one GPU of the test
box (IPC mappings of same-device memory use the same protocol as xGMI peers)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gfedntm_amd.utils.misc import graph_capture

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        from gfedntm_amd.parallel.aggregator import CollectiveAggregator
        from gfedntm_amd.parallel.xgmi import XgmiAllReduce
        xg = XgmiAllReduce(n, "cuda:0")
        cu = torch.cuda.get_device_properties(0).multi_processor_count
        chunk = (-(-n // world) + 3) // 4 * 4          # floats per rank, multiple of 4
        assert xg.nblk == max(1, min(cu // world, chunk // 1024)), xg.nblk
        ok = xg.validate(rounds=3)
        # graph capture: the captured kernel advances its epoch on every replay
        t = torch.zeros(n, device="cuda")
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            xg.allreduce_(t)
        ar = torch.arange(n, device="cuda", dtype=torch.float32)
        good = []
        for r in range(5):
            t.copy_(torch.remainder(ar * (rank + 1 + r), 13.0))
            g.replay()
            torch.cuda.synchronize()
            exp = sum(torch.remainder(ar * (j + 1 + r), 13.0) for j in range(world))
            good.append(bool(torch.equal(t, exp)))
        err = xg.error()
        xg.close()
        # the aggregator picks xgmi after validating it
        buf = torch.full((n,), float(rank + 1), device="cuda")
        agg = CollectiveAggregator(method="auto")
        method = agg.prepare(buf)
        agg.allreduce_(buf)
        torch.cuda.synchronize()
        agg_ok = bool(torch.all(buf == world * (world + 1) / 2).item())
        q.put((rank, ok, all(good), err, method, agg_ok))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


# 20_000_003 floats = the 80 MB beta share of ProdLDA K=200, V=100K: the size-aware
# grid (one workgroup per >= 4 KB slice, CUs split among the ranks sharing the GPU)
@pytest.mark.parametrize("world,n", [(2, 1_000_003), (3, 446_650), (2, 10), (2, 20_000_003)])
def test_xgmi_allreduce_exact(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(60)
    for r in res:
        assert len(r) == 6, r
        _, ok, graph_ok, err, method, agg_ok = r
        assert ok and graph_ok and err == 0 and method == "xgmi" and agg_ok, r


def _fused_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        import numpy as np
        from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
        from gfedntm_amd.models import AVITM
        from tests.helpers import random_csr
        out = {}
        for method in ("auto", "rccl"):
            torch.manual_seed(0)                     # same W0 and Philox seed on both ranks
            tm = AVITM(input_size=900, n_components=20, hidden_sizes=(32, 32), batch_size=64,
                       verbose=False, device="cuda", backend="fused")
            X = random_csr(300 + 50 * rank, 900, 40, seed=10 + rank)
            data = DeviceCSR(X, "cuda")
            e = tm.engine
            e.bind_data(data, BatchPlan.build(data.n_docs, 64, 30, seed=rank))
            n = [300.0, 350.0]
            e.set_fedavg_scale(n[rank] / sum(n))
            used = e.attach_fedavg(method=method)
            e.enable_graph(True)
            for s in range(30):
                e.step(s)
            torch.cuda.synchronize()
            out[method] = (used, tm.flat.shared.detach().cpu().numpy().copy(), e.fedavg_error())
        same_rank = np.array_equal(out["auto"][1], out["rccl"][1])
        q.put((rank, out["auto"][0], out["rccl"][0], same_rank, out["auto"][2],
               out["auto"][1][:1000].tolist()))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        dist.destroy_process_group()


def test_fused_fedavg_overlap_matches_eager():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fused_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(2)], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    for r in res:
        assert len(r) == 6, r
        _, used_auto, used_rccl, same, err, _ = r
        assert used_auto == "xgmi+overlap" and used_rccl == "rccl", r[:5]
        assert same and err == 0, r[:5]
    assert res[0][5] == res[1][5]                    # ranks hold the same averaged state


def _inplace_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    try:
        from gfedntm_amd.parallel.xgmi import XgmiAllReduce
        # a sub-block of a larger allocation, as the shared state is a slice of the flat buffer
        big = torch.zeros(n + 4096, device="cuda")
        buf = big[1024: 1024 + n]
        state = torch.remainder(torch.arange(n, device="cuda", dtype=torch.float32) * (rank + 3), 7.0)
        buf.copy_(state)
        xg = XgmiAllReduce(n, "cuda:0", data=buf)
        ok = xg.validate(rounds=2)
        restored = bool(torch.equal(buf, state))            # validation left the state alone
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            xg.allreduce_(buf)
        ar = torch.arange(n, device="cuda", dtype=torch.float32)
        good = []
        for r in range(4):
            buf.copy_(torch.remainder(ar * (rank + 1 + r), 13.0))
            g.replay()
            torch.cuda.synchronize()
            exp = sum(torch.remainder(ar * (j + 1 + r), 13.0) for j in range(world))
            good.append(bool(torch.equal(buf, exp)))
        err = xg.error()
        try:
            xg.allreduce_(torch.zeros(n, device="cuda"))
            wrong_buf_refused = False
        except ValueError:
            wrong_buf_refused = True
        xg.close()
        q.put((rank, ok, restored, all(good), err, wrong_buf_refused))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1_000_003), (3, 2_500_001)])
def test_xgmi_allreduce_inplace_exact(world, n):
    """In-place mode (large states): the data buffer itself is IPC-mapped (sub-block of a
    caching-allocator block: handle of the base + offset), no stage copy, a phase-3
    hand-off before returning; exact rank-ordered sums, graph replays, the validation
    restores the state, other buffers are refused."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_inplace_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(60)
    for r in res:
        assert len(r) == 6, r
        _, ok, restored, graph_ok, err, refused = r
        assert ok and restored and graph_ok and err == 0 and refused, r


def test_ipc_handles_identify_the_allocation():
    """The peer-mapping cache (parallel/xgmi.py _IPC_OPEN) is keyed by the exporter's pid
    and IPC handle bytes: two slices of ONE allocation must export the same handle (one
    shared mapping, refcounted), a different allocation a different one (never a stale
    mapping of freed memory at a reused address)."""
    import ctypes as C
    from gfedntm_amd.ops import native
    from gfedntm_amd.parallel.xgmi import _declare
    lib = native.kernels()
    _declare(lib)
    hs = lib.gfk_ipc_handle_size()

    def export(t):
        h, off = C.create_string_buffer(hs), C.c_int64(0)
        assert lib.gfk_ipc_get_range(C.c_void_p(t.data_ptr()), h, C.byref(off)) == 0
        return h.raw, off.value

    # (fresh segments: after earlier tests the caching allocator may carve both tensors
    # out of one cached allocation, which then rightly exports one handle)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    a = torch.zeros(1 << 22, device="cuda")
    b = torch.zeros(1 << 22, device="cuda")
    h0, o0 = export(a[:1024])
    h1, o1 = export(a[1 << 20:])
    assert h0 == h1 and o1 - o0 == 4 << 20
    hb, ob = export(b)
    if hb == h0:       # one allocation after all: the offsets must place b inside it
        assert ob - o0 == b.data_ptr() - a.data_ptr()
        c = torch.empty(3 << 24, dtype=torch.uint8, device="cuda")   # 48 MiB: its own segment
        hc, _ = export(c)
        assert hc != h0
    else:
        assert hb != h0
