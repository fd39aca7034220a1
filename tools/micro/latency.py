"""Runs tools/micro/latency.hip on the GPU: dependent-load latency by footprint,
scalar-load latency, latency after another kernel wrote the data, and the cost
of an empty kernel inside a hipGraph.  usage: python tools/micro/latency.py"""
import ctypes as C
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "..", "..", "build", "micro_latency.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(HERE, "latency.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                               "-shared", "-o", SO, src])
    lib = C.CDLL(SO)
    for f in ("launch_chase", "launch_sload"):
        getattr(lib, f).argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.launch_writer.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    lib.launch_empty.argtypes = [C.c_int, C.c_void_p]
    return lib


def ring(n_bytes, stride_bytes, dev):
    n = n_bytes // 4
    st = stride_bytes // 4
    idx = torch.arange(n, dtype=torch.int64)
    nxt = ((idx // st + 1) * st) % n
    return nxt.to(torch.int32).to(dev)


def main():
    if "--build-only" in sys.argv:
        build()
        return
    lib = build()
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = torch.zeros(3, dtype=torch.int64, device=dev)
    n = 2000
    print("footprint      stride  cycles/load  ns/load(realtime)")
    for fp, st in [(4 << 10, 64), (256 << 10, 128), (4 << 20, 4096), (64 << 20, 65536 + 64),
                   (512 << 20, (2 << 20) + 64)]:
        r = ring(fp, st, dev)
        for rep in range(2):
            lib.launch_chase(r.data_ptr(), n, out.data_ptr(), s)
        torch.cuda.synchronize()
        cyc, rt = out[0].item() / n, out[1].item() / n * 10.0
        print(f"{fp >> 10:>8} KiB {st:>8} {cyc:>10.0f} {rt:>12.0f}")
    # data just written by another kernel (each hop lands on a line another XCD wrote)
    r = ring(4 << 20, 4096, dev)
    lib.launch_writer(r.data_ptr(), r.numel(), 1024, s)
    lib.launch_chase(r.data_ptr(), 200, out.data_ptr(), s)
    torch.cuda.synchronize()
    print(f"after writer kernel (4 MiB, 4 KiB stride): {out[0].item() / 200:.0f} cycles/load, "
          f"{out[1].item() / 200 * 10:.0f} ns/load")
    r = ring(4 << 10, 64, dev)
    lib.launch_sload(r.data_ptr(), n, out.data_ptr(), s)
    lib.launch_sload(r.data_ptr(), n, out.data_ptr(), s)
    torch.cuda.synchronize()
    print(f"scalar-ish chase (readfirstlane), 4 KiB: {out[0].item() / n:.0f} cycles/load, "
          f"{out[1].item() / n * 10:.0f} ns/load")
    # empty kernels in a graph
    for grid in (1, 64, 256, 1024):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(100):
                lib.launch_empty(grid, torch.cuda.current_stream().cuda_stream)
        g.replay()
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(10):
            g.replay()
        t1.record()
        torch.cuda.synchronize()
        print(f"empty kernel in graph, grid {grid}: {t0.elapsed_time(t1) * 1e3 / 1000:.2f} us/kernel")
    print("clock (MHz) estimate:", torch.cuda.get_device_properties(0).name)


if __name__ == "__main__":
    main()
