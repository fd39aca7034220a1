"""Kernel-boundary cost vs dirty bytes: graphs of 100 kernels that each write n
floats (plain or non-temporal stores), or alternate write/read."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from latency import build  # noqa: E402


def timed(g, reps=10):
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        g.replay()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) * 1e3 / reps


def main():
    lib = build()
    lib.launch_wr.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    lib.launch_rd.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p]
    buf = torch.zeros(8 << 20, device="cuda")
    out = torch.zeros(4096, device="cuda")
    for grid in (64, 256):
        for n in (0, 256, 16 << 10, 256 << 10, 2 << 20):
            for nt in (0, 1):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    s = torch.cuda.current_stream().cuda_stream
                    for _ in range(100):
                        lib.launch_wr(buf.data_ptr(), n, nt, grid, s)
                us = timed(g) / 100
                print(f"grid {grid:4d} write {n * 4 >> 10:6d} KiB nt={nt}: {us:6.2f} us/kernel")
        for n in (256, 16 << 10, 256 << 10):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                s = torch.cuda.current_stream().cuda_stream
                for _ in range(50):
                    lib.launch_wr(buf.data_ptr(), n, 0, grid, s)
                    lib.launch_rd(buf.data_ptr(), n, out.data_ptr(), grid, s)
            us = timed(g) / 100
            print(f"grid {grid:4d} write->read {n * 4 >> 10:6d} KiB: {us:6.2f} us/kernel")


if __name__ == "__main__":
    main()
