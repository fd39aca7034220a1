"""Achievable bandwidth of the beta Adam read-modify-write (tools/micro/adam_bw.hip)."""
import ctypes as C
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "..", "..", "build", "micro", "adam_bw.so")


def main():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared",
                           "-o", SO, os.path.join(HERE, "adam_bw.hip")])
    lib = C.CDLL(SO)
    lib.launch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                           C.c_void_p]
    K = 200
    V = int(os.environ.get("ADAM_BW_V", "112000"))     # 112027: rows not 16-byte aligned
    p, m, v = (torch.rand(K * V, device="cuda") for _ in range(3))
    stream = torch.cuda.current_stream().cuda_stream
    nbytes = 6 * K * V * 4
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    pats = os.environ.get("ADAM_BW_PATTERNS", "0,1,2").split(",")
    names = {0: "mfma", 1: "rows4", 2: "flat4", 3: "rows1"}
    for which in (int(x) for x in pats):
        name = names[which]
        for grid in ((2 * cu, 4 * cu, 8 * cu, 16 * cu) if which != 2 else (4 * cu, 16 * cu)):
            for _ in range(3):
                lib.launch(which, p.data_ptr(), m.data_ptr(), v.data_ptr(), K, V, grid, stream)
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(20):
                lib.launch(which, p.data_ptr(), m.data_ptr(), v.data_ptr(), K, V, grid, stream)
            t1.record()
            torch.cuda.synchronize()
            us = t0.elapsed_time(t1) * 1e3 / 20
            print(json.dumps({"pattern": name, "V": V, "grid": grid, "us": round(us, 2),
                              "TB_per_s": round(nbytes / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
