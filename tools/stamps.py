"""Diagnostic: per-phase cycle shares of the single-workgroup posterior kernels.

Builds a -DGFK_STAMPS copy of the kernel library into build/stamps/, runs a few
eager steps and prints the s_memtime deltas between phase stamps (lane 0 of
workgroup 0).  Read the SHARES, not the absolute length (the stamps add fences).
"""
import os, subprocess, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
out = os.path.join(ROOT, "build", "stamps")
os.makedirs(out, exist_ok=True)
srcs = ["encoder.hip", "posterior.hip", "prodlda.hip", "neurallda.hip", "adam.hip", "step.cpp"]
objs = []
for s in srcs:
    o = os.path.join(out, s + ".o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                    "-munsafe-fp-atomics", "-DGFK_STAMPS", "-c", os.path.join(ROOT, "csrc", s), "-o", o],
                   check=True)
    objs.append(o)
so = os.path.join(out, "libgfedntm_kernels.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o", so] + objs, check=True)
from gfedntm_amd.ops import native
native.KERNELS_SO = so
import torch
from gfedntm_amd.models import AVITM
from gfedntm_amd.data.bow import DeviceCSR, BatchPlan
from tests.helpers import random_csr
tm = AVITM(input_size=4466, n_components=50, hidden_sizes=(50, 50), verbose=False, backend="fused",
           device="cuda")
X = random_csr(1000, 4466, 170, seed=0)
data = DeviceCSR(X, "cuda")
tm.engine.bind_data(data, BatchPlan.build(1000, 64, 50))
dbg = torch.zeros(64, dtype=torch.int64, device="cuda")
tm.engine._m.dbg = dbg.data_ptr()
tm.engine._a.dbg = dbg.data_ptr()
for s in range(20):
    tm.engine.step(s)
torch.cuda.synchronize()
d = dbg.cpu().numpy()
print("posterior_fwd cycles:", {n: int(d[i + 1] - d[i]) for i, n in enumerate(["stage", "colstats", "rows"])})
print("posterior_bwd_rows cycles:", int(d[9] - d[8]))
print("posterior_bwd_mlp cycles:", {n: int(d[11 + i] - d[10 + i]) for i, n in enumerate(["loads", "bn_bwd", "heads", "layers+dz0"])})
nf = ["stage", "mfma", "bn", "store+rowlse"]
print("prodlda_fwd cycles:", {nf[i]: int(d[17 + i] - d[16 + i]) for i in range(4)})
nbw = ["stage", "sparse", "dense+bn_bwd", "mfma+atomics"]
print("prodlda_bwd cycles:", {nbw[i]: int(d[25 + i] - d[24 + i]) for i in range(4)})
d16 = int(d[16])
print("prodlda_fwd staging detail (cycles from kernel start): glds issued", int(d[21]) - d16,
      "| scalars+nb", int(d[22]) - d16, "| beta staged", int(d[23]) - d16, "| barrier", int(d[17]) - d16)
print("adam cycles: prologue+segment", int(d[33] - d[32]), "| body", int(d[34] - d[33]))
