"""Diagnostic: per-phase cycle counts inside the fused-step kernels (s_memtime stamps).

Builds a -DGFK_STAMPS copy of the kernel library into build/stamps/, runs a few
eager steps and prints the s_memtime deltas between phase stamps (lane 0 of
workgroup 0).  Read the SHARES, not the absolute length (the stamps add fences).
"""
import os, subprocess, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
out = os.path.join(ROOT, "build", "stamps")
os.makedirs(out, exist_ok=True)
from tools.build_native import KERNEL_SRCS
srcs = [x for x in KERNEL_SRCS if os.path.exists(os.path.join(ROOT, "csrc", x))]
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
nf = ["stage", "mfma", "bn", "store+rowlse"]
print("prodlda_fwd cycles:", {nf[i]: int(d[17 + i] - d[16 + i]) for i in range(4)})
nbw = ["stage", "sparse", "dense+bn_bwd", "mfma+update"]
print("prodlda_bwd cycles:", {nbw[i]: int(d[25 + i] - d[24 + i]) for i in range(4)})
print("post_fwd cycles: stage", int(d[1] - d[0]), "| colstats", int(d[2] - d[1]), "| row", int(d[3] - d[2]))
print("row_bwd cycles:", int(d[9] - d[8]))
print("post_bwd cycles: stage", int(d[11] - d[10]), "| colsums", int(d[12] - d[11]), "| rest", int(d[13] - d[12]))
print("post_bwd rest: wg0 extras", int(d[14] - d[12]), "| bn_bwd", int(d[15] - d[14]),
      "| heads", int(d[29] - d[15]), "| hidden", int(d[13] - d[29]))
print("enc_in cycles: row+weights issue", int(d[5] - d[4]), "| gather+draws", int(d[6] - d[5]),
      "| input+hidden", int(d[7] - d[6]))
print("win_update (W_in tile 0) cycles: staging", int(d[41] - d[40]), "| mfma+update", int(d[42] - d[41]))
