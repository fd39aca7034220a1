"""Source identity of the kernel library.

``tools/build_native.py`` embeds :func:`source_hash` of the tree it compiles into
``libgfedntm_kernels.so`` (``gfk_source_hash()``); :func:`gfedntm_amd.ops.native.kernels`
recomputes it from the ``csrc/`` next to the package and refuses a library built from
other sources (a stale build, or one copied in from another tree), so the GPU tests, the
smoke run and the bench always run the committed kernels.  ``GFEDNTM_KERNELS_SO`` (A/B
timing of another build) bypasses the check on purpose.

No torch / numpy imports: the build script loads this file on its own.
"""
from __future__ import annotations

import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
# the kernel library's sources (compiled in this order) and compile flags.  fp32 division /
# sqrt and expf / logf use the hardware instructions (v_rcp / v_sqrt / v_exp / v_log,
# ~1 ulp) instead of the correctly rounded library sequences: the fused kernels'
# epilogues are VALU-bound, and every numerics test compares with a PyTorch fp32 oracle
# under tolerances, never bitwise.
KERNEL_SRCS = ["ctx.hip", "encoder.hip", "posterior.hip", "prodlda.hip", "neurallda.hip",
               "update.hip", "adam.hip", "comm.hip", "infer.hip", "step.cpp"]
KFLAGS = ["-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-result",
          "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-approx-transcendentals"]


def source_files(csrc: str = CSRC):
    hdr = sorted(f for f in os.listdir(csrc) if f.endswith(".h"))
    return [os.path.join(csrc, f) for f in KERNEL_SRCS + hdr
            if os.path.exists(os.path.join(csrc, f))]


def source_hash(arch: str = "gfx950", csrc: str = CSRC) -> str:
    """sha256 (first 16 hex digits) over the kernel sources, headers, flags and arch."""
    h = hashlib.sha256()
    h.update(("arch=" + arch + "\nflags=" + " ".join(KFLAGS) + "\n").encode())
    for p in source_files(csrc):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]
