"""Builds the in-tree native libraries for gfx950 (called by __graft_entry__.build()).

  gfedntm_amd/_lib/libgfedntm_kernels.so  -- HIP kernels + C++ step launcher (hipcc)
  gfedntm_amd/_lib/libgfedntm_runtime.so  -- host C++ runtime (tokenizer, CSR builder)

Incremental: an object is rebuilt only when its source or a header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(ROOT, "gfedntm_amd", "_lib")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
KERNEL_SRCS = ["ctx.hip", "encoder.hip", "posterior.hip", "prodlda.hip", "neurallda.hip", "update.hip",
               "adam.hip", "comm.hip", "infer.hip", "step.cpp"]
RUNTIME_SRCS = ["runtime.cpp"]


def _newer(src, obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def _compile(args):
    cmd, src = args
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed for {src}:\n{r.stderr[-4000:]}")
    return src


def build(verbose=True, jobs=8):
    os.makedirs(LIB, exist_ok=True)
    os.makedirs(OBJ, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    jobs_list, kobjs = [], []
    for s in KERNEL_SRCS:
        src = os.path.join(CSRC, s)
        if not os.path.exists(src):
            continue
        obj = os.path.join(OBJ, s + ".o")
        kobjs.append(obj)
        if _newer(src, obj, headers):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17",
                   "-munsafe-fp-atomics", "-Wno-unused-result", "-c", src, "-o", obj]
            jobs_list.append((cmd, s))
    robjs = []
    for s in RUNTIME_SRCS:
        src = os.path.join(CSRC, s)
        if not os.path.exists(src):
            continue
        obj = os.path.join(OBJ, s + ".host.o")
        robjs.append(obj)
        if _newer(src, obj, headers):
            jobs_list.append((["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-Wall", "-c", src,
                              "-o", obj], s))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in ex.map(_compile, jobs_list):
            if verbose:
                print(f"[build] compiled {s}", flush=True)
    kso = os.path.join(LIB, "libgfedntm_kernels.so")
    if kobjs and (not os.path.exists(kso) or any(os.path.getmtime(o) > os.path.getmtime(kso)
                                                 for o in kobjs)):
        r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", kso] + kobjs,
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-4000:])
        if verbose:
            print(f"[build] linked {kso}", flush=True)
    rso = os.path.join(LIB, "libgfedntm_runtime.so")
    if robjs and (not os.path.exists(rso) or any(os.path.getmtime(o) > os.path.getmtime(rso)
                                                 for o in robjs)):
        r = subprocess.run(["g++", "-shared", "-fPIC", "-pthread", "-o", rso] + robjs, capture_output=True,
                           text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-4000:])
        if verbose:
            print(f"[build] linked {rso}", flush=True)
    return kso


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
