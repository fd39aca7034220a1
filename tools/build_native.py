"""Builds the in-tree native libraries for gfx950 (called by __graft_entry__.build()).

  gfedntm_amd/_lib/libgfedntm_kernels.so  -- HIP kernels + C++ step launcher (hipcc)
  gfedntm_amd/_lib/libgfedntm_runtime.so  -- host C++ runtime (tokenizer, CSR builder)

Incremental: an object is rebuilt when its source or a header is newer, or when
the compiler, target arch or flags differ from the ones recorded for it (a
``.cmd`` file next to every object), so changing ``PYTORCH_ROCM_ARCH`` or a flag
never links stale objects.
"""
import concurrent.futures as cf
import glob
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIB = os.path.join(ROOT, "gfedntm_amd", "_lib")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the kernel sources and flags live next to the hash that identifies them
# (gfedntm_amd/ops/srchash.py, loaded standalone: no torch import at build time)
_spec = importlib.util.spec_from_file_location(
    "_gfk_srchash", os.path.join(ROOT, "gfedntm_amd", "ops", "srchash.py"))
srchash = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(srchash)
KERNEL_SRCS, KFLAGS = srchash.KERNEL_SRCS, srchash.KFLAGS
RUNTIME_SRCS = ["runtime.cpp"]


def _stale(src, obj, deps, cmd):
    """Rebuild if the object is missing, older than its inputs, or was built with a
    different command line (compiler / arch / flags)."""
    if not os.path.exists(obj):
        return True
    try:
        with open(obj + ".cmd") as f:
            if f.read() != " ".join(cmd):
                return True
    except OSError:
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + deps)


def _compile(args):
    cmd, src, obj = args
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed for {src}:\n{r.stderr[-4000:]}")
    with open(obj + ".cmd", "w") as f:
        f.write(" ".join(cmd))
    return src


def _link_stale(so, objs, cmd):
    if not os.path.exists(so) or any(os.path.getmtime(o) > os.path.getmtime(so) for o in objs):
        return True
    try:
        with open(os.path.join(OBJ, os.path.basename(so) + ".cmd")) as f:
            return f.read() != " ".join(cmd)
    except OSError:
        return True


def _link(so, cmd, verbose):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    with open(os.path.join(OBJ, os.path.basename(so) + ".cmd"), "w") as f:
        f.write(" ".join(cmd))
    if verbose:
        print(f"[build] linked {so}", flush=True)


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
        cmd = [HIPCC, f"--offload-arch={ARCH}"] + KFLAGS + ["-c", src, "-o", obj]
        if _stale(src, obj, headers, cmd):
            jobs_list.append((cmd, s, obj))
    # the source identity (gfk_source_hash), checked by gfedntm_amd/ops/native.py at load
    digest = srchash.source_hash(ARCH)
    hsrc = os.path.join(OBJ, "srchash.cpp")
    text = ('extern "C" const char* gfk_source_hash() { return "%s"; }\n'
            'extern "C" const char* gfk_build_arch() { return "%s"; }\n' % (digest, ARCH))
    if not os.path.exists(hsrc) or open(hsrc).read() != text:
        with open(hsrc, "w") as f:
            f.write(text)
    hobj = os.path.join(OBJ, "srchash.cpp.o")
    kobjs.append(hobj)
    hcmd = ["g++", "-O2", "-fPIC", "-c", hsrc, "-o", hobj]
    if _stale(hsrc, hobj, [], hcmd):
        jobs_list.append((hcmd, "srchash.cpp", hobj))
    robjs = []
    for s in RUNTIME_SRCS:
        src = os.path.join(CSRC, s)
        if not os.path.exists(src):
            continue
        obj = os.path.join(OBJ, s + ".host.o")
        robjs.append(obj)
        cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-pthread", "-Wall", "-c", src, "-o", obj]
        if _stale(src, obj, headers, cmd):
            jobs_list.append((cmd, s, obj))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for s in ex.map(_compile, jobs_list):
            if verbose:
                print(f"[build] compiled {s}", flush=True)
    kso = os.path.join(LIB, "libgfedntm_kernels.so")
    kcmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", kso] + kobjs
    if kobjs and _link_stale(kso, kobjs, kcmd):
        _link(kso, kcmd, verbose)
    rso = os.path.join(LIB, "libgfedntm_runtime.so")
    rcmd = ["g++", "-shared", "-fPIC", "-pthread", "-o", rso] + robjs
    if robjs and _link_stale(rso, robjs, rcmd):
        _link(rso, rcmd, verbose)
    return kso


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
