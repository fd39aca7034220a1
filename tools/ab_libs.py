"""Diagnostic: build the kernel library of a git revision (or of the working tree) into
abtmp/<name>/libgfedntm_kernels.so, for A/B timing of kernel variants in ONE GPU call:

    python tools/ab_libs.py A HEAD        # the committed sources
    python tools/ab_libs.py B             # the working tree
    GFEDNTM_KERNELS_SO=abtmp/A/libgfedntm_kernels.so python bench.py ...

(the Python package and the runtime library stay the working tree's: only variants
with the same kernel ABI can be compared this way).
"""
import concurrent.futures as cf
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.build_native import ARCH, HIPCC, KERNEL_SRCS, KFLAGS  # noqa: E402


def main(argv):
    name = argv[0]
    rev = argv[1] if len(argv) > 1 else None
    out = os.path.join(ROOT, "abtmp", name)   # (delete after the A/B call: not product)
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        src_dir = os.path.join(ROOT, "csrc")
        if rev:
            src_dir = os.path.join(tmp, "csrc")
            os.makedirs(src_dir)
            files = subprocess.run(["git", "ls-tree", "--name-only", rev, "csrc/"], cwd=ROOT,
                                   capture_output=True, text=True, check=True).stdout.split()
            for f in files:
                data = subprocess.run(["git", "show", f"{rev}:{f}"], cwd=ROOT, capture_output=True,
                                      check=True).stdout
                with open(os.path.join(tmp, f), "wb") as fh:
                    fh.write(data)
        jobs = []
        objs = []
        for s in KERNEL_SRCS:
            src = os.path.join(src_dir, s)
            if not os.path.exists(src):
                continue
            obj = os.path.join(tmp, s + ".o")
            objs.append(obj)
            flags = KFLAGS if os.environ.get("AB_FLAGS", "new") == "new" else \
                ["-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics", "-Wno-unused-result"]
            # AB_DEFS: extra -D definitions (diagnostic variants, e.g. "GFK_DIAG_BWD=1")
            defs = ["-D" + d for d in os.environ.get("AB_DEFS", "").split()]
            jobs.append([HIPCC, f"--offload-arch={ARCH}"] + flags + defs + ["-c", src, "-o", obj])
        with cf.ThreadPoolExecutor(8) as ex:
            for r in ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs):
                if r.returncode:
                    raise SystemExit(r.stderr[-3000:])
        so = os.path.join(out, "libgfedntm_kernels.so")
        subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", so] + objs,
                       check=True)
    print(so)


if __name__ == "__main__":
    main(sys.argv[1:])
