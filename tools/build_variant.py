"""Builds a variant of the kernel library with extra compiler flags, for A/B timing on one
box: ``python tools/build_variant.py abtmp/libnoxcd.so -DGFK_NO_XCD_MAP``, then run with
``GFEDNTM_KERNELS_SO=abtmp/libnoxcd.so`` (gfedntm_amd/ops/native.py loads it without the
source-hash check and logs that it did).  Objects go to build/variant/<name>/; the
committed library (tools/build_native.py) is untouched."""
import concurrent.futures as cf
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import build_native as bn  # noqa: E402


def main(out, flags):
    name = os.path.splitext(os.path.basename(out))[0]
    odir = os.path.join(bn.ROOT, "build", "variant", name)
    os.makedirs(odir, exist_ok=True)
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    jobs, objs = [], []
    for s in bn.KERNEL_SRCS:
        obj = os.path.join(odir, s + ".o")
        objs.append(obj)
        jobs.append([bn.HIPCC, f"--offload-arch={bn.ARCH}"] + bn.KFLAGS + flags
                    + ["-c", os.path.join(bn.CSRC, s), "-o", obj])
    hsrc = os.path.join(odir, "srchash.cpp")
    with open(hsrc, "w") as f:
        f.write('extern "C" const char* gfk_source_hash() { return "variant:%s"; }\n'
                'extern "C" const char* gfk_build_arch() { return "%s"; }\n' % (name, bn.ARCH))
    objs.append(hsrc + ".o")
    jobs.append(["g++", "-O2", "-fPIC", "-c", hsrc, "-o", hsrc + ".o"])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(f"{' '.join(cmd[-3:])}:\n{r.stderr[-3000:]}")

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        list(ex.map(run, jobs))
    run([bn.HIPCC, f"--offload-arch={bn.ARCH}", "-shared", "-fPIC", "-o", out] + objs)
    print(f"[variant] {out} ({' '.join(flags)})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
