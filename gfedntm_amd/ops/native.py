"""Loader for the in-tree native libraries (built by __graft_entry__.build()).

* ``libgfedntm_kernels.so`` -- CDNA4 (gfx950) HIP kernels + the C++ step
  launcher; called through ctypes with raw device pointers and the current
  HIP stream, so every launch of a training step is made from C++.
* ``libgfedntm_runtime.so`` -- host-side C++ runtime: CountVectorizer-
  compatible tokenizer / CSR builder, batch-plan builder.

On a GPU box the kernels library is REQUIRED: :func:`kernels` raises if it is
missing instead of silently falling back to PyTorch, and if it was built from other
sources than the ``csrc/`` of this tree (the source hash embedded by the build,
``ops/srchash.py``) -- unless ``GFEDNTM_KERNELS_SO`` names another build on purpose.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Sequence

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "_lib")
# GFEDNTM_KERNELS_SO: another build of the kernel library (A/B timing of kernel variants,
# tools/ab_libs.py); the in-tree library otherwise
KERNELS_SO_OVERRIDE = os.environ.get("GFEDNTM_KERNELS_SO") or None
KERNELS_SO = KERNELS_SO_OVERRIDE or os.path.join(LIB_DIR, "libgfedntm_kernels.so")
RUNTIME_SO = os.path.join(LIB_DIR, "libgfedntm_runtime.so")

_kernels: Optional[ctypes.CDLL] = None
_runtime: Optional[ctypes.CDLL] = None
_runtime_tried = False


def kernels_available() -> bool:
    return os.path.exists(KERNELS_SO)


def kernels() -> ctypes.CDLL:
    global _kernels
    if _kernels is None:
        if not kernels_available():
            raise RuntimeError(
                f"{KERNELS_SO} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(KERNELS_SO, mode=ctypes.RTLD_GLOBAL)
        _check_source(lib)
        from . import kernel_abi
        kernel_abi.declare(lib)
        _kernels = lib
    return _kernels


def _embedded_str(lib, name: str) -> Optional[str]:
    try:
        f = getattr(lib, name)
    except AttributeError:
        return None
    f.restype = ctypes.c_char_p
    f.argtypes = []
    return f().decode()


def _embedded_hash(lib) -> Optional[str]:
    return _embedded_str(lib, "gfk_source_hash")


def build_arch(lib=None) -> Optional[str]:
    """The offload arch the kernel library was compiled for (embedded by the build)."""
    return _embedded_str(lib if lib is not None else kernels(), "gfk_build_arch")


def _check_source(lib) -> None:
    """Refuse a kernel library whose embedded source hash is not this tree's."""
    from . import srchash
    if not os.path.isdir(srchash.CSRC):
        return                       # no sources next to the package: nothing to compare
    got = _embedded_hash(lib)
    # the hash covers the arch the library was built for (embedded next to it), not the
    # PYTORCH_ROCM_ARCH of the loading process
    arch = _embedded_str(lib, "gfk_build_arch") or os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
    want = srchash.source_hash(arch)
    if got == want:
        return
    if KERNELS_SO_OVERRIDE:
        import logging
        logging.getLogger("gfedntm_amd.native").warning(
            "GFEDNTM_KERNELS_SO=%s: source hash %s, tree %s (A/B build, not checked)",
            KERNELS_SO, got, want)
        return
    raise RuntimeError(
        f"{KERNELS_SO} was built from other sources (embedded hash {got}, csrc/ hashes to "
        f"{want}): rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")


def kernels_hash() -> Optional[str]:
    """The source hash embedded in the loaded kernel library (None if not loaded)."""
    return _embedded_hash(kernels()) if kernels_available() else None


def runtime() -> Optional[ctypes.CDLL]:
    global _runtime, _runtime_tried
    if not _runtime_tried:
        _runtime_tried = True
        if os.path.exists(RUNTIME_SO):
            _runtime = ctypes.CDLL(RUNTIME_SO)
            from . import runtime_abi
            runtime_abi.declare(_runtime)
    return _runtime


def tokenizer_available() -> bool:
    return runtime() is not None


def local_vocabulary(texts: Sequence[str]) -> Dict[str, int]:
    from . import runtime_abi
    return runtime_abi.local_vocabulary(runtime(), texts)


def vectorize(texts: Sequence[str], vocabulary: Dict[str, int]):
    from . import runtime_abi
    return runtime_abi.vectorize(runtime(), texts, vocabulary)
