"""Host C++ runtime (csrc/runtime.cpp): exact CountVectorizer parity and a sanitizer run."""
import os
import shutil
import subprocess

import numpy as np
import pytest
from sklearn.feature_extraction.text import CountVectorizer

from gfedntm_amd.ops import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
needs_rt = pytest.mark.skipif(not native.tokenizer_available(), reason="runtime not built")


def _corpus(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    words = ["Alpha", "beta", "GAMMA", "delta_x", "a", "I", "12", "x9", "the", "and", "foo-bar",
             "it's", "e.g.", "__init__", "Rock'n'roll", "v2.0", "ÀÉ"[:0] + "z", "\t", "CamelCase"]
    return [" ".join(rng.choice(words, size=rng.integers(0, 40))) + str(rng.choice([".", "!", ""]))
            for _ in range(n)]


@needs_rt
def test_vocabulary_and_csr_match_sklearn_exactly():
    from gfedntm_amd.ops import runtime_abi
    lib = native.runtime()
    texts = _corpus()
    ref = CountVectorizer(lowercase=True, stop_words="english").fit(texts).vocabulary_
    assert runtime_abi.local_vocabulary(lib, texts) == ref
    Xr = CountVectorizer(vocabulary=ref).transform(texts).astype(np.float32)
    Xr.sort_indices()
    Xo = runtime_abi.vectorize(lib, texts, ref)
    assert Xo.shape == Xr.shape and (Xo != Xr).nnz == 0
    assert np.array_equal(Xo.indptr, Xr.indptr) and np.array_equal(Xo.indices, Xr.indices)


@needs_rt
def test_non_ascii_corpus_falls_back_to_sklearn():
    from gfedntm_amd.data.vocab import local_vocabulary, vectorize
    from gfedntm_amd.ops import runtime_abi
    texts = _corpus(200) + ["Über naïve café", "ÉCOLE école"]
    assert runtime_abi.local_vocabulary(native.runtime(), texts) is None
    ref = CountVectorizer(stop_words="english").fit(texts).vocabulary_
    v = local_vocabulary(texts)
    assert v == ref and "über" in v
    assert (vectorize(texts, v) != CountVectorizer(vocabulary=ref).transform(texts)).nnz == 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_runtime_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "rt_sanitize")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-pthread", os.path.join(ROOT, "tools", "native_tests", "runtime_sanitize.cpp"),
           os.path.join(ROOT, "csrc", "runtime.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("sanitizer toolchain unavailable: " + r.stderr[-300:])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0 and "runtime sanitize ok" in run.stdout, run.stderr[-2000:]


def test_kernel_library_is_tied_to_the_sources(monkeypatch):
    """The kernel library embeds the hash of the csrc/ it was built from; the loader
    accepts exactly the tree's hash and refuses any other build unless
    GFEDNTM_KERNELS_SO names it on purpose (A/B timing)."""
    from gfedntm_amd.ops import srchash
    if not native.kernels_available():
        pytest.skip("kernel library not built")
    assert native.kernels_hash() == srchash.source_hash()

    class _Fn:
        def __init__(self, v):
            self.v = v
            self.restype = self.argtypes = None

        def __call__(self):
            return self.v

    class _Lib:
        def __init__(self, v):
            self.gfk_source_hash = _Fn(v)

    native._check_source(_Lib(srchash.source_hash().encode()))
    monkeypatch.setattr(native, "KERNELS_SO_OVERRIDE", None)
    with pytest.raises(RuntimeError, match="other sources"):
        native._check_source(_Lib(b"0000000000000000"))
    monkeypatch.setattr(native, "KERNELS_SO_OVERRIDE", "/tmp/ab/libgfedntm_kernels.so")
    native._check_source(_Lib(b"0000000000000000"))      # explicit A/B build: warn only


def test_source_check_uses_the_embedded_build_arch(monkeypatch):
    """The hash is recomputed with the arch the library was built for (embedded next to
    it), so a loader with another PYTORCH_ROCM_ARCH in its environment (or none) still
    accepts the tree's own build."""
    from gfedntm_amd.ops import srchash
    if not native.kernels_available():
        pytest.skip("kernel library not built")
    lib = native.kernels()
    assert native.build_arch(lib) == "gfx950"
    monkeypatch.setattr(native, "KERNELS_SO_OVERRIDE", None)
    for env in ("gfx942", None):
        if env is None:
            monkeypatch.delenv("PYTORCH_ROCM_ARCH", raising=False)
        else:
            monkeypatch.setenv("PYTORCH_ROCM_ARCH", env)
        native._check_source(lib)
    assert native.kernels_hash() == srchash.source_hash("gfx950")
