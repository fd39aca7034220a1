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
