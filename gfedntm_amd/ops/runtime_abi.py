"""ctypes binding of the host runtime (csrc/runtime.cpp): CountVectorizer-compatible
vocabulary building and CSR vectorisation, multithreaded in C++.

Exact for ASCII corpora; a corpus with any non-ASCII character goes to
scikit-learn (whose Unicode-aware ``\\w`` and ``str.lower`` the C++ tokenizer does
not replicate), so results never differ from the reference recipe.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp

P = C.c_void_p
I64P = C.POINTER(C.c_int64)


def declare(lib):
    lib.gfr_free.argtypes = [P]
    lib.gfr_vocabulary.argtypes = [C.c_char_p, I64P, C.c_int64, C.c_char_p, I64P, C.c_int64,
                                   C.c_int, C.POINTER(C.c_void_p), I64P, I64P]
    lib.gfr_vocabulary.restype = C.c_int
    lib.gfr_vectorize.argtypes = [C.c_char_p, I64P, C.c_int64, C.c_char_p, I64P,
                                  C.POINTER(C.c_int32), C.c_int64, C.c_int, I64P,
                                  C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), I64P]
    lib.gfr_vectorize.restype = C.c_int


def _threads() -> int:
    return int(os.environ.get("GFEDNTM_RUNTIME_THREADS", "0"))


def _pack(strings: Sequence[str]) -> Optional[Tuple[bytes, np.ndarray]]:
    """One byte buffer + int64 offsets; None if any string is not ASCII."""
    parts = []
    offs = np.zeros(len(strings) + 1, dtype=np.int64)
    for i, s in enumerate(strings):
        if not s.isascii():
            return None
        b = s.encode("ascii")
        parts.append(b)
        offs[i + 1] = offs[i] + len(b)
    return b"".join(parts), offs


def _ptr(a: np.ndarray, ctype):
    return a.ctypes.data_as(C.POINTER(ctype))


def local_vocabulary(lib, texts: Sequence[str]) -> Optional[Dict[str, int]]:
    """CountVectorizer(lowercase=True, stop_words='english').fit(texts).vocabulary_, or
    None when the corpus is not ASCII (caller falls back to scikit-learn)."""
    from sklearn.feature_extraction.text import ENGLISH_STOP_WORDS
    packed = _pack(list(texts))
    if packed is None:
        return None
    stop = _pack(sorted(ENGLISH_STOP_WORDS))
    buf, offs = packed
    sbuf, soffs = stop
    out, out_len, n = C.c_void_p(), C.c_int64(), C.c_int64()
    rc = lib.gfr_vocabulary(buf, _ptr(offs, C.c_int64), len(texts), sbuf, _ptr(soffs, C.c_int64),
                            len(soffs) - 1, _threads(), C.byref(out), C.byref(out_len), C.byref(n))
    if rc:
        raise RuntimeError(f"gfr_vocabulary failed ({rc})")
    try:
        raw = C.string_at(out, out_len.value).decode("ascii")
    finally:
        lib.gfr_free(out)
    terms: List[str] = raw.split("\n")[:-1] if raw else []
    return {t: i for i, t in enumerate(terms)}


def vectorize(lib, texts: Sequence[str], vocabulary: Dict[str, int]) -> Optional[sp.csr_matrix]:
    """CountVectorizer(vocabulary=vocabulary).transform(texts) as float32 CSR with sorted
    indices, or None for a non-ASCII corpus or vocabulary."""
    packed = _pack(list(texts))
    items = sorted(vocabulary.items(), key=lambda kv: kv[1])
    vpacked = _pack([k for k, _ in items])
    if packed is None or vpacked is None:
        return None
    buf, offs = packed
    vbuf, voffs = vpacked
    cols = np.asarray([v for _, v in items], dtype=np.int32)
    n = len(texts)
    indptr = np.zeros(n + 1, dtype=np.int64)
    ix, dv, nnz = C.c_void_p(), C.c_void_p(), C.c_int64()
    rc = lib.gfr_vectorize(buf, _ptr(offs, C.c_int64), n, vbuf, _ptr(voffs, C.c_int64),
                           _ptr(cols, C.c_int32), len(cols), _threads(), _ptr(indptr, C.c_int64),
                           C.byref(ix), C.byref(dv), C.byref(nnz))
    if rc:
        raise RuntimeError(f"gfr_vectorize failed ({rc})")
    try:
        k = nnz.value
        indices = np.ctypeslib.as_array(C.cast(ix, C.POINTER(C.c_int32)), shape=(max(k, 1),))[:k].copy()
        data = np.ctypeslib.as_array(C.cast(dv, C.POINTER(C.c_float)), shape=(max(k, 1),))[:k].copy()
    finally:
        lib.gfr_free(ix)
        lib.gfr_free(dv)
    n_cols = (max(vocabulary.values()) + 1) if vocabulary else 0
    return sp.csr_matrix((data, indices, indptr), shape=(n, n_cols))
