"""Vocabulary consensus utilities (stage 1 of the federation protocol).

Semantics (reference src/federation/client.py:358-376, server.py:270-288):
  * local vocabulary = CountVectorizer(lowercase=True, stop_words='english',
    default token_pattern) fitted on the client's documents;
  * global vocabulary = sorted union of all local vocabularies, term -> index
    by sorted position;
  * every client re-vectorizes its corpus with the global vocabulary.

Tokenization goes through the native C++ tokenizer (csrc/tokenizer.cpp) when
it is built -- it reproduces scikit-learn's default ``(?u)\\b\\w\\w+\\b``
pattern, lowercasing and the English stop-word list, and builds the CSR
matrix directly -- and falls back to scikit-learn otherwise.  Both paths are
checked against each other in tests/test_vocab.py.
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Sequence

import numpy as np
import scipy.sparse as sp


def _sklearn_cv(**kw):
    from sklearn.feature_extraction.text import CountVectorizer
    return CountVectorizer(input="content", lowercase=True, binary=False, **kw)


def local_vocabulary(texts: Sequence[str]) -> Dict[str, int]:
    """Term -> local column index, exactly as CountVectorizer.vocabulary_."""
    from ..ops import native
    if native.tokenizer_available():
        v = native.local_vocabulary(texts)      # None: non-ASCII corpus -> scikit-learn
        if v is not None:
            return v
    cv = _sklearn_cv(stop_words="english")
    cv.fit(texts)
    return {k: int(v) for k, v in cv.vocabulary_.items()}


def union_vocabulary(vocabs: Iterable[Iterable[str]]) -> List[str]:
    """Sorted union of terms (reference server.py:270-279)."""
    terms = set()
    for v in vocabs:
        terms.update(v)
    return sorted(terms)


def vocabulary_dict(terms: Sequence[str]) -> Dict[str, int]:
    return {t: i for i, t in enumerate(terms)}


def vectorize(texts: Sequence[str], vocabulary: Dict[str, int]) -> sp.csr_matrix:
    """Doc-term counts of ``texts`` over a fixed vocabulary (float32 CSR)."""
    from ..ops import native
    if native.tokenizer_available():
        m = native.vectorize(texts, vocabulary)
        if m is not None:
            return m
    cv = _sklearn_cv(vocabulary=vocabulary)
    m = cv.transform(texts).astype(np.float32)
    m.sort_indices()
    return m.tocsr()


def id2token(terms: Sequence[str]) -> Dict[int, str]:
    return {i: t for i, t in enumerate(terms)}
