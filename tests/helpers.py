"""Shared fixtures for tests: tiny synthetic corpora."""
import numpy as np
import scipy.sparse as sp

from gfedntm_amd.data.synthetic import generate_synthetic, node_vocabulary_terms, remap_to_vocabulary
from gfedntm_amd.data.vocab import union_vocabulary, vocabulary_dict


def tiny_corpus(V=300, K=8, n_docs=100, n_nodes=2, seed=0, nwords=(30, 60)):
    c = generate_synthetic(vocab_size=V, n_topics=K, n_docs=n_docs, n_nodes=n_nodes,
                           frozen_topics=2, seed=seed, nwords=nwords)
    terms = union_vocabulary([node_vocabulary_terms(c, i) for i in range(n_nodes)])
    voc = vocabulary_dict(terms)
    shards = [remap_to_vocabulary(c, i, voc) for i in range(n_nodes)]
    return c, terms, shards


def random_csr(n_docs, V, nnz_per_row, seed=0):
    rng = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for d in range(n_docs):
        k = rng.integers(1, nnz_per_row + 1)
        c = rng.choice(V, size=min(k, V), replace=False)
        rows += [d] * len(c)
        cols += list(c)
        vals += list(rng.integers(1, 5, size=len(c)).astype(np.float32))
    m = sp.csr_matrix((vals, (rows, cols)), shape=(n_docs, V), dtype=np.float32)
    m.sort_indices()
    return m
