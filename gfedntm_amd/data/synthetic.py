"""Synthetic federated LDA / ProdLDA corpora with ground truth.

Same generative process and npz schema as the reference generator
(reference src/utils/generate_synthetic.py:33-96 and
experiments/dss_tss/run_simulation.py:77-181):

  * K topics over V terms, beta_k ~ Dir(eta * 1_V);
  * every node shares ``frozen_topics`` topics at prior alpha and owns
    ``own_topics = (K - frozen) // n_nodes`` topics at alpha, the remaining
    topics get alpha / 1e4; the non-frozen prior is rotated by ``own_topics``
    from one node to the next;
  * doc length ~ U[nwords[0], nwords[1]); tokens are ``'wd<index>'``.

Instead of drawing one multinomial per token (the reference's O(tokens) Python
loop), the LDA counts of a document are drawn in one shot as
Multinomial(len, theta_d @ beta), which has exactly the same distribution.  The
``prodlda`` variant keeps the per-token topic draw but samples the words of a
(doc, topic) group jointly from normalize(beta_t ** theta_dt), which again
matches the reference's per-token draw in distribution.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional

import numpy as np
import scipy.sparse as sp


def rotate_left(values: List[float], d: int) -> List[float]:
    """Rotation used between nodes (reference rotateArray)."""
    if not values:
        return values
    d %= len(values)
    return values[d:] + values[:d]


@dataclasses.dataclass
class SyntheticCorpus:
    topic_vectors: np.ndarray          # [K, V] ground-truth topic-word
    doc_topics: List[np.ndarray]       # per node [n_docs, K]
    counts: List[sp.csr_matrix]        # per node [n_docs, V] (columns = generator vocab)
    n_nodes: int
    vocab_size: int
    n_topics: int
    frozen_topics: int
    beta: float
    alpha: float
    n_docs: int
    nwords: tuple

    def tokens(self, node: int, doc: int) -> List[str]:
        row = self.counts[node].getrow(doc)
        return [f"wd{j}" for j, c in zip(row.indices, row.data.astype(np.int64)) for _ in range(c)]

    def documents(self, node: int) -> List[List[str]]:
        """Token lists for one node (reference ``documents[node]``)."""
        return [self.tokens(node, d) for d in range(self.counts[node].shape[0])]

    def texts(self, node: int) -> List[str]:
        """Space-joined documents as the reference client builds them (client.py:345-347)."""
        return [" ".join(t) for t in self.documents(node)]

    def save_npz(self, path: str) -> None:
        """Writes the reference ``synthetic_all_nodes.npz`` schema."""
        docs = np.empty(self.n_nodes, dtype=object)
        for i in range(self.n_nodes):
            docs[i] = self.documents(i)
        np.savez(path, n_nodes=self.n_nodes, vocab_size=self.vocab_size, n_topics=self.n_topics,
                 frozen_topics=self.frozen_topics, beta=self.beta, alpha=self.alpha,
                 n_docs=self.n_docs, nwords=np.asarray(self.nwords),
                 topic_vectors=self.topic_vectors, doc_topics=np.stack(self.doc_topics),
                 documents=docs)

    def save_counts_npz(self, path: str) -> None:
        """Compact, pickle-free variant: per-node CSR counts instead of token lists."""
        arrays = dict(n_nodes=self.n_nodes, vocab_size=self.vocab_size, n_topics=self.n_topics,
                      frozen_topics=self.frozen_topics, beta=self.beta, alpha=self.alpha,
                      n_docs=self.n_docs, nwords=np.asarray(self.nwords),
                      topic_vectors=self.topic_vectors, doc_topics=np.stack(self.doc_topics))
        for i, m in enumerate(self.counts):
            arrays[f"counts{i}_indptr"] = m.indptr
            arrays[f"counts{i}_indices"] = m.indices
            arrays[f"counts{i}_data"] = m.data
        np.savez(path, **arrays)

    @staticmethod
    def load_counts_npz(path: str) -> "SyntheticCorpus":
        z = np.load(path, allow_pickle=False)
        n = int(z["n_nodes"])
        V = int(z["vocab_size"])
        counts = []
        for i in range(n):
            ip = z[f"counts{i}_indptr"]
            counts.append(sp.csr_matrix((z[f"counts{i}_data"], z[f"counts{i}_indices"], ip),
                                        shape=(len(ip) - 1, V)))
        return SyntheticCorpus(z["topic_vectors"], list(z["doc_topics"]), counts, n, V,
                               int(z["n_topics"]), int(z["frozen_topics"]), float(z["beta"]),
                               float(z["alpha"]), int(z["n_docs"]), tuple(z["nwords"].tolist()))


def node_priors(n_topics: int, n_nodes: int, frozen_topics: int, alpha: float) -> List[np.ndarray]:
    """Dirichlet prior of every node (frozen part + rotated own part)."""
    own = (n_topics - frozen_topics) // n_nodes
    frozen = frozen_topics * [alpha]
    nofrozen = own * [alpha] + (n_topics - frozen_topics - own) * [alpha / 10000.0]
    out = []
    for _ in range(n_nodes):
        out.append(np.asarray(frozen + nofrozen, dtype=np.float64))
        nofrozen = rotate_left(nofrozen, own)
    return out


def generate_synthetic(vocab_size: int = 5000, n_topics: int = 50, beta: float = 1e-2,
                       alpha: Optional[float] = None, n_docs: int = 1000,
                       nwords=(150, 250), n_nodes: int = 5, frozen_topics: int = 5,
                       alg: str = "lda", seed: int = 0) -> SyntheticCorpus:
    rng = np.random.default_rng(seed)
    alpha = 1.0 / n_topics if alpha is None else alpha
    topic_vectors = rng.dirichlet(vocab_size * [beta], n_topics)
    priors = node_priors(n_topics, n_nodes, frozen_topics, alpha)
    doc_topics = [rng.dirichlet(p, n_docs) for p in priors]
    counts = []
    for node in range(n_nodes):
        lens = rng.integers(nwords[0], nwords[1], size=n_docs)
        theta = doc_topics[node]
        if alg == "lda":
            p = theta @ topic_vectors
            p /= p.sum(axis=1, keepdims=True)
            dense = rng.multinomial(lens, p)
        elif alg == "prodlda":
            dense = np.zeros((n_docs, vocab_size), dtype=np.int64)
            per_topic = rng.multinomial(lens, theta / theta.sum(axis=1, keepdims=True))
            for d in range(n_docs):
                for t in np.nonzero(per_topic[d])[0]:
                    w = np.power(topic_vectors[t], theta[d, t])
                    dense[d] += rng.multinomial(per_topic[d, t], w / w.sum())
        else:
            raise ValueError("alg must be 'lda' or 'prodlda'")
        counts.append(sp.csr_matrix(dense.astype(np.float32)))
    return SyntheticCorpus(topic_vectors, doc_topics, counts, n_nodes, vocab_size, n_topics,
                           frozen_topics, beta, alpha, n_docs, tuple(nwords))


def node_vocabulary_terms(corpus: SyntheticCorpus, node: int) -> List[str]:
    """Local vocabulary of a synthetic node without materializing token strings.

    ``'wd<j>'`` tokens survive CountVectorizer unchanged (lowercase, >= 2 word
    characters, not an English stop word), so the local vocabulary is exactly
    the set of generator columns with a non-zero count.
    """
    cols = np.unique(corpus.counts[node].indices)
    return [f"wd{j}" for j in cols]


def remap_to_vocabulary(corpus: SyntheticCorpus, node: int, vocab: dict) -> sp.csr_matrix:
    """Re-index a node's counts to the global vocabulary (sorted-union order)."""
    m = corpus.counts[node].tocoo()
    col_map = np.full(corpus.vocab_size, -1, dtype=np.int64)
    for j in np.unique(m.col):
        col_map[j] = vocab[f"wd{j}"]
    out = sp.csr_matrix((m.data, (m.row, col_map[m.col])),
                        shape=(m.shape[0], len(vocab)), dtype=np.float32)
    out.sort_indices()
    return out
