"""Topic-model quality metrics.

* TSS / DSS on synthetic ground truth -- reference experiments/dss_tss/run_simulation.py:321-355
  and federated_avitm.py:152-193.
* NPMI coherence -- the reference delegates to the (missing) topicmodeler/gensim
  ``c_npmi`` (tm_wrapper.py:358-384).  Defined here precisely: for the top-N
  words of each topic, the mean over unordered word pairs of
  log((P(wi,wj)+eps) / (P(wi) P(wj))) / -log(P(wi,wj)+eps), eps = 1e-12, with
  probabilities estimated from document co-occurrence in a reference corpus
  (bag-of-words data has no word order, so there is no sliding window).  The
  co-occurrence counts are one GEMM on the device: D_bin[:, W]^T D_bin[:, W]
  over the union W of all topics' top words.
* Topic diversity (TD) and rank-biased overlap (RBO) -- tm_wrapper.py:386-400.
* Word-mover's distance between topic sets given word vectors -- aux_scripts/evaluation/wmd.py.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch


def tss(betas: np.ndarray, topic_vectors: np.ndarray) -> float:
    """Topic similarity score: sum over ground-truth topics of the best Bhattacharyya
    coefficient with a learned topic (run_simulation.py:321-334)."""
    return float(np.sum(np.max(np.sqrt(betas).dot(np.sqrt(topic_vectors.T)), axis=0)))


def dss(thetas_true: np.ndarray, thetas: np.ndarray, n_docs: Optional[int] = None) -> float:
    """Document similarity score (run_simulation.py:337-355)."""
    n_docs = len(thetas_true) if n_docs is None else n_docs
    a = np.sqrt(thetas_true).dot(np.sqrt(thetas_true.T))
    b = np.sqrt(thetas).dot(np.sqrt(thetas.T))
    return float(np.sum(np.abs(a - b)) / n_docs)


def betas_to_ground_truth_vocab(betas: np.ndarray, id2token: Dict[int, str], vocab_size: int,
                                prefix: str = "wd") -> np.ndarray:
    """Re-index a [K, V_learned] topic-word matrix onto the generator vocabulary
    ('wd<j>' -> column j), zero elsewhere, L1-normalised (reference
    auxiliary_functions.py:441-483, vectorised)."""
    out = np.zeros((betas.shape[0], vocab_size), dtype=np.float64)
    cols = np.array([int(id2token[i][len(prefix):]) for i in range(betas.shape[1])])
    out[:, cols] = betas
    s = out.sum(axis=1, keepdims=True)
    s[s == 0] = 1.0
    return out / s


def npmi_coherence(topics: Sequence[Sequence[int]], corpus: sp.csr_matrix, eps: float = 1e-12,
                   per_topic: bool = False, device=None):
    """NPMI of topics given as vocabulary indices, on a reference doc-term matrix."""
    topics = [list(map(int, t)) for t in topics]
    words = sorted({w for t in topics for w in t})
    pos = {w: i for i, w in enumerate(words)}
    sub = (corpus[:, words] > 0).astype(np.float32)
    n_docs = corpus.shape[0]
    dev = torch.device(device) if device is not None else torch.device("cpu")
    d = torch.from_numpy(sub.toarray()).to(dev)
    co = (d.t() @ d).double() / n_docs          # P(wi, wj); diagonal = P(wi)
    p = torch.diagonal(co)
    scores = []
    for t in topics:
        idx = torch.tensor([pos[w] for w in t], device=dev)
        pij = co[idx][:, idx]
        pi = p[idx]
        pmi = torch.log((pij + eps) / (pi[:, None] * pi[None, :] + 1e-300))
        npmi = pmi / (-torch.log(pij + eps))
        iu = torch.triu_indices(len(t), len(t), 1, device=dev)
        scores.append(float(npmi[iu[0], iu[1]].mean().item()))
    return scores if per_topic else float(np.mean(scores))


def topic_diversity(topics: Sequence[Sequence], topk: int = 25) -> float:
    """Fraction of unique words among the top-k words of all topics."""
    words = [w for t in topics for w in list(t)[:topk]]
    return len(set(words)) / max(len(words), 1)


def rbo(list1: Sequence, list2: Sequence, p: float = 0.9) -> float:
    """Extrapolated rank-biased overlap of two ranked lists (Webber et al. 2010)."""
    k = max(len(list1), len(list2))
    if k == 0:
        return 1.0
    x = 0
    s1, s2 = set(), set()
    summ = 0.0
    for d in range(1, k + 1):
        a = list1[d - 1] if d <= len(list1) else None
        b = list2[d - 1] if d <= len(list2) else None
        if a == b and a is not None:
            x += 1
        else:
            if a is not None and a in s2:
                x += 1
            if b is not None and b in s1:
                x += 1
        if a is not None:
            s1.add(a)
        if b is not None:
            s2.add(b)
        summ += (x / d) * p ** d
    return float((x / k) * p ** k + (1 - p) / p * summ)


def inverted_rbo(topics: Sequence[Sequence], topk: int = 10, p: float = 0.9) -> float:
    """1 - mean pairwise RBO between topics (topic distinctness)."""
    n = len(topics)
    if n < 2:
        return 1.0
    vals = [rbo(list(topics[i])[:topk], list(topics[j])[:topk], p)
            for i in range(n) for j in range(i + 1, n)]
    return float(1.0 - np.mean(vals))


def word_movers_distance(words1: Sequence[str], words2: Sequence[str], vectors: Dict[str, np.ndarray]
                         ) -> float:
    """WMD between two bags of words with uniform weights (exact EMD via LP)."""
    from scipy.optimize import linprog
    a = [w for w in words1 if w in vectors]
    b = [w for w in words2 if w in vectors]
    if not a or not b:
        return float("inf")
    va = np.stack([vectors[w] for w in a])
    vb = np.stack([vectors[w] for w in b])
    cost = np.sqrt(((va[:, None, :] - vb[None, :, :]) ** 2).sum(-1))
    n, m = cost.shape
    A_eq, b_eq = [], []
    for i in range(n):
        row = np.zeros(n * m); row[i * m:(i + 1) * m] = 1; A_eq.append(row); b_eq.append(1.0 / n)
    for j in range(m):
        row = np.zeros(n * m); row[j::m] = 1; A_eq.append(row); b_eq.append(1.0 / m)
    res = linprog(cost.ravel(), A_eq=np.array(A_eq), b_eq=np.array(b_eq), bounds=(0, None),
                  method="highs")
    return float(res.fun)


def mean_min_wmd(topics_ref: List[List[str]], topics_cmp: List[List[str]],
                 vectors: Dict[str, np.ndarray], n_words: int = 10) -> float:
    """Mean over reference topics of the minimum WMD to any compared topic (wmd.py:56-80)."""
    d = np.array([[word_movers_distance(t1[:n_words], t2[:n_words], vectors) for t2 in topics_cmp]
                  for t1 in topics_ref])
    return float(np.mean(np.min(d, axis=1)))
