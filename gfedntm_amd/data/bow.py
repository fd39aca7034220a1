"""Bag-of-words corpora: host CSR, device CSR, reference-compatible datasets,
and the deterministic minibatch schedule that drives device-resident training.

The reference densifies every document to a float row of length V on the host
and copies B x V x 4 bytes to the device every step (reference
src/models/base/pytorchavitm/datasets/bow_dataset.py:30-34,
contextualized_topic_models/datasets/dataset.py:30-48).  Here the whole local
shard lives in HBM as CSR (int32 indptr/indices + fp32 counts); kernels gather
the non-zeros directly and the host never touches a minibatch.

``BOWDataset`` / ``CTMDataset`` keep the reference ``__getitem__`` contract
({'X': row} / {'X_bow', 'X_contextual'[, 'labels']}) for user code that wants
a torch DataLoader.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch
from torch.utils.data import Dataset


def to_csr(x) -> sp.csr_matrix:
    """Any dense/sparse doc-term matrix -> float32 CSR with sorted indices."""
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    m = sp.csr_matrix(x, dtype=np.float32)
    m.sum_duplicates()
    m.sort_indices()
    return m


class BOWDataset(Dataset):
    """Reference-compatible BoW dataset (reference bow_dataset.py:6-34), CSR-backed."""

    def __init__(self, X, idx2token):
        self.csr = to_csr(X)
        self.idx2token = idx2token

    @property
    def X(self) -> sp.csr_matrix:
        return self.csr

    def __len__(self):
        return self.csr.shape[0]

    def __getitem__(self, i):
        return {"X": torch.from_numpy(self.csr[i].toarray().ravel())}


class CTMDataset(Dataset):
    """Reference-compatible CTM dataset (reference dataset.py:6-48), CSR-backed."""

    def __init__(self, X_contextual, X_bow, idx2token, qt=None, labels=None):
        self.csr = to_csr(X_bow)
        if self.csr.shape[0] != len(X_contextual):
            raise ValueError("BoW and contextual embeddings have different sizes")
        if labels is not None and labels.shape[0] != self.csr.shape[0]:
            raise ValueError("labels and BoW have different sizes")
        self.X_contextual = np.asarray(X_contextual, dtype=np.float32)
        self.idx2token = idx2token
        self.labels = None if labels is None else (
            labels.toarray() if sp.issparse(labels) else np.asarray(labels)).astype(np.float32)
        self.qt = qt

    @property
    def X_bow(self) -> sp.csr_matrix:
        return self.csr

    def __len__(self):
        return self.csr.shape[0]

    def __getitem__(self, i):
        out = {"X_bow": torch.from_numpy(self.csr[i].toarray().ravel()),
               "X_contextual": torch.from_numpy(self.X_contextual[i])}
        if self.labels is not None:
            out["labels"] = torch.from_numpy(self.labels[i])
        return out


class DeviceCSR:
    """A CSR document-term matrix resident on one device.

    ``indptr`` is int32 [D+1], ``indices`` int32 [nnz] (sorted per row),
    ``values`` fp32 [nnz].  ``row_len_max`` is kept for kernel launch sizing.
    """

    def __init__(self, csr: sp.csr_matrix, device, contextual: Optional[np.ndarray] = None,
                 labels: Optional[np.ndarray] = None):
        csr = to_csr(csr)
        if csr.nnz >= 2**31:
            raise ValueError("shard too large for int32 CSR offsets; split it")
        self.n_docs, self.vocab_size = csr.shape
        self.device = torch.device(device)
        self.indptr = torch.from_numpy(csr.indptr.astype(np.int32)).to(self.device)
        self.indices = torch.from_numpy(csr.indices.astype(np.int32)).to(self.device)
        self.values = torch.from_numpy(csr.data.astype(np.float32)).to(self.device)
        lens = np.diff(csr.indptr)
        self.row_len_max = int(lens.max()) if len(lens) else 0
        self.nnz = int(csr.nnz)
        self.contextual = None if contextual is None else torch.from_numpy(
            np.ascontiguousarray(contextual, dtype=np.float32)).to(self.device)
        self.labels = None if labels is None else torch.from_numpy(
            np.ascontiguousarray(labels, dtype=np.float32)).to(self.device)

    def dense_rows(self, doc_ids: torch.Tensor) -> torch.Tensor:
        """Densify a set of rows on device (used by the pure-torch backend)."""
        doc_ids = doc_ids.to(self.device, torch.long)
        starts = self.indptr[doc_ids].long()
        lens = self.indptr[doc_ids + 1].long() - starts
        n = doc_ids.numel()
        out = torch.zeros(n, self.vocab_size, device=self.device, dtype=torch.float32)
        total = int(lens.sum().item()) if n else 0
        if total == 0:
            return out
        row_of = torch.repeat_interleave(torch.arange(n, device=self.device), lens)
        first = torch.cumsum(lens, 0) - lens
        pos = torch.arange(total, device=self.device) - first[row_of] + starts[row_of]
        out[row_of, self.indices[pos].long()] = self.values[pos]
        return out


@dataclasses.dataclass
class BatchPlan:
    """Deterministic plan of minibatches for ``n_steps`` local steps.

    Mirrors ``DataLoader(shuffle=True, drop_last=False)`` iteration with the
    iterator reset at every epoch end (reference federated_avitm.py:114-138):
    each epoch is a fresh permutation cut into ceil(D/B) batches, the last
    one possibly short.  ``order`` is the concatenated permutation stream,
    and step s uses ``order[start[s] : start[s] + size[s]]``.
    """

    order: np.ndarray        # int32 [n_epochs * D]
    start: np.ndarray        # int32 [n_steps]
    size: np.ndarray         # int32 [n_steps]
    epoch: np.ndarray        # int32 [n_steps]
    mb: np.ndarray           # int32 [n_steps]  minibatch index within the epoch
    epoch_end: np.ndarray    # bool  [n_steps]  True on the last minibatch of an epoch
    n_docs: int
    batch_size: int

    @property
    def n_steps(self) -> int:
        return len(self.start)

    @staticmethod
    def build(n_docs: int, batch_size: int, n_steps: int, seed: int = 0) -> "BatchPlan":
        if n_docs <= 0:
            raise ValueError("empty shard")
        per_epoch = -(-n_docs // batch_size)
        n_epochs = -(-n_steps // per_epoch) if n_steps else 0
        rng = np.random.default_rng(seed)
        order = np.concatenate([rng.permutation(n_docs) for _ in range(max(n_epochs, 1))])
        s = np.arange(n_steps)
        ep, mb = s // per_epoch, s % per_epoch
        start = ep * n_docs + mb * batch_size
        size = np.minimum(batch_size, n_docs - mb * batch_size)
        return BatchPlan(order.astype(np.int32), start.astype(np.int32), size.astype(np.int32),
                         ep.astype(np.int32), mb.astype(np.int32), mb == per_epoch - 1,
                         n_docs, batch_size)

    def batch(self, step: int) -> np.ndarray:
        return self.order[self.start[step]: self.start[step] + self.size[step]]


def corpus_from_texts(texts: Sequence[str], vocabulary: Dict[str, int]) -> sp.csr_matrix:
    from .vocab import vectorize
    return vectorize(texts, vocabulary)


def stack_shards(shards: List[sp.csr_matrix]) -> sp.csr_matrix:
    return sp.vstack(shards, format="csr")
