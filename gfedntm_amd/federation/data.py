"""Client corpora for the federation (reference main.py:138-152, client.py:321-356).

* ``synthetic``: node ``id-1`` of a synthetic corpus -- either this framework's
  pickle-free counts npz (:meth:`SyntheticCorpus.save_counts_npz`) or the
  reference ``synthetic_all_nodes.npz`` schema, whose ``documents`` entry is an
  object array and therefore needs ``allow_pickle`` (only for files you trust;
  the flag is explicit).
* ``real``: a parquet with ``bow_text`` (and optionally ``embeddings``, arrays
  or space-separated strings) filtered by ``fos``.

A :class:`ClientCorpus` answers the two questions of stage 1: the local
vocabulary (CountVectorizer semantics) and the BoW over the agreed global
vocabulary.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import numpy as np
import scipy.sparse as sp

from ..data.synthetic import SyntheticCorpus, node_vocabulary_terms, remap_to_vocabulary
from ..data.vocab import local_vocabulary, vectorize


@dataclasses.dataclass
class ClientCorpus:
    texts: Optional[List[str]] = None
    synthetic: Optional[SyntheticCorpus] = None
    node: int = 0
    embeddings: Optional[np.ndarray] = None
    ground_truth_thetas: Optional[np.ndarray] = None
    ground_truth_betas: Optional[np.ndarray] = None

    @property
    def n_docs(self) -> int:
        if self.synthetic is not None:
            return self.synthetic.counts[self.node].shape[0]
        return len(self.texts)

    def ground_truth(self):
        """(doc-topic [D, K], topic-word [K, V_gen]) of the generator, or None: explicit
        fields (loaded files) or the node of an in-memory synthetic corpus."""
        if self.ground_truth_thetas is not None and self.ground_truth_betas is not None:
            return np.asarray(self.ground_truth_thetas), np.asarray(self.ground_truth_betas)
        if self.synthetic is not None and getattr(self.synthetic, "topic_vectors", None) is not None:
            return (np.asarray(self.synthetic.doc_topics[self.node]),
                    np.asarray(self.synthetic.topic_vectors))
        return None

    def local_terms(self) -> List[str]:
        if self.synthetic is not None:
            return sorted(node_vocabulary_terms(self.synthetic, self.node))
        return sorted(local_vocabulary(self.texts))

    def bow(self, vocab: Dict[str, int]) -> sp.csr_matrix:
        if self.synthetic is not None:
            return remap_to_vocabulary(self.synthetic, self.node, vocab)
        return vectorize(self.texts, vocab)


def _parse_embeddings(col) -> np.ndarray:
    vals = list(col)
    if vals and isinstance(vals[0], str):
        return np.stack([np.asarray(v.split(), dtype=np.float32) for v in vals])
    return np.stack([np.asarray(v, dtype=np.float32) for v in vals])


def load_client_corpus(data_type: str, source: str, client_id: int, fos: Optional[str] = None,
                       allow_pickle: bool = False) -> ClientCorpus:
    """``client_id`` is 1-based like the reference (node ``client_id - 1``)."""
    if data_type == "synthetic":
        with np.load(source, allow_pickle=False) as z:
            is_counts = "counts0_indptr" in z.files
        if is_counts:
            sc = SyntheticCorpus.load_counts_npz(source)
            node = client_id - 1
            return ClientCorpus(synthetic=sc, node=node, ground_truth_thetas=sc.doc_topics[node],
                                ground_truth_betas=sc.topic_vectors)
        if not allow_pickle:
            raise ValueError(f"{source} stores token lists as object arrays; pass "
                             "allow_pickle=True (--allow-pickle) only for files you trust, or "
                             "regenerate it with save_counts_npz")
        with np.load(source, allow_pickle=True) as z:
            docs = z["documents"][client_id - 1]
            texts = [" ".join(d) for d in docs]
            dt = z["doc_topics"][client_id - 1]
            tv = z["topic_vectors"]
        return ClientCorpus(texts=texts, ground_truth_thetas=np.asarray(dt),
                            ground_truth_betas=np.asarray(tv))
    if data_type == "real":
        import pandas as pd
        df = pd.read_parquet(source)
        if fos is not None:
            df = df[df["fos"] == fos]
        texts = [" ".join(map(str, row)) for row in df[["bow_text"]].values.tolist()]
        emb = _parse_embeddings(df["embeddings"]) if "embeddings" in df.columns else None
        return ClientCorpus(texts=texts, embeddings=emb)
    raise ValueError(f"data_type must be 'synthetic' or 'real', got {data_type!r}")
