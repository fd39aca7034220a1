"""Dataset preparation for AVITM / CTM training outside the federation.

Reference behaviour:
  * ``prepare_dataset`` -- src/models/base/pytorchavitm/utils/data_preparation.py:11-64:
    75/25 train/validation split (``random_state=42``), an English-stop-word
    CountVectorizer fitted on the training documents, BoW datasets of both;
  * ``prepare_ctm_dataset`` / ``prepare_hold_out_dataset`` /
    ``TopicModelDataPreparation`` / ``get_bag_of_words`` --
    contextualized_topic_models/utils/data_preparation.py:14-328;
  * ``WhiteSpacePreprocessing`` -- contextualized_topic_models/utils/preprocessing.py:6-60.

Differences: the matrices stay sparse (CSR) end to end -- the datasets hand them
to the device as CSR, nothing is densified on the host; documents may be given
as token lists or as strings.  SentenceTransformer is not installable here (and
the reference's import of it is commented out, so its embedding helpers were
dead code): contextual embeddings come from ``custom_embeddings`` or from a
user-supplied ``embedder(texts) -> np.ndarray`` callable.
"""
from __future__ import annotations

import string
import warnings
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp

from .bow import BOWDataset, CTMDataset

Embedder = Callable[[List[str]], np.ndarray]


def _as_text(doc) -> str:
    return doc if isinstance(doc, str) else " ".join(doc)


def _split(n: int, val_size: float, seed: int = 42):
    from sklearn.model_selection import train_test_split
    return train_test_split(np.arange(n), test_size=val_size, random_state=seed)


def _english_vectorizer(**kw):
    from sklearn.feature_extraction.text import CountVectorizer
    return CountVectorizer(input="content", lowercase=True, stop_words="english", binary=False, **kw)


def _id2token(cv) -> Dict[int, str]:
    return {i: t for i, t in enumerate(cv.get_feature_names_out())}


def prepare_dataset(corpus: Sequence, val_size: float = 0.25):
    """(train BOWDataset, val BOWDataset, input_size, id2token, docs_train, vectorizer)."""
    tr, va = _split(len(corpus), val_size)
    docs_train = [corpus[i] for i in tr]
    cv = _english_vectorizer()
    train_bow = cv.fit_transform([_as_text(d) for d in docs_train]).astype(np.float32)
    id2token = _id2token(cv)
    val_bow = cv.transform([_as_text(corpus[i]) for i in va]).astype(np.float32)
    return (BOWDataset(train_bow, id2token), BOWDataset(val_bow, id2token), len(id2token),
            id2token, docs_train, cv)


def get_bag_of_words(data: Sequence[Sequence], min_length: int) -> sp.csr_matrix:
    """Token-index sequences -> BoW rows of length ``min_length`` (rows whose indices
    sum to 0 are dropped and None entries ignored, like the reference)."""
    rows = []
    for x in data:
        a = np.asarray([v for v in x if v is not None], dtype=np.int64)
        if a.sum() == 0:
            continue
        rows.append(np.bincount(a, minlength=min_length))
    if not rows:
        return sp.csr_matrix((0, min_length), dtype=np.float32)
    width = max(len(r) for r in rows)
    return sp.csr_matrix(np.stack([np.pad(r, (0, width - len(r))) for r in rows]).astype(np.float32))


class TopicModelDataPreparation:
    """Vectorizer + contextual-embedding bookkeeping for CTM datasets."""

    def __init__(self, contextualized_model: Optional[str] = None, show_warning: bool = True,
                 max_seq_length: int = 128, embedder: Optional[Embedder] = None):
        self.contextualized_model = contextualized_model
        self.embedder = embedder
        self.vocab: List[str] = []
        self.id2token: Dict[int, str] = {}
        self.vectorizer = None
        self.label_encoder = None
        self.show_warning = show_warning
        self.max_seq_length = max_seq_length

    def _embed(self, texts: List[str], custom: Optional[np.ndarray]) -> np.ndarray:
        if custom is not None:
            if not isinstance(custom, np.ndarray):
                raise TypeError("contextualized embeddings must be a numpy.ndarray")
            return custom
        if self.embedder is None:
            raise RuntimeError("no contextual model available offline: pass custom_embeddings "
                               "or an embedder callable")
        return np.asarray(self.embedder(list(texts)), dtype=np.float32)

    def load(self, contextualized_embeddings, bow_embeddings, id2token, labels=None) -> CTMDataset:
        return CTMDataset(contextualized_embeddings, bow_embeddings, id2token, qt=self, labels=labels)

    def fit(self, text_for_contextual, text_for_bow, labels=None, custom_embeddings=None):
        from sklearn.feature_extraction.text import CountVectorizer
        if text_for_bow is not None and len(text_for_contextual) != len(text_for_bow):
            raise ValueError("text_for_contextual and text_for_bow differ in length")
        if custom_embeddings is not None and len(custom_embeddings) != len(text_for_contextual):
            raise ValueError("custom_embeddings and texts differ in length")
        if self.contextualized_model is None and custom_embeddings is None and self.embedder is None:
            raise ValueError("a contextualized model or contextualized embeddings must be defined")
        self.vectorizer = CountVectorizer()
        bow = self.vectorizer.fit_transform(text_for_bow).astype(np.float32)
        emb = self._embed(text_for_contextual, custom_embeddings)
        self.vocab = list(self.vectorizer.get_feature_names_out())
        self.id2token = dict(enumerate(self.vocab))
        enc = None
        if labels:
            from sklearn.preprocessing import OneHotEncoder
            self.label_encoder = OneHotEncoder()
            enc = self.label_encoder.fit_transform(np.asarray(labels).reshape(-1, 1)).toarray()
        return CTMDataset(emb, bow, self.id2token, qt=self, labels=enc)

    def transform(self, text_for_contextual, text_for_bow=None, custom_embeddings=None, labels=None):
        if custom_embeddings is not None and len(custom_embeddings) != len(text_for_contextual):
            raise ValueError("custom_embeddings and texts differ in length")
        if text_for_bow is not None:
            if len(text_for_bow) != len(text_for_contextual):
                raise ValueError("text_for_contextual and text_for_bow differ in length")
            bow = self.vectorizer.transform(text_for_bow).astype(np.float32)
        else:
            if self.show_warning:
                warnings.warn("no text_for_bow: expected only for cross-lingual ZeroShotTM")
            bow = sp.csr_matrix((len(text_for_contextual), max(len(self.vocab), 1)), dtype=np.float32)
        emb = self._embed(text_for_contextual, custom_embeddings)
        enc = None
        if labels:
            enc = self.label_encoder.transform(np.asarray(labels).reshape(-1, 1)).toarray()
        return CTMDataset(emb, bow, self.id2token, qt=self, labels=enc)


def prepare_ctm_dataset(corpus: Sequence, unpreprocessed_corpus: Optional[Sequence] = None,
                        custom_embeddings: Optional[np.ndarray] = None,
                        embedder: Optional[Embedder] = None, val_size: float = 0.25,
                        contextualized_model: str = "paraphrase-distilroberta-base-v1"):
    """(train CTMDataset, val CTMDataset, input_size, id2token, qt, embeddings_train,
    all embeddings, docs_train)."""
    if custom_embeddings is None:
        if unpreprocessed_corpus is None:
            raise TypeError("custom embeddings or an unpreprocessed corpus must be provided")
        if embedder is None:
            raise RuntimeError("no contextual model available offline: pass an embedder")
        custom_embeddings = np.asarray(embedder([_as_text(d) for d in unpreprocessed_corpus]),
                                       dtype=np.float32)
    custom_embeddings = np.asarray(custom_embeddings, dtype=np.float32)
    tr, va = _split(len(corpus), val_size)
    docs_train = [corpus[i] for i in tr]
    cv = _english_vectorizer()
    train_bow = cv.fit_transform([_as_text(d) for d in docs_train]).astype(np.float32)
    id2token = _id2token(cv)
    qt = TopicModelDataPreparation(contextualized_model=contextualized_model, embedder=embedder)
    qt.vectorizer, qt.id2token, qt.vocab = cv, id2token, list(id2token.values())
    emb_train, emb_val = custom_embeddings[tr], custom_embeddings[va]
    train = qt.load(emb_train, train_bow, id2token)
    val_docs = [_as_text(corpus[i]) for i in va]
    val = qt.transform(val_docs, val_docs, custom_embeddings=emb_val)
    return train, val, len(id2token), id2token, qt, emb_train, custom_embeddings, docs_train


def prepare_hold_out_dataset(hold_out_corpus: Sequence, qt: TopicModelDataPreparation,
                             unpreprocessed_ho_corpus: Optional[Sequence] = None,
                             embeddings_ho: Optional[np.ndarray] = None,
                             embedder: Optional[Embedder] = None) -> CTMDataset:
    if embeddings_ho is None:
        if unpreprocessed_ho_corpus is None:
            raise TypeError("custom embeddings or an unpreprocessed corpus must be provided")
        fn = embedder or qt.embedder
        if fn is None:
            raise RuntimeError("no contextual model available offline: pass an embedder")
        embeddings_ho = np.asarray(fn([_as_text(d) for d in unpreprocessed_ho_corpus]), dtype=np.float32)
    docs = [_as_text(d) for d in hold_out_corpus]
    return qt.transform(docs, docs, custom_embeddings=np.asarray(embeddings_ho, dtype=np.float32))


def english_stopwords() -> frozenset:
    """English stop words (nltk is not installed; scikit-learn's list is used)."""
    from sklearn.feature_extraction.text import ENGLISH_STOP_WORDS
    return ENGLISH_STOP_WORDS


class WhiteSpacePreprocessing:
    """Lowercase, strip punctuation, drop stop words, keep the ``vocabulary_size`` most
    frequent alphabetic tokens (>= 2 letters); documents left empty are removed."""

    def __init__(self, documents: Sequence[str], stopwords_language: str = "english",
                 vocabulary_size: int = 2000, stopwords: Optional[Sequence[str]] = None):
        if stopwords is None:
            if stopwords_language != "english":
                raise ValueError("only English stop words are bundled; pass stopwords=")
            stopwords = english_stopwords()
        self.documents = list(documents)
        self.stopwords = set(stopwords)
        self.vocabulary_size = vocabulary_size

    def preprocess(self) -> Tuple[List[str], List[str], List[str]]:
        from sklearn.feature_extraction.text import CountVectorizer
        table = str.maketrans(string.punctuation, " " * len(string.punctuation))
        docs = [" ".join(w for w in d.lower().translate(table).split() if w not in self.stopwords)
                for d in self.documents]
        cv = CountVectorizer(max_features=self.vocabulary_size, token_pattern=r"\b[a-zA-Z]{2,}\b")
        cv.fit(docs)
        vocab = set(cv.get_feature_names_out())
        docs = [" ".join(w for w in d.split() if w in vocab) for d in docs]
        kept = [(d, raw) for d, raw in zip(docs, self.documents) if d]
        return [d for d, _ in kept], [r for _, r in kept], sorted(vocab)
