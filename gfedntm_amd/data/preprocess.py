"""Corpus preprocessing for topic modelling (stop words, equivalences, frequency
filters) producing the ``bow_text`` parquet the federation clients read.

Reference: aux_scripts/preprocessing/text_preproc.py:44-136 drives the external
topicmodeler (tm_wrapper.py:171-198, an empty git submodule in the reference)
with the preprocessing parameters ``min_lemas 15, no_below 15, no_above 0.4,
keep_n 100000`` plus stop-word and equivalence word lists in the JSON format
``{name, description, valid_for, visibility, wordlist: [...]}`` (equivalences as
``"term:replacement"``).  The filter semantics follow the gensim dictionary the
topicmodeler uses: tokens are whitespace-separated lemmas; stop words are
removed and equivalences applied; documents with fewer than ``min_lemas``
lemmas are dropped; the vocabulary keeps tokens present in at least
``no_below`` documents and at most ``no_above`` of them, then the ``keep_n``
most frequent (by document frequency, ties by first appearance).

Output (``out_dir``): ``corpus.parquet`` (input columns + ``bow_text``),
``vocabulary.txt`` (one term per line) and ``trainconfig.json``.
"""
from __future__ import annotations

import datetime
import json
import os
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np


def load_wordlists(paths: Iterable[str]) -> Tuple[Set[str], Dict[str, str]]:
    """Stop words and equivalences from word-list JSON files (``valid_for`` decides;
    entries with a ':' are equivalences)."""
    stop: Set[str] = set()
    equiv: Dict[str, str] = {}
    for p in paths:
        with open(p, encoding="utf8") as f:
            wl = json.load(f)
        kind = wl.get("valid_for", "stopwords")
        for w in wl.get("wordlist", []):
            if kind == "equivalences" or ":" in w:
                a, _, b = w.partition(":")
                equiv[a.strip()] = b.strip()
            else:
                stop.add(w.strip())
    return stop, equiv


class CorpusPreprocessor:
    def __init__(self, stopwords: Iterable[str] = (), equivalences: Optional[Dict[str, str]] = None,
                 min_lemas: int = 15, no_below: int = 15, no_above: float = 0.4,
                 keep_n: int = 100000):
        self.stopwords = set(stopwords)
        self.equivalences = dict(equivalences or {})
        self.min_lemas, self.no_below, self.no_above, self.keep_n = min_lemas, no_below, no_above, keep_n
        self.vocabulary: List[str] = []

    def clean(self, doc: str) -> List[str]:
        eq, stop = self.equivalences, self.stopwords
        out = []
        for t in doc.split():
            if t in stop:
                continue
            t = eq.get(t, t)
            if t and t not in stop:
                out.append(t)
        return out

    def fit_transform(self, docs: Sequence[str]) -> Tuple[List[str], np.ndarray]:
        """(bow_text of the kept documents, boolean mask of kept input documents)."""
        toks = [self.clean(d) for d in docs]
        keep = np.array([len(t) >= self.min_lemas for t in toks], dtype=bool)
        kept = [t for t, k in zip(toks, keep) if k]
        n = len(kept)
        df: Dict[str, int] = {}
        for t in kept:
            for w in dict.fromkeys(t):
                df[w] = df.get(w, 0) + 1
        max_df = self.no_above * n
        cand = [w for w, c in df.items() if c >= self.no_below and c <= max_df]
        order = {w: i for i, w in enumerate(df)}                     # first appearance
        cand.sort(key=lambda w: (-df[w], order[w]))
        vocab = set(cand[: self.keep_n])
        self.vocabulary = sorted(vocab)
        return [" ".join(w for w in t if w in vocab) for t in kept], keep


def preprocess_parquet(parquet_in: str, out_dir: str, id_field: str = "id",
                       lemmas_field: str = "lemmas", wordlists: Sequence[str] = (),
                       min_lemas: int = 15, no_below: int = 15, no_above: float = 0.4,
                       keep_n: int = 100000, trainer: str = "ctm") -> Dict:
    import pandas as pd
    stop, equiv = load_wordlists(wordlists)
    df = pd.read_parquet(parquet_in)
    pp = CorpusPreprocessor(stop, equiv, min_lemas, no_below, no_above, keep_n)
    bow, keep = pp.fit_transform(df[lemmas_field].fillna("").astype(str).tolist())
    out = df.loc[keep].copy()
    out["bow_text"] = bow
    os.makedirs(out_dir, exist_ok=True)
    out.to_parquet(os.path.join(out_dir, "corpus.parquet"))
    with open(os.path.join(out_dir, "vocabulary.txt"), "w", encoding="utf8") as f:
        f.write("\n".join(pp.vocabulary) + ("\n" if pp.vocabulary else ""))
    name = os.path.splitext(os.path.basename(parquet_in))[0]
    cfg = {
        "name": name, "description": "", "visibility": "Public", "trainer": trainer,
        "Preproc": {"min_lemas": min_lemas, "no_below": no_below, "no_above": no_above,
                    "keep_n": keep_n, "stopwords": list(wordlists), "equivalences": []},
        "TrDtSet": {"name": name, "Dtsets": [{"parquet": parquet_in, "source": name,
                                              "idfld": id_field, "lemmasfld": [lemmas_field],
                                              "filter": ""}]},
        "TMparam": {}, "creation_date": datetime.datetime.now().isoformat(),
        "hierarchy-level": 0, "htm-version": None,
        "n_docs_in": int(len(df)), "n_docs_out": int(keep.sum()), "vocab_size": len(pp.vocabulary),
    }
    with open(os.path.join(out_dir, "trainconfig.json"), "w", encoding="utf8") as f:
        json.dump(cfg, f, indent=2)
    return cfg
