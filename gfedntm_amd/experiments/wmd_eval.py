"""Word-mover's distances between non-collaborative (node) models and every model.

Reference: aux_scripts/evaluation/wmd.py:13-110 -- for each K, a [nodes x all
models] table of mean over the node model's topics of the minimum WMD to the
other model's topics, on the top ``n_words`` words, one CSV per (K, n_words).
The reference loads word2vec-google-news-300 through gensim's downloader; there
is no network here, so the word vectors are given as a file: word2vec text
format (``word v1 v2 ...`` per line, optional header) or an ``.npz`` with
``words`` and ``vectors`` arrays.  Vectors are L2-normalised like gensim's
``init_sims(replace=True)``.  Model folders are the ones written by
:mod:`gfedntm_amd.experiments.collab` (``topics.json``).
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Dict, List

import numpy as np

from ..eval.metrics import mean_min_wmd


def load_vectors(path: str) -> Dict[str, np.ndarray]:
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            words, vecs = [str(w) for w in z["words"]], np.asarray(z["vectors"], dtype=np.float64)
    else:
        words, rows = [], []
        with open(path, encoding="utf8") as f:
            for i, line in enumerate(f):
                parts = line.rstrip().split(" ")
                if i == 0 and len(parts) == 2 and all(p.isdigit() for p in parts):
                    continue
                words.append(parts[0])
                rows.append(np.asarray(parts[1:], dtype=np.float64))
        vecs = np.stack(rows)
    vecs = vecs / np.maximum(np.linalg.norm(vecs, axis=1, keepdims=True), 1e-12)
    return dict(zip(words, vecs))


def _topics(folder: str) -> List[List[str]]:
    with open(os.path.join(folder, "topics.json")) as f:
        return json.load(f)


def wmd_tables(path_models: str, path_save: str, vectors: Dict[str, np.ndarray],
               nr_tpcs_lst=(10, 20, 30, 40, 50), n_words_lst=(10, 50, 100, 200, 300)):
    import pandas as pd
    names = sorted(n for n in os.listdir(path_models) if os.path.isdir(os.path.join(path_models, n)))
    centr = sorted((n for n in names if n.startswith("centralized")), key=lambda n: int(n.split("_")[1]))
    os.makedirs(path_save, exist_ok=True)
    written = []
    for k in nr_tpcs_lst:
        nodes = [n for n in names if n.startswith("non_collaborative") and int(n.split("_")[-3]) == k]
        if not nodes:
            continue
        cols = [f"Node {i + 1}" for i in range(len(nodes))] + [f"Centr {n.split('_')[1]}" for n in centr]
        every = nodes + centr
        for nw in n_words_lst:
            d = np.zeros((len(nodes), len(every)))
            for i, ref in enumerate(nodes):
                tr = _topics(os.path.join(path_models, ref))
                for j, cmp_ in enumerate(every):
                    d[i, j] = mean_min_wmd(tr, _topics(os.path.join(path_models, cmp_)), vectors, nw)
            out = os.path.join(path_save, f"wmds_{k}tpcs_{nw}_words.csv")
            pd.DataFrame(d, index=cols[: len(nodes)], columns=cols).to_csv(out)
            written.append(out)
    return written


def main(argv=None):
    p = argparse.ArgumentParser(description="WMD between topic models")
    p.add_argument("--path_models", required=True)
    p.add_argument("--path_save", required=True)
    p.add_argument("--vectors", required=True, help="word2vec text file or .npz (words, vectors)")
    p.add_argument("--nr_tpcs_lst", type=str, default="10,20,30,40,50")
    p.add_argument("--n_words_lst", type=str, default="10,50,100,200,300")
    a = p.parse_args(argv)
    return wmd_tables(a.path_models, a.path_save, load_vectors(a.vectors),
                      [int(x) for x in a.nr_tpcs_lst.split(",")],
                      [int(x) for x in a.n_words_lst.split(",")])


if __name__ == "__main__":
    main()
