"""Collaborative (centralized) vs non-collaborative topic models on a real corpus.

Reference: experiments/collab_vs_non_collab/train.py:22-101 -- for every
iteration, centralized models with K in ``ntopics_centralized`` on the whole
corpus, then one model per field of study (``fos`` column) and K; RBO and TD of
each model (tm_wrapper.py:386-400).  The reference shells out to the external
topicmodeler (empty submodule); here the models are this framework's ProdLDA /
CombinedTM.  Every model folder (``centralized_{K}_{iter}_{date}`` /
``non_collaborative_{fos}_{K}_{iter}_{date}``) holds ``model.npz`` (betas,
thetas, topics as the federation writes them), ``topics.json`` (top words per
topic, for WMD) and ``metrics.json`` (TD, inverted RBO, NPMI on its corpus).

Usage: ``python -m gfedntm_amd.experiments.collab --path_corpus corpus.parquet
--models_folder out/ --ntopics_centralized 10,20``
"""
from __future__ import annotations

import argparse
import datetime
import json
import logging
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..data.bow import BOWDataset, CTMDataset
from ..data.vocab import local_vocabulary, vectorize
from ..eval.export import postprocess_thetas, save_model_as_npz
from ..eval.metrics import inverted_rbo, npmi_coherence, topic_diversity
from ..utils.config import load_config, model_kwargs_from_params


def train_one(texts: List[str], n_topics: int, params: Dict, out_dir: str, device,
              trainer: str = "avitm", embeddings: Optional[np.ndarray] = None, n_words: int = 300,
              seed: int = 0) -> Dict:
    from ..models import AVITM, CombinedTM
    vocab = local_vocabulary(texts)
    X = vectorize(texts, vocab)
    id2token = {i: t for t, i in vocab.items()}
    kw = model_kwargs_from_params(params)
    kw.update(n_components=n_topics, verbose=False)
    torch.manual_seed(seed)
    if trainer == "ctm":
        if embeddings is None:
            raise ValueError("the ctm trainer needs an embeddings column")
        tm = CombinedTM(input_size=len(vocab), contextual_size=embeddings.shape[1], device=device, **kw)
        ds = CTMDataset(embeddings, X, id2token)
    else:
        tm = AVITM(input_size=len(vocab), device=device, **kw)
        ds = BOWDataset(X, id2token)
    tm.fit(ds)
    betas = tm.get_topic_word_distribution()
    thetas = postprocess_thetas(tm.get_doc_topic_distribution(ds, 20))
    top = np.argsort(-betas, axis=1)[:, :n_words]
    topics_words = [[id2token[int(i)] for i in row] for row in top]
    os.makedirs(out_dir, exist_ok=True)
    save_model_as_npz(os.path.join(out_dir, "model.npz"), betas, thetas, n_topics,
                      [t[:10] for t in topics_words])
    with open(os.path.join(out_dir, "topics.json"), "w") as f:
        json.dump(topics_words, f)
    metrics = {"n_topics": n_topics, "n_docs": len(texts), "vocab_size": len(vocab),
               "td": topic_diversity(topics_words, 25), "irbo": inverted_rbo(topics_words, 10),
               "npmi": float(npmi_coherence(top[:, :10], X, device=device))}
    with open(os.path.join(out_dir, "metrics.json"), "w") as f:
        json.dump(metrics, f, indent=2)
    return metrics


def train(path_corpus: str, models_folder: str, ntopics_centralized: List[int],
          ntopics_nodes: Optional[List[int]] = None, iters: int = 1, start: int = 0,
          fos_name: str = "fos", text_field: str = "bow_text", trainer: str = "avitm",
          params: Optional[Dict] = None, device=None, logger=None) -> List[Dict]:
    import pandas as pd
    logger = logger or logging.getLogger("gfedntm_amd.collab")
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    params = dict(params or load_config().training_params)
    df = pd.read_parquet(path_corpus)
    emb = None
    if trainer == "ctm" and "embeddings" in df.columns:
        from ..federation.data import _parse_embeddings
        emb = _parse_embeddings(df["embeddings"])
    texts = df[text_field].fillna("").astype(str).tolist()
    stamp = datetime.datetime.now().strftime("%Y%m%d")
    out: List[Dict] = []
    for it in range(start, start + iters):
        for k in ntopics_centralized:
            name = f"centralized_{k}_{it}_{stamp}"
            logger.info("-- -- Training centralized model: %s", name)
            m = train_one(texts, k, params, os.path.join(models_folder, name), device, trainer, emb,
                          seed=it)
            out.append({"name": name, **m})
        for f in df[fos_name].unique():
            mask = (df[fos_name] == f).to_numpy()
            sub = [t for t, keep in zip(texts, mask) if keep]
            for k in (ntopics_nodes or ntopics_centralized):
                name = f"non_collaborative_{f}_{k}_{it}_{stamp}"
                logger.info("-- -- Training non-collaborative model: %s", name)
                m = train_one(sub, k, params, os.path.join(models_folder, name), device, trainer,
                              None if emb is None else emb[mask], seed=it)
                out.append({"name": name, "fos": str(f), **m})
    with open(os.path.join(models_folder, "summary.json"), "w") as fh:
        json.dump(out, fh, indent=2)
    return out


def main(argv=None):
    p = argparse.ArgumentParser(description="collaborative vs non-collaborative models")
    p.add_argument("--path_corpus", required=True)
    p.add_argument("--models_folder", required=True)
    p.add_argument("--trainer", default="avitm", choices=["avitm", "ctm"])
    p.add_argument("--iters", type=int, default=1)
    p.add_argument("--start", type=int, default=0)
    p.add_argument("--ntopics_nodes", type=str, default=None)
    p.add_argument("--ntopics_centralized", type=str, default="10,20,30,40,50")
    p.add_argument("--fos_name", type=str, default="fos")
    p.add_argument("--config", type=str, default=None, help="INI with the [ntms] parameters")
    p.add_argument("--device", type=str, default=None)
    a = p.parse_args(argv)
    logging.basicConfig(level="INFO")
    ks = [int(x) for x in a.ntopics_centralized.split(",")]
    kn = [int(x) for x in a.ntopics_nodes.split(",")] if a.ntopics_nodes else None
    return train(a.path_corpus, a.models_folder, ks, kn, a.iters, a.start, a.fos_name,
                 trainer=a.trainer, params=load_config(a.config).training_params, device=a.device)


if __name__ == "__main__":
    main()
