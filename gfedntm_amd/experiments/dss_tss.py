"""DSS / TSS simulation on synthetic LDA/ProdLDA corpora.

Reference: experiments/dss_tss/run_simulation.py:358-739 (+ config/*/config.json).
Per iteration: one synthetic generation (per-node asymmetric Dirichlet priors,
``frozen_topics`` shared topics); models are trained on the first ``n_docs``
documents of each node and evaluated on the next ``n_docs_global_inf``:

  centralized  one ProdLDA on the union of all nodes' training documents
  non_colab    one ProdLDA per node on its own documents (scores averaged)
  baseline     TSS of an independent random topic matrix; DSS of independently
               drawn document-topic proportions
  federated    (new: the reference simulator has no federated arm) the nodes as
               federation clients -- per-minibatch sample-weighted FedAvg,
               LocalFederation on one device

  federated_matched  (new) the same federation run for as many rounds as the
               centralized model takes optimizer steps (equal update budget)
  federated_grads    (new) the nodes as clients of classic synchronous data
               parallelism (``agg="grads"``: the sample-weighted gradient average, one
               optimizer step per round on every replica) -- not the reference protocol
  federated_bf16delta (new) the federated arm over the opt-in reduced-byte FedAvg wire
               (``fedavg_wire="bf16delta"``: bf16 departures from the last average)

TSS = sum over true topics of the best Bhattacharyya coefficient with a learned
topic (learned betas re-indexed onto the generator vocabulary).  With
``reference_tss`` (default on) the betas go through the reference simulator's
softmax chain: ``get_topic_word_distribution()`` is already softmax(beta), the
simulator applies ``softmax`` again (run_simulation.py:417, :469) and its
``convert_topic_word_to_init_size`` a third time (run_simulation.py:257) before
the re-indexing + L1 normalisation, and that re-indexing shifts every word by one
column (:func:`_reference_reindex`) -- the resulting, nearly uniform and shifted,
topics are what the published TSS numbers (8.679 centralized at eta=0.01)
measure.  ``reference_tss=False`` scores softmax(beta) on the correct columns.  DSS = mean
absolute difference of the documents' Bhattacharyya similarity matrices, true
vs inferred.  ``experiment`` 0 sweeps ``frozen_topics_list``, 1 sweeps
``eta_list`` (the topic Dirichlet parameter beta).  Results: ``results.json`` and
``results.csv`` (mean / std over ``iters``) instead of a pickled DataFrame.

Usage: ``python -m gfedntm_amd.experiments.dss_tss --config cfg.json --out results/``
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import time
from typing import Dict, List

import numpy as np
import scipy.sparse as sp
import torch

from ..data.bow import BOWDataset
from ..data.synthetic import SyntheticCorpus, generate_synthetic, node_priors
from ..eval.metrics import betas_to_ground_truth_vocab, dss, tss

DEFAULTS = dict(n_nodes=5, vocab_size=5000, n_topics=50, beta=1e-2, alpha=0.1, n_docs=10000,
                n_docs_inf=1000, n_docs_global_inf=1000, nwords={"min_words": 150, "max_words": 250},
                alg="lda", frozen_topics=5, frozen_topics_list="5 10 15 20 25 30 35 40",
                eta_list="1e-2 0.02 0.03 0.04 0.08 1", experiment=1, iters=20,
                # model (run_simulation.py:271-318)
                hidden_sizes=[100, 100], num_epochs=100, batch_size=64, lr=2e-3,
                # new
                federated=True, device=None, backend="auto", seed=0, arms=None,
                reference_tss=True)

ARMS = ("centralized", "non_colab", "baseline", "federated", "federated_matched",
        "federated_grads", "federated_bf16delta")


def _vocab_of(counts: sp.csr_matrix):
    cols = np.unique(counts.indices)
    terms = sorted(f"wd{j}" for j in cols)            # CountVectorizer order
    return terms, {t: i for i, t in enumerate(terms)}


def _remap(counts: sp.csr_matrix, vocab: Dict[str, int]) -> sp.csr_matrix:
    """Re-index generator columns onto ``vocab`` (columns outside it dropped)."""
    m = counts.tocoo()
    cmap = np.full(counts.shape[1], -1, dtype=np.int64)
    for j in np.unique(m.col):
        cmap[j] = vocab.get(f"wd{j}", -1)
    keep = cmap[m.col] >= 0
    out = sp.csr_matrix((m.data[keep], (m.row[keep], cmap[m.col][keep])),
                        shape=(counts.shape[0], len(vocab)), dtype=np.float32)
    out.sort_indices()
    return out


def _model_kw(cfg, input_size, device):
    return dict(input_size=input_size, n_components=cfg["n_topics"], model_type="prodLDA",
                hidden_sizes=tuple(cfg["hidden_sizes"]), activation="softplus", dropout=0.2,
                learn_priors=True, batch_size=cfg["batch_size"], lr=cfg["lr"], momentum=0.99,
                solver="adam", num_epochs=cfg["num_epochs"], reduce_on_plateau=False,
                topic_prior_mean=0.0, topic_prior_variance=None, num_samples=20,
                verbose=False, backend=cfg["backend"], device=device)


def train_and_score(cfg, train_counts: sp.csr_matrix, inf_counts: sp.csr_matrix,
                    topic_vectors: np.ndarray, inf_thetas: np.ndarray, device, seed: int):
    """Train one ProdLDA (75/25 train/validation split, early stopping like the
    reference's prepare_dataset + fit) and return (TSS, DSS)."""
    from sklearn.model_selection import train_test_split

    from ..models import AVITM
    tr, va = train_test_split(np.arange(train_counts.shape[0]), test_size=0.25, random_state=42)
    terms, vocab = _vocab_of(train_counts[tr])
    id2token = dict(enumerate(terms))
    torch.manual_seed(seed)
    tm = AVITM(**_model_kw(cfg, len(terms), device))
    tm.fit(BOWDataset(_remap(train_counts[tr], vocab), id2token),
           BOWDataset(_remap(train_counts[va], vocab), id2token))
    return _score(tm, id2token, vocab, cfg, inf_counts, topic_vectors, inf_thetas)


def _softmax_rows(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    e = np.exp(x - x.max(axis=1, keepdims=True))
    return e / e.sum(axis=1, keepdims=True)


def _reference_reindex(wd: np.ndarray, id2token: Dict[int, str], vocab_size: int) -> np.ndarray:
    """The reference simulator's re-indexing, defect included: its documents name
    generator column j 'wd<j>' (run_simulation.py:174) but the lookup list is
    ``all_words = ['wd1' .. 'wd<V>']`` (run_simulation.py:418-420), so token 'wd<j>'
    lands in column j - 1 and 'wd0' is dropped -- every learned topic is compared
    with the ground truth shifted by one word."""
    out = np.zeros((wd.shape[0], vocab_size), dtype=np.float64)
    src = [i for i in range(wd.shape[1]) if int(id2token[i][2:]) >= 1]
    cols = np.array([int(id2token[i][2:]) - 1 for i in src], dtype=np.int64)
    out[:, cols] = wd[:, src]
    s = out.sum(axis=1, keepdims=True)
    s[s == 0] = 1.0
    return out / s


def _score(tm, id2token, vocab, cfg, inf_counts, topic_vectors, inf_thetas):
    wd = tm.get_topic_word_distribution()                  # softmax(beta)
    # the TSS of the learned topic-word distribution on the right columns ...
    true_tss = tss(betas_to_ground_truth_vocab(wd, id2token, cfg["vocab_size"]), topic_vectors)
    if cfg.get("reference_tss", True):
        # ... and the number the reference simulator would print for the same model
        wd = _softmax_rows(_softmax_rows(wd))              # run_simulation.py:417 + :257
        betas = _reference_reindex(wd, id2token, cfg["vocab_size"])
    else:
        betas = betas_to_ground_truth_vocab(wd, id2token, cfg["vocab_size"])
    thetas = np.asarray(tm.get_doc_topic_distribution(BOWDataset(_remap(inf_counts, vocab),
                                                                 id2token)))
    return tss(betas, topic_vectors), dss(inf_thetas, thetas), true_tss


def run_iteration(cfg, frozen_topics: int, eta: float, device, seed: int) -> Dict[str, tuple]:
    arms = cfg.get("arms") or [a for a in ARMS
                               if not a.startswith("federated") or cfg["federated"]]
    n_nodes, K, V = cfg["n_nodes"], cfg["n_topics"], cfg["vocab_size"]
    n_tr, n_inf = cfg["n_docs"], cfg["n_docs_global_inf"]
    nw = cfg["nwords"]
    nwords = (nw["min_words"], nw["max_words"]) if isinstance(nw, dict) else tuple(nw)
    sc = generate_synthetic(vocab_size=V, n_topics=K, beta=eta, alpha=cfg["alpha"],
                            n_docs=n_tr + max(cfg["n_docs_inf"], n_inf), nwords=nwords,
                            n_nodes=n_nodes, frozen_topics=frozen_topics, alg=cfg["alg"], seed=seed)
    train = [c[:n_tr] for c in sc.counts]
    inf_counts = sp.vstack([c[n_tr:n_tr + n_inf] for c in sc.counts]).tocsr()
    inf_thetas = np.concatenate([t[n_tr:n_tr + n_inf] for t in sc.doc_topics])
    out: Dict[str, tuple] = {}
    log = logging.getLogger("gfedntm_amd.dss_tss")
    t0 = time.perf_counter()

    def done(arm):
        log.info("  %-18s TSS %.3f DSS %.1f (TSS of softmax(beta) on the right columns "
                 "%.3f) (%.1f s)", arm, out[arm][0], out[arm][1], out[arm][2],
                 time.perf_counter() - t0)
    if "baseline" in arms:
        rng = np.random.default_rng(seed + 7)
        rand_topics = rng.dirichlet(V * [eta], K)
        priors = node_priors(K, n_nodes, frozen_topics, cfg["alpha"])
        rand_thetas = np.concatenate([rng.dirichlet(p, n_inf) for p in priors])
        t = tss(rand_topics, sc.topic_vectors)
        out["baseline"] = (t, dss(inf_thetas, rand_thetas), t)
        done("baseline")
    if "centralized" in arms:
        out["centralized"] = train_and_score(cfg, sp.vstack(train).tocsr(), inf_counts,
                                             sc.topic_vectors, inf_thetas, device, seed)
        done("centralized")
    if "non_colab" in arms:
        s = [train_and_score(cfg, c, inf_counts, sc.topic_vectors, inf_thetas, device, seed + i)
             for i, c in enumerate(train)]
        out["non_colab"] = tuple(float(np.mean([r[j] for r in s])) for j in range(3))
        done("non_colab")
    if "federated" in arms:
        out["federated"] = _federated(cfg, sc, train, inf_counts, inf_thetas, device, seed)
        done("federated")
    if "federated_matched" in arms:
        # as many rounds as the centralized fit's optimizer steps (75 % train split)
        n_central = int(0.75 * sum(c.shape[0] for c in train))
        rounds = cfg["num_epochs"] * -(-n_central // cfg["batch_size"])
        out["federated_matched"] = _federated(cfg, sc, train, inf_counts, inf_thetas, device,
                                              seed, rounds=rounds)
        done("federated_matched")
    if "federated_grads" in arms:
        out["federated_grads"] = _federated(cfg, sc, train, inf_counts, inf_thetas, device, seed,
                                            agg="grads")
        done("federated_grads")
    if "federated_bf16delta" in arms:
        out["federated_bf16delta"] = _federated(cfg, sc, train, inf_counts, inf_thetas, device,
                                                seed, wire="bf16delta")
        done("federated_bf16delta")
    return out


def _federated(cfg, sc, train, inf_counts, inf_thetas, device, seed, rounds=None,
               agg: str = "params", wire: str = "fp32"):
    from ..federation.data import ClientCorpus
    from ..federation.runner import LocalFederation
    sub = SyntheticCorpus(sc.topic_vectors, [t[: c.shape[0]] for t, c in zip(sc.doc_topics, train)],
                          train, sc.n_nodes, sc.vocab_size, sc.n_topics, sc.frozen_topics,
                          sc.beta, sc.alpha, train[0].shape[0], sc.nwords)
    corpora = [ClientCorpus(synthetic=sub, node=i) for i in range(sc.n_nodes)]
    params = {k: v for k, v in _model_kw(cfg, 0, device).items()
              if k not in ("input_size", "verbose", "backend", "device")}
    steps_per_epoch = -(-max(c.shape[0] for c in train) // cfg["batch_size"])
    if rounds is None:
        rounds = cfg["num_epochs"] * steps_per_epoch
    params["num_epochs"] = -(-rounds // steps_per_epoch)
    fed = LocalFederation(corpora, params, max_iters=rounds, device=device,
                          backend=cfg["backend"], seed=seed, agg=agg, fedavg_wire=wire)
    fed.run()
    logging.getLogger("gfedntm_amd.dss_tss").info(
        "  federated round: %s, FedAvg %s", "batched launches" if fed._batched is not None
        else "per-client steps", fed.fold_plan or fed.agg.__class__.__name__)
    tm = fed.clients[0].tm                     # every client holds the averaged state
    id2token = dict(enumerate(fed.terms))
    return _score(tm, id2token, fed.vocab, cfg, inf_counts, sc.topic_vectors, inf_thetas)


def run(cfg: Dict, out_dir: str, logger=None) -> Dict:
    logger = logger or logging.getLogger("gfedntm_amd.dss_tss")
    c = dict(DEFAULTS)
    c.update(cfg)
    device = c["device"] or ("cuda" if torch.cuda.is_available() else "cpu")
    if int(c["experiment"]) == 0:
        sweep = [int(x) for x in str(c["frozen_topics_list"]).split()]
        points = [(f, c["beta"]) for f in sweep]
        index_name = "frozen_topics"
    else:
        sweep = [float(x) for x in str(c["eta_list"]).split()]
        frozen = [int(x) for x in str(c["frozen_topics_list"]).split()]
        f = frozen[1] if len(frozen) > 1 else c["frozen_topics"]   # as the reference does
        points = [(f, e) for e in sweep]
        index_name = "eta"
    rows: List[Dict] = []
    for (frozen, eta), x in zip(points, sweep):
        acc: Dict[str, List[tuple]] = {}
        for it in range(int(c["iters"])):
            logger.info("%s=%s iteration %d", index_name, x, it)
            res = run_iteration(c, frozen, eta, device, seed=int(c["seed"]) + 1000 * it)
            for k, v in res.items():
                acc.setdefault(k, []).append(v)
        row = {index_name: x}
        for k, vals in acc.items():
            a = np.asarray(vals, dtype=np.float64)
            row.update({f"{k}_betas_mean": a[:, 0].mean(), f"{k}_betas_std": a[:, 0].std(),
                        f"{k}_thetas_mean": a[:, 1].mean(), f"{k}_thetas_std": a[:, 1].std(),
                        f"{k}_tss_true_mean": a[:, 2].mean(), f"{k}_tss_true_std": a[:, 2].std()})
        rows.append(row)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "results.json"), "w") as f:
        json.dump({"config": c, "index": index_name, "rows": rows}, f, indent=2, default=str)
    import pandas as pd
    pd.DataFrame(rows).set_index(index_name).to_csv(os.path.join(out_dir, "results.csv"))
    return {"index": index_name, "rows": rows}


def main(argv=None):
    p = argparse.ArgumentParser(description="DSS / TSS simulation")
    p.add_argument("--config", required=True, help="config.json (reference schema + extras)")
    p.add_argument("--out", required=True, help="results folder")
    p.add_argument("--iters", type=int, default=None, help="override the config's iters")
    a = p.parse_args(argv)
    logging.basicConfig(level="INFO")
    with open(a.config, encoding="utf8") as f:
        cfg = json.load(f)
    if a.iters is not None:
        cfg["iters"] = a.iters
    return run(cfg, a.out)


if __name__ == "__main__":
    main()
