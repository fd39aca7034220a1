"""Topic-model wrapper: root models, hierarchical submodels (HTM-WS / HTM-DS), topic
coherence against a reference corpus, RBO and topic diversity.

Reference: src/aux_modules/tmWrapper/tm_wrapper.py:15-400.  The reference drives the
external topicmodeler (an empty git submodule in the reference tree) through
``python topicmodeling.py --preproc / --train / --hierarchical`` subprocesses and
reads its ``TMmodel`` folder back.  Here the trainers are this framework's models,
run in-process (the fused HIP engine on a GPU):

  trainer "avitm"  ProdLDA / NeuralLDA (``model_type`` of the parameters)
  trainer "ctm"    CombinedTM when the corpus has an ``embeddings`` column, else the
                   AVITM model of ``model_type``
  trainer "mallet" not available (no Java / Mallet in this stack): raises

Model folder (the topicmodeler layout the reference reads back, tm_wrapper.py:200-400):

  {model}/config.json           trainer, TMparam, hierarchy-level, htm-version,
                                expansion_tpc, thr (``_get_model_config``)
  {model}/corpus.parquet        training corpus (root: the given corpus; submodel: derived)
  {model}/TMmodel/betas.npy     [K, V] topic-word distributions
  {model}/TMmodel/thetas.npz    [D, K] sparse doc-topic matrix (3e-3 threshold, L1)
  {model}/TMmodel/alphas.npy    [K] mean document-topic proportion
  {model}/TMmodel/vocab.txt     the model vocabulary, one term per line
  {model}/TMmodel/tpc_descriptions.txt   top words of every topic, one line per topic
  {model}/TMmodel/topic_coherence.npy    NPMI of every topic on the training corpus
  {model}/TMmodel/{new_topic_coherence,rbo,td}.npy   written by ``calculate_*``

Hierarchical submodels (the topicmodeler's ``--hierarchical`` step) expand topic
``e`` of a father model:

  HTM-WS (word selection): every token of word w in document d is assigned to topic k
      with probability theta_dk beta_kw / sum_j theta_dj beta_jw; the submodel corpus
      keeps, per document, the tokens assigned to e (Binomial(count, p) per CSR
      non-zero, drawn on the device); documents left empty are dropped.
  HTM-DS (document selection): the documents with theta_de > thr, all their tokens.
"""
from __future__ import annotations

import json
import logging
import pathlib
import shutil
import time
from typing import Dict, List, Optional

import numpy as np
import scipy.sparse as sp
import torch

from ..data.vocab import local_vocabulary, vectorize
from ..eval.export import postprocess_thetas
from ..eval.metrics import inverted_rbo, npmi_coherence, topic_diversity
from ..utils.misc import mallet_corpus_to_df

# TMparam fields per trainer (tm_wrapper.py:_get_model_config); "avitm" uses the ctm list
CTM_FIELDS = ["ntopics", "thetas_thr", "labels", "model_type", "ctm_model_type", "hidden_sizes",
              "activation", "dropout_in", "dropout_out", "learn_priors", "lr", "momentum", "solver",
              "num_epochs", "reduce_on_plateau", "batch_size", "topic_prior_mean",
              "topic_prior_variance", "num_samples", "num_data_loader_workers", "contextual_size"]
MALLET_FIELDS = ["ntopics", "labels", "thetas_thr", "mallet_path", "alpha", "optimize_interval",
                 "num_threads", "num_iterations", "doc_topic_thr", "token_regexp"]
EXTRA_FIELDS = ["dropout", "n_components", "backend"]     # framework extras, kept when given


def read_corpus(path):
    """A training corpus as a DataFrame with a ``bow_text`` column: a parquet file or
    directory (``bow_text``, else ``text`` / ``lemmas``; optional ``embeddings``) or a
    Mallet import file (``<id> 0 <text>`` lines)."""
    import pandas as pd
    p = pathlib.Path(path)
    if p.is_dir() or p.suffix == ".parquet":
        df = pd.read_parquet(p)
    else:
        df = mallet_corpus_to_df(str(p))
    if "bow_text" not in df.columns:
        for alt in ("text", "lemmas"):
            if alt in df.columns:
                df = df.rename(columns={alt: "bow_text"})
                break
        else:
            raise ValueError(f"{path}: no bow_text / text / lemmas column")
    df["bow_text"] = df["bow_text"].fillna("").astype(str)
    return df.reset_index(drop=True)


def htm_ws_counts(X: sp.csr_matrix, thetas: np.ndarray, betas: np.ndarray, topic: int,
                  seed: int = 0, device=None, chunk: int = 1 << 20) -> sp.csr_matrix:
    """Tokens of every (d, w) non-zero of ``X`` assigned to ``topic``:
    Binomial(x_dw, theta_d,topic beta_topic,w / sum_k theta_dk beta_kw)."""
    X = X.tocsr()
    dev = torch.device(device) if device is not None else torch.device("cpu")
    th = torch.as_tensor(np.asarray(thetas, dtype=np.float32), device=dev)
    be = torch.as_tensor(np.asarray(betas, dtype=np.float32), device=dev)
    rows = np.repeat(np.arange(X.shape[0], dtype=np.int64), np.diff(X.indptr))
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    out = np.empty(X.nnz, dtype=np.float32)
    for a in range(0, X.nnz, chunk):
        b = min(X.nnz, a + chunk)
        r = torch.as_tensor(rows[a:b], device=dev)
        c = torch.as_tensor(X.indices[a:b].astype(np.int64), device=dev)
        x = torch.as_tensor(X.data[a:b].astype(np.float32), device=dev)
        num = th[r, topic] * be[topic, c]
        den = (th[r] * be[:, c].t()).sum(1)
        p = torch.where(den > 0, num / den.clamp_min(1e-30), torch.zeros_like(num)).clamp(0, 1)
        out[a:b] = torch.binomial(x, p, generator=gen).cpu().numpy()
    res = sp.csr_matrix((out, X.indices.copy(), X.indptr.copy()), shape=X.shape)
    res.eliminate_zeros()
    return res


def counts_to_texts(X: sp.csr_matrix, terms: List[str]) -> List[str]:
    """Whitespace documents that re-vectorize to the counts of ``X``."""
    X = X.tocsr()
    out = []
    for d in range(X.shape[0]):
        s, e = X.indptr[d], X.indptr[d + 1]
        out.append(" ".join(" ".join([terms[w]] * int(c))
                            for w, c in zip(X.indices[s:e], X.data[s:e]) if c > 0))
    return out


def _bool(v) -> bool:
    return v if isinstance(v, bool) else str(v).strip().lower() in ("true", "1", "yes")


class TMWrapper:
    """Same entry points as the reference TMWrapper (tm_wrapper.py:15-400)."""

    def __init__(self, logger=None, device=None, seed: int = 0):
        self._logger = logger or logging.getLogger("TMWrapper")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda" if torch.cuda.is_available() else "cpu")
        self.seed = int(seed)

    # ------------------------------------------------------------------ config
    def _get_model_config(self, trainer: str, TMparam: dict, hierarchy_level: int,
                          htm_version: Optional[str], expansion_tpc: Optional[int],
                          thr: Optional[float]) -> dict:
        fields = (MALLET_FIELDS if trainer == "mallet" else CTM_FIELDS) + EXTRA_FIELDS
        return {"trainer": trainer,
                "TMparam": {t: TMparam[t] for t in fields if t in TMparam},
                "hierarchy-level": hierarchy_level, "htm-version": htm_version,
                "expansion_tpc": expansion_tpc, "thr": thr}

    def _fresh_dir(self, model_path: pathlib.Path) -> None:
        if model_path.exists():
            old = pathlib.Path(str(model_path) + "_old")
            if old.exists():
                shutil.rmtree(old)
            shutil.move(str(model_path), str(old))
            self._logger.info(f"-- -- Creating backup of existing model in {old}")
        model_path.mkdir(parents=True, exist_ok=True)

    # ------------------------------------------------------------------ training
    def _model_kwargs(self, p: Dict) -> Dict:
        tpv = p.get("topic_prior_variance")
        return dict(
            n_components=int(p.get("ntopics", p.get("n_components", 10))),
            model_type=str(p.get("model_type", "prodLDA")),
            hidden_sizes=tuple(int(h) for h in p.get("hidden_sizes", (100, 100))),
            activation=str(p.get("activation", "softplus")),
            dropout=float(p.get("dropout", p.get("dropout_in", 0.2))),
            learn_priors=_bool(p.get("learn_priors", True)),
            batch_size=int(p.get("batch_size", 64)), lr=float(p.get("lr", 2e-3)),
            momentum=float(p.get("momentum", 0.99)), solver=str(p.get("solver", "adam")),
            num_epochs=int(p.get("num_epochs", 100)),
            reduce_on_plateau=_bool(p.get("reduce_on_plateau", False)),
            topic_prior_mean=float(p.get("topic_prior_mean", 0.0)),
            topic_prior_variance=None if tpv in (None, "", "None") else float(tpv),
            num_samples=int(p.get("num_samples", 20)), verbose=False, device=self.device,
            seed=self.seed, backend=str(p.get("backend", "auto")))

    def _fit(self, df, cfg: Dict):
        from ..data.bow import BOWDataset, CTMDataset
        from ..models import AVITM, CombinedTM
        trainer = cfg["trainer"]
        if trainer == "mallet":
            raise NotImplementedError("the Mallet (Gibbs LDA) trainer is not available in this "
                                      "stack; use trainer='avitm' or 'ctm'")
        texts = df["bow_text"].tolist()
        vocab = local_vocabulary(texts)
        terms = sorted(vocab, key=vocab.get)
        X = vectorize(texts, vocab)
        id2tok = dict(enumerate(terms))
        kw = self._model_kwargs(cfg["TMparam"])
        torch.manual_seed(self.seed)
        if trainer == "ctm" and "embeddings" in df.columns:
            from ..federation.data import _parse_embeddings
            emb = _parse_embeddings(df["embeddings"])
            tm = CombinedTM(input_size=len(terms), contextual_size=emb.shape[1], **kw)
            ds = CTMDataset(emb, X, id2tok)
        else:
            tm = AVITM(input_size=len(terms), **kw)
            ds = BOWDataset(X, id2tok)
        tm.fit(ds, n_samples=1)
        return tm, ds, terms, X

    def _save_tmmodel(self, d: pathlib.Path, tm, ds, terms: List[str], X, n_samples: int,
                      thr: float) -> None:
        d.mkdir(parents=True, exist_ok=True)
        betas = tm.get_topic_word_distribution()
        thetas = postprocess_thetas(tm.get_doc_topic_distribution(ds, n_samples), thr)
        th = sp.csr_matrix(thetas.astype(np.float32))
        np.save(d / "betas.npy", betas)
        sp.save_npz(d / "thetas.npz", th)
        np.save(d / "alphas.npy", np.asarray(th.mean(axis=0)).ravel())
        (d / "vocab.txt").write_text("\n".join(terms) + "\n", encoding="utf-8")
        top = np.argsort(-betas, axis=1)
        (d / "tpc_descriptions.txt").write_text(
            "\n".join(", ".join(terms[i] for i in row[:15]) for row in top) + "\n", encoding="utf-8")
        coh = npmi_coherence(top[:, :10], X, per_topic=True, device=self.device)
        np.save(d / "topic_coherence.npy", np.asarray(coh))

    def _train_model(self, model_path: pathlib.Path) -> None:
        """Train the model described by ``model_path/config.json`` on
        ``model_path/corpus.parquet`` and write ``model_path/TMmodel``."""
        t0 = time.perf_counter()
        cfg = json.loads((model_path / "config.json").read_text(encoding="utf-8"))
        df = read_corpus(model_path / "corpus.parquet")
        if len(df) == 0:
            raise ValueError(f"{model_path}: empty training corpus")
        tm, ds, terms, X = self._fit(df, cfg)
        p = cfg["TMparam"]
        self._save_tmmodel(model_path / "TMmodel", tm, ds, terms, X,
                           int(p.get("num_samples", 20)), float(p.get("thetas_thr", 3e-3)))
        self._logger.info(f"Total training time --> {time.perf_counter() - t0}")

    # ------------------------------------------------------------------ preprocessing
    def preproc_corpus_tm(self, path_preproc, Dtset: str, TrDtset: dict, train_config: dict,
                          nw: int = 0) -> pathlib.Path:
        """Write the dataset / training configs (tm_wrapper.py:171-198) and preprocess:
        the lemmas of every dataset of ``TrDtset['Dtsets']`` through
        :class:`~gfedntm_amd.data.preprocess.CorpusPreprocessor` with the ``Preproc``
        parameters of ``train_config`` -> ``corpus.parquet`` + ``vocabulary.txt``."""
        import pandas as pd
        from ..data.preprocess import CorpusPreprocessor, load_wordlists
        path_preproc = pathlib.Path(path_preproc)
        path_preproc.mkdir(parents=True, exist_ok=True)
        (path_preproc / "stats").mkdir(parents=True, exist_ok=True)
        dts_cfg = path_preproc / Dtset
        dts_cfg.write_text(json.dumps(TrDtset, ensure_ascii=False, indent=2, default=str),
                           encoding="utf-8")
        train_config = dict(train_config)
        train_config["TrDtSet"] = dts_cfg.resolve().as_posix()
        (path_preproc / "trainconfig.json").write_text(
            json.dumps(train_config, ensure_ascii=False, indent=2, default=str), encoding="utf-8")
        pp = train_config.get("Preproc", {})
        frames = []
        for ds in TrDtset.get("Dtsets", []):
            df = pd.read_parquet(ds["parquet"])
            flds = ds.get("lemmasfld", ["lemmas"])
            flds = [flds] if isinstance(flds, str) else list(flds)
            text = df[flds].fillna("").astype(str).agg(" ".join, axis=1)
            frames.append(pd.DataFrame({"id": df[ds.get("idfld", "id")].astype(str)
                                        if ds.get("idfld", "id") in df.columns else df.index.astype(str),
                                        "raw": text, "source": ds.get("source", "")}))
        corpus = pd.concat(frames, ignore_index=True) if frames else pd.DataFrame(
            {"id": [], "raw": [], "source": []})
        stop, equiv = load_wordlists(list(pp.get("stopwords", [])) + list(pp.get("equivalences", [])))
        cp = CorpusPreprocessor(stop, equiv, int(pp.get("min_lemas", 15)), int(pp.get("no_below", 15)),
                                float(pp.get("no_above", 0.4)), int(pp.get("keep_n", 100000)))
        bow, keep = cp.fit_transform(corpus["raw"].tolist())
        out = corpus.loc[keep, ["id", "source"]].copy()
        out["bow_text"] = bow
        out.to_parquet(path_preproc / "corpus.parquet")
        (path_preproc / "vocabulary.txt").write_text("\n".join(cp.vocabulary) + "\n", encoding="utf-8")
        self._logger.info(f"-- -- Preprocessed {len(out)} of {len(corpus)} documents, "
                          f"vocabulary {len(cp.vocabulary)}")
        return path_preproc

    # ------------------------------------------------------------------ models
    def train_root_model(self, models_folder, name: str, path_corpus, trainer: str,
                         training_params: dict) -> pathlib.Path:
        """Root (level-0) model in ``models_folder/name`` (tm_wrapper.py:200-277)."""
        model_path = pathlib.Path(models_folder) / name
        corpus = pathlib.Path(path_corpus)
        if not corpus.exists():
            raise FileNotFoundError(f"The provided corpus file does not exist: {corpus}")
        self._fresh_dir(model_path)
        read_corpus(corpus).to_parquet(model_path / "corpus.parquet")
        cfg = self._get_model_config(trainer, training_params, 0, None, None, None)
        (model_path / "config.json").write_text(json.dumps(cfg, ensure_ascii=False, indent=2,
                                                           default=str), encoding="utf-8")
        self._train_model(model_path)
        return model_path

    def create_submodel_corpus(self, father_model_path, version: str, expansion_topic: int,
                               thr: Optional[float] = None):
        """The training corpus of an HTM submodel of ``father_model_path``."""
        father = pathlib.Path(father_model_path)
        tmd = father / "TMmodel"
        df = read_corpus(father / "corpus.parquet")
        thetas = sp.load_npz(tmd / "thetas.npz").toarray()
        if not 0 <= expansion_topic < thetas.shape[1]:
            raise ValueError(f"expansion topic {expansion_topic} out of range")
        v = version.upper()
        if v == "HTM-DS":
            if thr is None:
                raise ValueError("HTM-DS needs a document-selection threshold thr")
            sub = df.loc[thetas[:, expansion_topic] > thr].copy()
        elif v == "HTM-WS":
            terms = [t for t in (tmd / "vocab.txt").read_text(encoding="utf-8").split("\n") if t]
            X = vectorize(df["bow_text"].tolist(), {t: i for i, t in enumerate(terms)})
            betas = np.load(tmd / "betas.npy")
            kept = htm_ws_counts(X, thetas, betas, expansion_topic, seed=self.seed,
                                 device=self.device)
            texts = np.asarray(counts_to_texts(kept, terms), dtype=object)
            mask = np.diff(kept.indptr) > 0
            sub = df.loc[mask].copy()
            sub["bow_text"] = texts[mask]
        else:
            raise ValueError("version must be 'HTM-WS' or 'HTM-DS'")
        return sub.reset_index(drop=True)

    def train_htm_submodel(self, version: str, father_model_path, name: str, trainer: str,
                           training_params: dict, expansion_topic: int,
                           thr: Optional[float] = None) -> pathlib.Path:
        """Second-level model of ``father_model_path`` expanding ``expansion_topic``
        (tm_wrapper.py:279-356)."""
        father = pathlib.Path(father_model_path)
        model_path = father / name
        self._fresh_dir(model_path)
        cfg = self._get_model_config(trainer, training_params, 1, version, expansion_topic, thr)
        (model_path / "config.json").write_text(json.dumps(cfg, ensure_ascii=False, indent=2,
                                                           default=str), encoding="utf-8")
        sub = self.create_submodel_corpus(father, version, expansion_topic, thr)
        self._logger.info(f"-- -- {version} submodel corpus: {len(sub)} documents")
        sub.to_parquet(model_path / "corpus.parquet")
        self._train_model(model_path)
        return model_path

    # ------------------------------------------------------------------ metrics
    def _topic_words(self, model_path, n: int) -> List[List[str]]:
        tmd = pathlib.Path(model_path) / "TMmodel"
        terms = [t for t in (tmd / "vocab.txt").read_text(encoding="utf-8").split("\n") if t]
        top = np.argsort(-np.load(tmd / "betas.npy"), axis=1)[:, :n]
        return [[terms[i] for i in row] for row in top]

    def calculate_cohr_vs_ref(self, model_path, corpus_val) -> np.ndarray:
        """NPMI of every topic (top-10 words) on a reference corpus (Mallet file or
        parquet); saved as ``TMmodel/new_topic_coherence.npy`` (tm_wrapper.py:358-384)."""
        tmd = pathlib.Path(model_path) / "TMmodel"
        terms = [t for t in (tmd / "vocab.txt").read_text(encoding="utf-8").split("\n") if t]
        ref = read_corpus(corpus_val)
        X = vectorize(ref["bow_text"].tolist(), {t: i for i, t in enumerate(terms)})
        top = np.argsort(-np.load(tmd / "betas.npy"), axis=1)[:, :10]
        cohr = np.asarray(npmi_coherence(top, X, per_topic=True, device=self.device))
        np.save(tmd / "new_topic_coherence.npy", cohr)
        return cohr

    def calculate_rbo(self, model_path) -> float:
        """Inverted rank-biased overlap of the topics' top-10 words (tm_wrapper.py:386-392)."""
        rbo = inverted_rbo(self._topic_words(model_path, 10), topk=10)
        np.save(pathlib.Path(model_path) / "TMmodel" / "rbo.npy", np.asarray(rbo))
        return rbo

    def calculate_td(self, model_path) -> float:
        """Topic diversity of the topics' top-25 words (tm_wrapper.py:394-400)."""
        td = topic_diversity(self._topic_words(model_path, 25), topk=25)
        np.save(pathlib.Path(model_path) / "TMmodel" / "td.npy", np.asarray(td))
        return td
