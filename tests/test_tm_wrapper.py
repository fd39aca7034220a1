"""TMWrapper (reference src/aux_modules/tmWrapper/tm_wrapper.py): root models, HTM-WS /
HTM-DS submodels, preprocessing configs, coherence vs a reference corpus, RBO, TD
(tiny CPU runs)."""
import json

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sp

from gfedntm_amd.experiments.tm_wrapper import TMWrapper, counts_to_texts, htm_ws_counts
from gfedntm_amd.utils import misc

WORDS = ("alpha beta gamma delta epsilon zeta eta theta iota kappa lambda omicron sigma "
         "tau upsilon omega river mountain forest ocean").split()


def _docs(n, seed):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, size=rng.integers(10, 25))) for _ in range(n)]


def _params(k=3):
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(ntopics=k, num_epochs=2, batch_size=16, hidden_sizes=(16, 16), backend="torch",
             num_samples=4)
    return p


def test_htm_ws_counts_extremes():
    X = sp.csr_matrix(np.array([[2, 0, 3], [1, 4, 0]], dtype=np.float32))
    th = np.array([[1.0, 0.0], [0.0, 1.0]])
    be = np.full((2, 3), 1 / 3)
    out = htm_ws_counts(X, th, be, topic=0, seed=0)
    assert np.array_equal(out.toarray(), [[2, 0, 3], [0, 0, 0]])
    # p = 1/2 everywhere: Binomial(40, 1/2) per non-zero
    X = sp.csr_matrix(np.full((200, 5), 40, dtype=np.float32))
    out = htm_ws_counts(X, np.full((200, 2), 0.5), np.full((2, 5), 0.2), 0, seed=1).toarray()
    assert abs(out.mean() - 20) < 0.5 and out.max() <= 40
    texts = counts_to_texts(sp.csr_matrix(np.array([[2, 0, 1]], dtype=np.float32)), ["a", "b", "c"])
    assert texts == ["a a c"]


def test_root_submodels_and_metrics(tmp_path):
    pq = tmp_path / "corpus.parquet"
    pd.DataFrame({"id": range(60), "bow_text": _docs(60, 0)}).to_parquet(pq)
    w = TMWrapper(device="cpu")
    root = w.train_root_model(str(tmp_path / "models"), "root", str(pq), "avitm", _params())
    tmd = root / "TMmodel"
    betas, thetas = np.load(tmd / "betas.npy"), sp.load_npz(tmd / "thetas.npz")
    assert betas.shape[0] == 3 and np.allclose(betas.sum(1), 1, atol=1e-5)
    assert thetas.shape == (60, 3) and np.allclose(thetas.sum(1), 1, atol=1e-5)
    vocab = (tmd / "vocab.txt").read_text().split()
    assert len(vocab) == betas.shape[1] and set(vocab) <= set(WORDS)
    assert len((tmd / "tpc_descriptions.txt").read_text().strip().split("\n")) == 3
    assert np.load(tmd / "topic_coherence.npy").shape == (3,)
    cfg = json.loads((root / "config.json").read_text())
    assert cfg["hierarchy-level"] == 0 and cfg["TMparam"]["ntopics"] == 3 and cfg["trainer"] == "avitm"

    # retraining into the same folder keeps a backup (tm_wrapper.py:238-246)
    w.train_root_model(str(tmp_path / "models"), "root", str(pq), "avitm", _params())
    assert (tmp_path / "models" / "root_old" / "TMmodel" / "betas.npy").exists()

    th = thetas.toarray()
    thr = 0.05
    ds = w.train_htm_submodel("HTM-DS", root, "sub_ds", "avitm", _params(2), expansion_topic=1, thr=thr)
    assert len(pd.read_parquet(ds / "corpus.parquet")) == int((th[:, 1] > thr).sum())
    ws = w.train_htm_submodel("HTM-WS", root, "sub_ws", "avitm", _params(2), expansion_topic=0)
    sub = pd.read_parquet(ws / "corpus.parquet")
    assert 0 < len(sub) <= 60
    orig = pd.read_parquet(root / "corpus.parquet").set_index("id")["bow_text"]
    for i, t in zip(sub["id"], sub["bow_text"]):         # a token subset of the father document
        have = pd.Series(orig[i].split()).value_counts()
        for wd, c in pd.Series(t.split()).value_counts().items():
            assert have.get(wd, 0) >= c
    for s in (ds, ws):
        c = json.loads((s / "config.json").read_text())
        assert c["hierarchy-level"] == 1 and (s / "TMmodel" / "betas.npy").exists()
    assert json.loads((ds / "config.json").read_text())["thr"] == thr

    val = tmp_path / "val.txt"
    misc.corpus_df_to_mallet(pd.DataFrame({"id": range(20), "text": _docs(20, 9)}), str(val))
    coh = w.calculate_cohr_vs_ref(root, val)
    assert coh.shape == (3,) and np.all(np.isfinite(coh))
    assert 0 <= w.calculate_td(root) <= 1 and (tmd / "td.npy").exists()
    assert np.isfinite(w.calculate_rbo(root)) and (tmd / "rbo.npy").exists()
    with pytest.raises(ValueError):
        w.train_htm_submodel("HTM-XX", root, "bad", "avitm", _params(), 0)
    with pytest.raises(NotImplementedError):
        w.train_root_model(str(tmp_path / "models"), "m", str(pq), "mallet", _params())


def test_preproc_corpus_tm(tmp_path):
    raw = tmp_path / "raw.parquet"
    pd.DataFrame({"corpusid": range(30), "lemmas": _docs(30, 3)}).to_parquet(raw)
    sw = tmp_path / "sw.json"
    sw.write_text(json.dumps({"name": "sw", "valid_for": "stopwords", "wordlist": ["alpha", "beta"]}))
    TrDtset = {"name": "tiny", "Dtsets": [{"parquet": str(raw), "source": "s2", "idfld": "corpusid",
                                           "lemmasfld": ["lemmas"], "filter": ""}]}
    cfg = {"name": "tiny", "trainer": "ctm",
           "Preproc": {"min_lemas": 5, "no_below": 2, "no_above": 0.9, "keep_n": 100,
                       "stopwords": [str(sw)], "equivalences": []}}
    out = TMWrapper(device="cpu").preproc_corpus_tm(tmp_path / "pp", "tiny.json", TrDtset, cfg, 2)
    df = pd.read_parquet(out / "corpus.parquet")
    voc = (out / "vocabulary.txt").read_text().split()
    assert len(df) > 0 and "alpha" not in voc and "beta" not in voc
    assert json.loads((out / "trainconfig.json").read_text())["TrDtSet"].endswith("tiny.json")
