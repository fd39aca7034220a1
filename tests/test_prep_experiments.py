"""Dataset preparation, corpus preprocessing, Mallet helpers and the experiment
drivers (tiny CPU configurations)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from gfedntm_amd.data import prep
from gfedntm_amd.data.preprocess import CorpusPreprocessor, load_wordlists, preprocess_parquet
from gfedntm_amd.utils import misc

WORDS = ("alpha beta gamma delta epsilon zeta eta theta iota kappa lambda omicron sigma "
         "tau upsilon omega river mountain forest ocean").split()


def _docs(n=40, seed=0):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, size=rng.integers(8, 20))) for _ in range(n)]


def test_prepare_dataset_split_and_vocab():
    docs = [d.split() for d in _docs()]
    tr, va, n_in, id2token, docs_train, cv = prep.prepare_dataset(docs)
    assert len(tr) == 30 and len(va) == 10 and n_in == len(id2token) == tr.X.shape[1]
    from sklearn.model_selection import train_test_split
    exp_train, _ = train_test_split(docs, test_size=0.25, random_state=42)
    assert docs_train == exp_train
    # the vectorizer was fitted on the training split only
    from sklearn.feature_extraction.text import CountVectorizer
    ref = CountVectorizer(stop_words="english").fit([" ".join(d) for d in exp_train])
    assert list(ref.get_feature_names_out()) == [id2token[i] for i in range(n_in)]


def test_ctm_preparation_and_hold_out():
    docs = _docs(40)
    emb = np.random.default_rng(1).standard_normal((40, 8)).astype(np.float32)
    tr, va, n_in, id2token, qt, emb_tr, emb_all, _ = prep.prepare_ctm_dataset(docs, custom_embeddings=emb)
    assert tr.X_contextual.shape == (30, 8) and va.X_contextual.shape == (10, 8)
    assert va.X_bow.shape[1] == n_in
    ho = prep.prepare_hold_out_dataset(docs[:5], qt, embeddings_ho=emb[:5])
    assert ho.X_bow.shape == (5, n_in)
    with pytest.raises(RuntimeError):
        prep.prepare_ctm_dataset(docs, unpreprocessed_corpus=docs)      # no embedder offline
    tr2, *_ = prep.prepare_ctm_dataset(docs, unpreprocessed_corpus=docs,
                                       embedder=lambda t: np.ones((len(t), 4), np.float32))
    assert tr2.X_contextual.shape[1] == 4
    q = prep.TopicModelDataPreparation(embedder=lambda t: np.zeros((len(t), 3), np.float32))
    ds = q.fit(docs, docs, labels=["a", "b"] * 20)
    assert ds.labels.shape == (40, 2)


def test_get_bag_of_words_and_whitespace():
    bow = prep.get_bag_of_words([np.array([1, 2, 2]), np.array([0, 0]), np.array([3, None], dtype=object)], 5)
    assert bow.shape == (2, 5) and bow[0, 2] == 2 and bow[1, 3] == 1
    docs = ["The River, the forest!", "and the", "Ocean ocean river"]
    pre, raw, vocab = prep.WhiteSpacePreprocessing(docs, vocabulary_size=10).preprocess()
    assert pre == ["river forest", "ocean ocean river"] and raw == [docs[0], docs[2]]
    assert set(vocab) == {"river", "forest", "ocean"}


def test_corpus_preprocessor(tmp_path):
    sw = tmp_path / "sw.json"
    sw.write_text(json.dumps({"name": "s", "valid_for": "stopwords", "wordlist": ["omega"]}))
    eq = tmp_path / "eq.json"
    eq.write_text(json.dumps({"name": "e", "valid_for": "equivalences", "wordlist": ["tau:sigma"]}))
    stop, equiv = load_wordlists([str(sw), str(eq)])
    assert stop == {"omega"} and equiv == {"tau": "sigma"}
    docs = _docs(60, seed=3)
    pp = CorpusPreprocessor(stop, equiv, min_lemas=10, no_below=3, no_above=0.99, keep_n=12)
    bow, keep = pp.fit_transform(docs)
    assert len(bow) == keep.sum() and len(pp.vocabulary) <= 12
    assert all("omega" not in d.split() and "tau" not in d.split() for d in bow)
    df = pd.DataFrame({"id": range(60), "lemmas": docs, "fos": ["a", "b"] * 30})
    src = tmp_path / "c.parquet"
    df.to_parquet(src)
    from gfedntm_amd.experiments import text_preproc
    cfg = text_preproc.main(["--path_preproc", str(tmp_path / "pp"), "--parquetFile", str(src),
                             "--idfld", "id", "--wordlists", f"{sw},{eq}", "--min_lemas", "10",
                             "--no_below", "3"])
    out = pd.read_parquet(tmp_path / "pp" / "iter_0" / "corpus.parquet")
    assert "bow_text" in out.columns and len(out) == cfg["n_docs_out"]
    vocab = (tmp_path / "pp" / "iter_0" / "vocabulary.txt").read_text().split()
    assert len(vocab) == cfg["vocab_size"]


def test_mallet_roundtrip_and_typed_config(tmp_path):
    df = pd.DataFrame({"id": ["d1", "d2"], "text": ["a b c", "x 0 y"]})
    f = str(tmp_path / "corpus.txt")
    misc.corpus_df_to_mallet(df, f)
    back = misc.mallet_corpus_to_df(f)
    assert back["id"].tolist() == ["d1", "d2"] and back["text"].tolist() == ["a b c", "x 0 y"]
    ini = tmp_path / "e.cf"
    ini.write_text("[a]\nntopics = 7\nlr = 0.1\nhidden_sizes = (10,20)\nlearn_priors = True\n"
                   "labels = x\ntopic_prior_variance = 3\ntrainer = ctm\n")
    c = misc.read_config_experiments(str(ini))
    assert c == {"ntopics": 7, "lr": 0.1, "hidden_sizes": (10, 20), "learn_priors": True,
                 "labels": "", "topic_prior_variance": None, "trainer": "ctm"}


def test_dss_tss_simulation_tiny(tmp_path):
    from gfedntm_amd.experiments import dss_tss
    cfg = dict(n_nodes=2, vocab_size=150, n_topics=5, beta=0.05, alpha=0.5, n_docs=60,
               n_docs_inf=20, n_docs_global_inf=20, nwords={"min_words": 20, "max_words": 40},
               frozen_topics_list="1 3", experiment=0, iters=1, hidden_sizes=[16, 16],
               num_epochs=2, batch_size=16, device="cpu", backend="torch")
    res = dss_tss.run(cfg, str(tmp_path))
    assert [r["frozen_topics"] for r in res["rows"]] == [1, 3]
    for r in res["rows"]:
        for arm in ("centralized", "non_colab", "baseline", "federated", "federated_matched",
                    "federated_grads"):
            assert np.isfinite(r[f"{arm}_betas_mean"]) and np.isfinite(r[f"{arm}_thetas_mean"])
            assert 0 < r[f"{arm}_betas_mean"] <= cfg["n_topics"] + 1e-6
    assert os.path.exists(tmp_path / "results.csv")


def test_reference_tss_softmax_chain():
    """reference_tss: softmax(beta) (get_topic_word_distribution) -> softmax
    (run_simulation.py:417) -> softmax (run_simulation.py:257) -> the reference's
    one-off re-index onto 'wd1'..'wd<V>' + L1 normalisation, as a literal
    re-statement of the reference loop."""
    from scipy.special import softmax
    from gfedntm_amd.experiments import dss_tss
    from gfedntm_amd.eval.metrics import tss

    rng = np.random.default_rng(0)
    K, Vl, Vg = 4, 30, 50
    beta = rng.standard_normal((K, Vl)) * 3
    id2token = {i: f"wd{j}" for i, j in enumerate(sorted(rng.choice(Vg, Vl, replace=False)))}
    topic_vectors = rng.dirichlet([0.05] * Vg, K)

    class TM:
        def get_topic_word_distribution(self):
            return softmax(beta, axis=1)

        def get_doc_topic_distribution(self, ds):
            return np.full((2, K), 1.0 / K)

    betas = softmax(TM().get_topic_word_distribution(), axis=1)
    wd = softmax(betas, axis=1)
    all_words = ["wd" + str(w) for w in np.arange(Vg + 1) if w > 0]     # run_simulation.py:418
    ref = np.zeros((K, Vg))
    for i in range(K):
        for idx, word in id2token.items():
            for j in range(len(all_words)):
                if all_words[j] == word:
                    ref[i, j] = wd[i][idx]
                    break
    ref = ref / ref.sum(1, keepdims=True)
    cfg = dict(vocab_size=Vg, reference_tss=True)
    import scipy.sparse as sp
    inf = sp.csr_matrix(np.ones((2, Vl), dtype=np.float32))
    vocab = {t: i for i, t in id2token.items()}
    got_tss, _, _ = dss_tss._score(TM(), id2token, vocab, cfg, inf, topic_vectors,
                                np.full((2, K), 1.0 / K))
    assert abs(got_tss - tss(ref, topic_vectors)) < 1e-9


def test_collab_and_wmd(tmp_path):
    from gfedntm_amd.experiments import collab, wmd_eval
    docs = _docs(48, seed=5)
    pq = tmp_path / "corpus.parquet"
    pd.DataFrame({"bow_text": docs, "fos": ["cs", "bio", "eco"] * 16}).to_parquet(pq)
    from gfedntm_amd.utils.config import load_config
    params = dict(load_config().training_params)
    params.update(num_epochs=2, batch_size=16, hidden_sizes=(16, 16), backend="torch")
    out = collab.train(str(pq), str(tmp_path / "models"), [3], params=params, device="cpu")
    assert len(out) == 1 + 3
    for m in out:
        assert 0 < m["td"] <= 1 and np.isfinite(m["npmi"])
    rng = np.random.default_rng(0)
    vec = tmp_path / "vec.txt"
    vec.write_text(f"{len(WORDS)} 4\n" + "\n".join(
        w + " " + " ".join(f"{x:.4f}" for x in rng.standard_normal(4)) for w in WORDS))
    written = wmd_eval.wmd_tables(str(tmp_path / "models"), str(tmp_path / "wmd"),
                                  wmd_eval.load_vectors(str(vec)), [3], [5])
    assert len(written) == 1
    t = pd.read_csv(written[0], index_col=0)
    assert t.shape == (3, 4) and np.all(np.isfinite(t.to_numpy()))
    assert np.allclose(np.diag(t.to_numpy()[:, :3]), 0, atol=1e-6)   # a model vs itself
