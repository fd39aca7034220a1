"""Vocabulary consensus, synthetic generator, CSR datasets and the batch plan."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from gfedntm_amd.data.bow import BatchPlan, BOWDataset, CTMDataset, DeviceCSR
from gfedntm_amd.data.synthetic import (SyntheticCorpus, generate_synthetic, node_priors,
                                        node_vocabulary_terms, remap_to_vocabulary, rotate_left)
from gfedntm_amd.data.vocab import local_vocabulary, union_vocabulary, vectorize, vocabulary_dict


def test_local_vocabulary_matches_countvectorizer():
    from sklearn.feature_extraction.text import CountVectorizer
    texts = ["The quick brown fox jumps over the lazy dog", "A dog and a cat, the CAT!",
             "x y zz zzz 42 4 über naïve café"]
    cv = CountVectorizer(input="content", lowercase=True, stop_words="english").fit(texts)
    assert local_vocabulary(texts) == {k: int(v) for k, v in cv.vocabulary_.items()}


def test_union_and_vectorize():
    a, b = ["dog", "cat", "zebra"], ["ant", "dog"]
    terms = union_vocabulary([a, b])
    assert terms == sorted(set(a) | set(b))
    voc = vocabulary_dict(terms)
    m = vectorize(["dog dog cat", "ant zebra unknownword"], voc)
    assert isinstance(m, sp.csr_matrix) and m.dtype == np.float32
    assert m[0, voc["dog"]] == 2 and m[0, voc["cat"]] == 1 and m[1, voc["ant"]] == 1
    assert m.sum() == 5


def test_node_priors_rotation():
    pri = node_priors(10, 2, 2, 0.1)
    own = (10 - 2) // 2
    assert all(np.allclose(p[:2], 0.1) for p in pri)
    assert np.allclose(pri[0][2:2 + own], 0.1) and np.allclose(pri[0][2 + own:], 1e-5)
    assert list(pri[1][2:]) == rotate_left(list(pri[0][2:]), own)


def test_synthetic_shapes_and_remap(tmp_path):
    c = generate_synthetic(vocab_size=200, n_topics=6, n_docs=40, n_nodes=3, frozen_topics=2,
                           nwords=(20, 30), seed=3)
    assert c.topic_vectors.shape == (6, 200) and np.allclose(c.topic_vectors.sum(1), 1)
    lens = np.asarray(c.counts[0].sum(1)).ravel()
    assert lens.min() >= 20 and lens.max() < 30
    terms = union_vocabulary([node_vocabulary_terms(c, i) for i in range(3)])
    voc = vocabulary_dict(terms)
    X = remap_to_vocabulary(c, 1, voc)
    # remap == re-vectorising the token texts with the global vocabulary
    ref = vectorize(c.texts(1), voc)
    assert (X != ref).nnz == 0
    p = str(tmp_path / "s.npz")
    c.save_counts_npz(p)
    d = SyntheticCorpus.load_counts_npz(p)
    assert (d.counts[2] != c.counts[2]).nnz == 0 and np.allclose(d.topic_vectors, c.topic_vectors)


def test_batch_plan_semantics():
    plan = BatchPlan.build(n_docs=10, batch_size=4, n_steps=7, seed=0)
    # 3 batches per epoch (4, 4, 2), drop_last=False, epoch ends flagged
    assert plan.size.tolist() == [4, 4, 2, 4, 4, 2, 4]
    assert plan.epoch_end.tolist() == [False, False, True, False, False, True, False]
    ep0 = np.concatenate([plan.batch(s) for s in range(3)])
    assert sorted(ep0.tolist()) == list(range(10))
    ep1 = np.concatenate([plan.batch(s) for s in range(3, 6)])
    assert sorted(ep1.tolist()) == list(range(10)) and not np.array_equal(ep0, ep1)


def test_datasets_and_device_csr():
    X = sp.random(12, 30, density=0.2, format="csr", dtype=np.float32, random_state=0)
    ds = BOWDataset(X, {i: f"w{i}" for i in range(30)})
    assert len(ds) == 12 and torch.allclose(ds[3]["X"], torch.from_numpy(X[3].toarray()[0]))
    emb = np.random.default_rng(0).normal(size=(12, 5)).astype(np.float32)
    cds = CTMDataset(emb, X, {i: f"w{i}" for i in range(30)})
    item = cds[2]
    assert item["X_contextual"].shape == (5,) and item["X_bow"].shape == (30,)
    d = DeviceCSR(X, "cpu")
    rows = d.dense_rows(torch.tensor([0, 5, 11]))
    assert torch.allclose(rows, torch.from_numpy(X[[0, 5, 11]].toarray()))
    with pytest.raises(Exception):
        CTMDataset(emb[:5], X, {})
