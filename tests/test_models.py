"""Model parity with the reference: state_dict keys/shapes (wire compatibility),
loss math, training API, persistence."""
import numpy as np
import pytest
import torch

from gfedntm_amd.data.bow import BOWDataset, CTMDataset
from gfedntm_amd.models import AVITM, CombinedTM, ZeroShotTM
from gfedntm_amd.models.functional import avitm_loss_explicit
from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
from tests.helpers import random_csr, tiny_corpus

AVITM_KEYS = [
    ("prior_mean", (10,)), ("prior_variance", (10,)), ("beta", (10, 120)),
    ("inf_net.input_layer.weight", (50, 120)), ("inf_net.input_layer.bias", (50,)),
    ("inf_net.hiddens.l_0.0.weight", (50, 50)), ("inf_net.hiddens.l_0.0.bias", (50,)),
    ("inf_net.f_mu.weight", (10, 50)), ("inf_net.f_mu.bias", (10,)),
    ("inf_net.f_mu_batchnorm.running_mean", (10,)), ("inf_net.f_mu_batchnorm.running_var", (10,)),
    ("inf_net.f_mu_batchnorm.num_batches_tracked", ()),
    ("inf_net.f_sigma.weight", (10, 50)), ("inf_net.f_sigma.bias", (10,)),
    ("inf_net.f_sigma_batchnorm.running_mean", (10,)),
    ("inf_net.f_sigma_batchnorm.running_var", (10,)),
    ("inf_net.f_sigma_batchnorm.num_batches_tracked", ()),
    ("beta_batchnorm.running_mean", (120,)), ("beta_batchnorm.running_var", (120,)),
    ("beta_batchnorm.num_batches_tracked", ()),
]


def _avitm(**kw):
    base = dict(input_size=120, n_components=10, hidden_sizes=(50, 50), batch_size=16,
                verbose=False, backend="torch", device="cpu", seed=0)
    base.update(kw)
    return AVITM(**base)


def test_avitm_state_dict_matches_reference_layout():
    tm = _avitm()
    sd = tm.model.state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == AVITM_KEYS
    assert [k for k, _ in tm.model.named_parameters()][:3] == ["prior_mean", "prior_variance", "beta"]
    assert torch.allclose(sd["prior_variance"], torch.full((10,), 1 - 1 / 10))
    assert sd["inf_net.f_mu_batchnorm.num_batches_tracked"].dtype == torch.int64


def test_ctm_combined_layout():
    tm = CombinedTM(input_size=40, contextual_size=12, n_components=5, hidden_sizes=(8, 8),
                    verbose=False, backend="torch", device="cpu")
    sd = tm.model.state_dict()
    assert sd["inf_net.adapt_bert.weight"].shape == (40, 12)
    assert sd["inf_net.input_layer.weight"].shape == (8, 80)      # concat[BoW, adapt] = 2V


def test_loss_matches_explicit_oracle():
    tm = _avitm()
    m = tm.model
    m.train()
    m.inf_net.dropout_enc.p = 0.0
    m.drop_theta.p = 0.0
    m.reparameterize = lambda mu, lv: mu
    x = torch.from_numpy(random_csr(16, 120, 10, seed=1).toarray())
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    pm, pv, mu, var, logvar, wd = m(x)
    loss_mod = (kl_terms(pm, pv, mu, var, logvar, 10) + reconstruction_terms(x, wd)).sum()
    m.load_state_dict(sd)
    loss_fun, _, _ = avitm_loss_explicit(m, x, torch.zeros(16, 10), torch.ones(16, 50),
                                         torch.ones(16, 10))
    torch.testing.assert_close(loss_mod, loss_fun, rtol=1e-5, atol=1e-4)


def test_kl_formula():
    pm, pv = torch.zeros(3), torch.full((3,), 0.5)
    mu = torch.tensor([[0.1, -0.2, 0.3]])
    lv = torch.tensor([[0.0, -1.0, 0.5]])
    kl = kl_terms(pm, pv, mu, lv.exp(), lv, 3)
    ref = 0.5 * ((lv.exp() / pv).sum() + ((pm - mu) ** 2 / pv).sum() - 3 + pv.log().sum() - lv.sum())
    torch.testing.assert_close(kl[0], ref)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_fit_and_inference_api(model_type, tmp_path):
    c, terms, shards = tiny_corpus(V=150, K=6, n_docs=60, n_nodes=1)
    ds = BOWDataset(shards[0], {i: t for i, t in enumerate(terms)})
    tm = AVITM(input_size=len(terms), n_components=6, model_type=model_type, hidden_sizes=(20, 20),
               batch_size=16, num_epochs=2, verbose=False, backend="torch", device="cpu", seed=0)
    tm.fit(ds)
    th = tm.get_doc_topic_distribution(ds, n_samples=5)
    assert th.shape == (60, 6) and np.allclose(th.sum(1), 1, atol=1e-5)
    topics = tm.get_topics(5)
    assert len(topics) == 6 and all(len(t) == 5 and t[0] in terms for t in topics)
    wd = tm.get_topic_word_distribution()
    assert wd.shape == (6, len(terms)) and np.allclose(wd.sum(1), 1, atol=1e-6)
    assert len(tm.get_predicted_topics(ds, 3)) == 60
    # weights-only persistence round trip
    tm.model_dir = str(tmp_path)
    path = tm.save(str(tmp_path))
    assert path and path.endswith("epoch_1.pth")
    tm2 = AVITM(input_size=len(terms), n_components=6, model_type=model_type, hidden_sizes=(20, 20),
                batch_size=16, verbose=False, backend="torch", device="cpu", seed=1)
    import os
    tm2.load(os.path.dirname(path), 1)
    for k, v in tm.model.state_dict().items():
        assert torch.equal(v, tm2.model.state_dict()[k]), k


def test_neural_lda_double_softmax_flag():
    tm = _avitm(model_type="LDA")
    twm = tm.get_topic_word_matrix()
    assert np.allclose(twm.sum(1), 1, atol=1e-5)                    # softmax_V(BN_K(beta))
    d1 = tm.get_topic_word_distribution()                           # reference B9: softmax again
    tm.compat_double_softmax = False
    d2 = tm.get_topic_word_distribution()
    assert np.allclose(d2, twm) and not np.allclose(d1, d2)


def test_ctm_train_with_labels_and_zeroshot():
    rng = np.random.default_rng(0)
    X = random_csr(40, 30, 6, seed=2)
    emb = rng.normal(size=(40, 8)).astype(np.float32)
    lab = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 40)]
    ds = CTMDataset(emb, X, {i: f"w{i}" for i in range(30)}, labels=lab)
    tm = CombinedTM(input_size=30, contextual_size=8, n_components=4, hidden_sizes=(10, 10),
                    batch_size=8, num_epochs=1, label_size=3, verbose=False, backend="torch",
                    device="cpu")
    tm.fit(ds)                                                      # label loss path (B8 fixed)
    assert tm.get_doc_topic_distribution(ds, 2).shape == (40, 4)
    zs = ZeroShotTM(input_size=30, contextual_size=8, n_components=4, hidden_sizes=(10, 10),
                    batch_size=8, num_epochs=1, label_size=3, verbose=False, backend="torch",
                    device="cpu")
    zs.fit(ds)                                                      # labels with zeroshot (B12 fixed)
    assert zs.get_word_distribution_by_topic_id(0)[0][0].startswith("w")
    th = zs.get_doc_topic_distribution(ds, 2)
    assert len(zs.get_top_documents_per_topic_id(list(range(40)), th, 1, k=3)) == 3


def test_invalid_arguments():
    with pytest.raises(ValueError):
        _avitm(model_type="foo")
    with pytest.raises(TypeError):
        _avitm(hidden_sizes=[10, 10])
    with pytest.raises(ValueError):
        _avitm(solver="lbfgs")
