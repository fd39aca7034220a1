"""Quality metrics (TSS/DSS/NPMI/TD/RBO/WMD) and the npz export layout."""
import numpy as np
import scipy.sparse as sp

from gfedntm_amd.eval.export import (client_model_path, load_model_npz, postprocess_thetas,
                                     save_model_as_npz, server_model_path)
from gfedntm_amd.eval.metrics import (betas_to_ground_truth_vocab, dss, inverted_rbo,
                                      mean_min_wmd, npmi_coherence, rbo, topic_diversity, tss,
                                      word_movers_distance)


def test_tss_dss():
    rng = np.random.default_rng(0)
    gt = rng.dirichlet(np.ones(20), 4)
    assert abs(tss(gt, gt) - 4.0) < 1e-9                  # every topic matched with BC = 1
    assert tss(rng.dirichlet(np.ones(20), 4), gt) < 4.0
    th = rng.dirichlet(np.ones(4), 30)
    assert dss(th, th) == 0.0 and dss(th, rng.dirichlet(np.ones(4), 30)) > 0


def test_betas_to_gt_vocab():
    b = np.array([[0.5, 0.5], [0.2, 0.8]])
    out = betas_to_ground_truth_vocab(b, {0: "wd3", 1: "wd0"}, 5)
    assert out.shape == (2, 5) and out[0, 3] == 0.5 and out[1, 0] == 0.8


def test_npmi_simple():
    # words 0,1 always co-occur; word 2 never with them
    X = sp.csr_matrix(np.array([[1, 1, 0], [1, 1, 0], [0, 0, 1], [0, 0, 1]], dtype=np.float32))
    assert abs(npmi_coherence([[0, 1]], X) - 1.0) < 1e-6
    assert npmi_coherence([[0, 2]], X) < -0.9


def test_diversity_rbo_wmd():
    assert topic_diversity([["a", "b"], ["c", "d"]]) == 1.0
    assert topic_diversity([["a", "b"], ["a", "b"]]) == 0.5
    assert abs(rbo(list("abcdef"), list("abcdef")) - 1.0) < 1e-9
    assert rbo(list("abc"), list("xyz")) == 0.0
    assert inverted_rbo([list("abc"), list("xyz")]) == 1.0
    vec = {"a": np.array([0.0, 0.0]), "b": np.array([1.0, 0.0]), "c": np.array([0.0, 3.0])}
    assert abs(word_movers_distance(["a"], ["b"], vec) - 1.0) < 1e-6
    assert abs(mean_min_wmd([["a"]], [["b"], ["c"]], vec) - 1.0) < 1e-6


def test_npz_layout(tmp_path):
    th = postprocess_thetas(np.array([[0.001, 0.5, 0.499], [0.2, 0.3, 0.5]]))
    assert th[0, 0] == 0 and np.allclose(th.sum(1), 1)
    p = client_model_path(str(tmp_path / "client"), 3, "20240101")
    assert p.endswith("client3/model_3_20240101.npz")
    betas = np.full((3, 4), 0.25)
    save_model_as_npz(p, betas, th, 3, [["a", "b"], ["c", "d"], ["e", "f"]])
    z = load_model_npz(p)
    assert set(z) == {"betas", "thetas", "ntopics", "topics"} and int(z["ntopics"]) == 3
    assert z["topics"][1][0] == "c"
    sp_path = str(tmp_path / "s.npz")
    save_model_as_npz(sp_path, betas, sp.csr_matrix(th), 3, None)
    z2 = load_model_npz(sp_path)
    assert sp.issparse(z2["thetas"]) and np.allclose(z2["thetas"].toarray(), th)
    with np.load(sp_path, allow_pickle=False) as raw:
        assert {"thetas_data", "thetas_indices", "thetas_indptr", "thetas_shape"} <= set(raw.files)
    assert server_model_path("/x", "20240101") == "/x/global_model_20240101.npz"
