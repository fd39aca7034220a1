"""theta-inference kernel (csrc/infer.hip) vs PyTorch / numpy fp32-fp64 oracles.

* posterior moments (mu, log sigma^2 after the running-statistics batch-norm) vs the
  reference encoder in eval mode (inference_network.py:76-85), AVITM and CTM inputs;
* the S-sample mean of softmax(mu + eps * sigma) vs the same formula in float64 with
  the kernel's Philox4x32-10 / Box-Muller draws reproduced in numpy;
* the fused threshold + L1 post-processing vs eval/export.py postprocess_thetas;
* chunk independence and the get_doc_topic_distribution entry point.
"""
import numpy as np
import pytest
import torch

from gfedntm_amd.data.bow import BatchPlan, BOWDataset, DeviceCSR
from gfedntm_amd.eval.export import postprocess_thetas
from gfedntm_amd.models import AVITM, CombinedTM, ZeroShotTM
from tests.helpers import random_csr

pytestmark = pytest.mark.gpu

U32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(seed: int, c0, c1, c2, c3):
    """csrc/gfk_common.h philox(): 10 rounds, key (seed lo, seed hi)."""
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    shape = np.broadcast(np.asarray(c0), np.asarray(c1), np.asarray(c2), np.asarray(c3)).shape
    x = [np.broadcast_to(np.asarray(v, dtype=np.uint64), shape).copy() for v in (c0, c1, c2, c3)]
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * x[0]
        p1 = np.uint64(0xCD9E8D57) * x[2]
        x = [((p1 >> np.uint64(32)) ^ x[1] ^ k0) & U32, p1 & U32,
             ((p0 >> np.uint64(32)) ^ x[3] ^ k1) & U32, p0 & U32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & U32
        k1 = (k1 + np.uint64(0xBB67AE85)) & U32
    return x


def infer_normals(seed: int, n_docs: int, K: int, S: int) -> np.ndarray:
    """[S, n_docs, K] draws of csrc/infer.hip: Philox(idx = d K + k, ctr = s / 4,
    tag RNG_INFER = 4), Box-Muller on both halves."""
    idx = (np.arange(n_docs, dtype=np.uint64)[:, None] * np.uint64(K)
           + np.arange(K, dtype=np.uint64)[None, :])
    out = np.empty((S, n_docs, K))
    for c in range((S + 3) // 4):
        r = philox4x32_10(seed, idx, c, 4, 0x5EED)
        f = [v.astype(np.float64) for v in r]
        u1 = (np.floor(f[0] / 256) + 1) / 2**24
        u2 = np.floor(f[1] / 256) / 2**24
        u3 = (np.floor(f[2] / 256) + 1) / 2**24
        u4 = np.floor(f[3] / 256) / 2**24
        ra, rb = np.sqrt(-2 * np.log(u1)), np.sqrt(-2 * np.log(u3))
        n4 = (ra * np.cos(2 * np.pi * u2), ra * np.sin(2 * np.pi * u2),
              rb * np.cos(2 * np.pi * u4), rb * np.sin(2 * np.pi * u4))
        for j in range(4):
            if 4 * c + j < S:
                out[4 * c + j] = n4[j]
    return out


def _trained(K=20, H=(32, 24), V=700, n_docs=300, steps=5, seed=0, model_type="prodLDA",
             activation="softplus"):
    torch.manual_seed(seed)
    tm = AVITM(input_size=V, n_components=K, model_type=model_type, hidden_sizes=H,
               batch_size=64, verbose=False, device="cuda", backend="fused",
               activation=activation)
    X = random_csr(n_docs, V, 40, seed=1)
    data = DeviceCSR(X, "cuda")
    tm.engine.bind_data(data, BatchPlan.build(n_docs, 64, steps, seed=seed))
    for s in range(steps):       # non-trivial running statistics
        tm.engine.step(s)
    torch.cuda.synchronize()
    return tm, X, data


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("K,H", [(20, (32, 24)), (100, (40,)), (200, (50, 50)),
                                 (50, (100, 100, 80)), (30, (200, 64))])
def test_moments_match_eval_encoder(model_type, K, H):
    tm, X, data = _trained(K=K, H=H, model_type=model_type)
    mom = tm.engine.theta_infer(data, moments=True)
    tm.model.eval()
    with torch.no_grad():
        mu, ls = tm.model.inf_net(torch.from_numpy(X.toarray()).cuda())
    torch.testing.assert_close(mom[:, 0], mu, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(mom[:, 1], ls, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("activation", ["rrelu", "selu"])
def test_moments_eval_activation(activation):
    """Eval-mode activations in the inference kernel (RReLU: the mean slope)."""
    tm, X, data = _trained(K=20, H=(32, 24), activation=activation)
    mom = tm.engine.theta_infer(data, moments=True)
    tm.model.eval()
    with torch.no_grad():
        mu, ls = tm.model.inf_net(torch.from_numpy(X.toarray()).cuda())
    torch.testing.assert_close(mom[:, 0], mu, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(mom[:, 1], ls, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("K,S", [(20, 20), (130, 7)])
def test_theta_mean_matches_philox_oracle(K, S):
    tm, X, data = _trained(K=K, H=(32, 24))
    seed = 0x1234_5678_9ABC
    mom = tm.engine.theta_infer(data, moments=True).double().cpu().numpy()
    th = tm.engine.theta_infer(data, n_samples=S, seed=seed).double().cpu().numpy()
    eps = infer_normals(seed, X.shape[0], K, S)
    z = mom[None, :, 0] + eps * np.exp(0.5 * mom[None, :, 1])
    z -= z.max(-1, keepdims=True)
    e = np.exp(z)
    ref = (e / e.sum(-1, keepdims=True)).mean(0)
    np.testing.assert_allclose(th, ref, rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(th.sum(1), 1.0, atol=1e-5)


def test_postprocess_chunking_and_api():
    tm, X, data = _trained()
    e = tm.engine
    th = e.theta_infer(data, n_samples=20, seed=5)
    th_small = e.theta_infer(data, n_samples=20, seed=5, chunk=37)     # other grid + chunks
    assert torch.equal(th, th_small)
    thr = float(np.float32(3e-3))
    pp = e.theta_infer(data, n_samples=20, seed=5, postprocess=True, threshold=thr)
    np.testing.assert_allclose(pp.cpu().numpy(), postprocess_thetas(th.cpu().numpy(), thr),
                               rtol=1e-5, atol=1e-6)
    ds = BOWDataset(X, {i: str(i) for i in range(X.shape[1])})
    api = tm.get_doc_topic_distribution(ds, n_samples=20, seed=5)
    np.testing.assert_array_equal(api, th.cpu().numpy())


@pytest.mark.parametrize("cls", [CombinedTM, ZeroShotTM])
def test_ctm_moments(cls):
    torch.manual_seed(0)
    V, C, K, n = 300, 48, 16, 150
    X = random_csr(n, V, 30, seed=3)
    emb = np.random.default_rng(0).standard_normal((n, C)).astype(np.float32)
    tm = cls(input_size=V, contextual_size=C, n_components=K, hidden_sizes=(32, 32),
             batch_size=64, verbose=False, device="cuda", backend="fused")
    data = DeviceCSR(X, "cuda", contextual=emb)
    tm.engine.bind_data(data, BatchPlan.build(n, 64, 3, seed=0))
    for s in range(3):
        tm.engine.step(s)
    mom = tm.engine.theta_infer(data, moments=True)
    tm.model.eval()
    with torch.no_grad():
        mu, ls = tm.model.inf_net(torch.from_numpy(X.toarray()).cuda(), data.contextual, None)
    torch.testing.assert_close(mom[:, 0], mu, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(mom[:, 1], ls, rtol=1e-4, atol=1e-4)
