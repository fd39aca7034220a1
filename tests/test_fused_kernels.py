"""Fused HIP step vs the PyTorch fp32 oracle (same weights, same noise).

The kernels draw their dropout masks / Gaussian noise from Philox; the test
reads them back from the engine workspace and feeds them to the functional
oracle (gfedntm_amd/models/functional.py), then compares loss, every
gradient, BN running statistics and the post-Adam parameters.
"""
import copy

import numpy as np
import pytest
import torch

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
from gfedntm_amd.models import AVITM
from gfedntm_amd.models.functional import avitm_loss_explicit
from gfedntm_amd.ops import kernel_abi as abi
from gfedntm_amd.ops.engine import UPDATE_FUSED, UPDATE_GRAD
from tests.helpers import random_csr

pytestmark = pytest.mark.gpu


def _pair(model_type="prodLDA", V=700, K=20, H=(32, 24), B=64, activation="softplus", seed=0,
          **fused_kw):
    torch.manual_seed(seed)
    kw = dict(input_size=V, n_components=K, model_type=model_type, hidden_sizes=H,
              batch_size=B, activation=activation, verbose=False, device="cuda")
    fused = AVITM(backend="fused", **kw, **fused_kw)
    fused.engine.set_update_mode(UPDATE_GRAD)       # gradients materialised for the oracle
    ref = AVITM(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    return fused, ref


def _bind(tm, X, n_steps=3, seed=0, B=64):
    data = DeviceCSR(X, "cuda")
    plan = BatchPlan.build(data.n_docs, B, n_steps, seed=seed)
    tm.engine.bind_data(data, plan)
    return data, plan


# Gradients that are zero in exact arithmetic (batch-norm removes the bias of the
# layer before it; the prior mean sees sum_b mu_b = 0 after BN): both sides hold
# rounding noise, so they are compared against the scale of their layer instead.
_NOISE_KEYS = ("inf_net.f_mu.bias", "inf_net.f_sigma.bias", "prior_mean")


def _check_grads(g, ref):
    for k, p in ref.model.named_parameters():
        scale = p.grad.abs().max().item() + 1e-6
        atol = 2e-4 * scale + 1e-4
        if k in _NOISE_KEYS:
            atol = 1e-3 * max(q.grad.abs().max().item() for q in ref.model.parameters())
        torch.testing.assert_close(g[k], p.grad, rtol=2e-3, atol=atol,
                                   msg=lambda m: f"{k}: {m}")


def _grads_of(tm_fused):
    e = tm_fused.engine
    return {k: e.gradient(k).detach().clone() for k, _ in e.param_order}


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("B,n_docs,K,H,V", [(64, 150, 20, (32, 24), 700), (32, 45, 20, (32, 24), 700),
                                            (128, 300, 50, (50, 50), 2000),     # 128-row batches
                                            (64, 150, 10, (50, 50), 5000),      # K = 10, V = 5 k
                                            (64, 80, 50, (50, 50), 100000),     # V = 100 k
                                            (64, 100, 100, (40,), 700),
                                            (64, 200, 50, (50, 50, 50), 700),
                                            (64, 100, 200, (50, 50), 700),       # K > 128, L2 mode
                                            (64, 120, 25, (30, 20), 700),        # odd K, odd strides
                                            (64, 80, 50, (50, 50), 30000),       # many V tiles
                                            (64, 80, 50, (50, 50), 40000),       # persistent decoder
                                            (64, 80, 200, (50, 50), 40000),      # persistent, 4 k ranges
                                            (64, 80, 20, (32, 24), 40000),       # persistent, one k range
                                            (128, 200, 100, (50, 50), 70000),    # k ranges of 2 tiles, B=128
                                            (64, 80, 200, (50, 50), 112000)])    # the BASELINE K=200 class
def test_step_matches_oracle(model_type, B, n_docs, K, H, V):
    _oracle_step(model_type, B, n_docs, K, H, V)


@pytest.mark.parametrize("B,n_docs,K,H,V", [(64, 80, 200, (50, 50), 40000),   # the auto choice
                                            (64, 80, 50, (50, 50), 30001),    # K % 8 = 2, V % 64 != 0
                                            (32, 45, 25, (30, 20), 7000),     # odd K, B = 32
                                            (16, 30, 20, (32, 24), 700),      # B = 16, K % 8 = 4
                                            (32, 60, 250, (50,), 5000),       # K = 250 (NP = 32)
                                            (64, 150, 256, (50,), 5000),      # K = 256, B = 64: forced k split
                                            # more strips than waves (V > 65k on 256 CUs): a
                                            # wave's second strip reads its first pairs from
                                            # the ring slots the previous strip refilled
                                            (64, 80, 200, (50, 50), 80000),   # NP = 25, ring 5
                                            (64, 80, 204, (50,), 80000),      # NP = 26, ring 13
                                            (64, 80, 120, (50,), 80000),      # NP = 16, ring 8
                                            (64, 80, 250, (50,), 80000)])     # NP = 32, ring 8
def test_strip_forward_matches_oracle(monkeypatch, B, n_docs, K, H, V):
    """prodlda_fwd_strip_kernel (GFEDNTM_FWD_STRIP=1 forces it): per-wave column strips,
    beta by buffer loads straight into the MFMA B registers, k paired for ds_read_b64,
    the next pairs through a <= 13-pair ring (more than 13 pairs: the current strip's
    later pairs, then the next's)."""
    monkeypatch.setenv("GFEDNTM_FWD_STRIP", "1")
    from gfedntm_amd.ops.engine import STAGE_FWD_STRIP
    fused, _ = _pair("prodLDA", V=V, K=K, H=H, B=B)
    assert fused.engine._m.stage_flags & STAGE_FWD_STRIP
    _oracle_step("prodLDA", B, n_docs, K, H, V)


@pytest.mark.parametrize("pre", ["3", "2", "0"])
@pytest.mark.parametrize("B,n_docs,K,V", [(64, 80, 200, 40000), (32, 60, 64, 40000),
                                          (64, 100, 64, 40000), (64, 70, 100, 30011)])
def test_bwd_precomputed_dlogit_matches_oracle(monkeypatch, pre, B, n_docs, K, V):
    """Persistent 4-k-range backward: the logit-gradient tiles precomputed once per tile
    by prodlda_dlogit -- software-pipelined (GFEDNTM_BWD_PRE=3, the default at B = 64;
    B = 32 runs the =2 kernel), two workgroups per CU (=2) -- or recomputed
    by every range workgroup (=0): all match the oracle (K = 100: a partial last k tile;
    V = 30011: a partial last vocabulary tile)."""
    monkeypatch.setenv("GFEDNTM_BWD_PRE", pre)
    fused, _ = _pair("prodLDA", V=V, K=K, H=(50, 50), B=B)
    m = fused.engine._m
    want = 2 if (pre == "3" and B != 64) else int(pre)
    assert m.n_dpart < m.n_tiles and m.bwd_pre == want
    _oracle_step("prodLDA", B, n_docs, K, (50, 50), V)


def test_large_k_few_tiles_forces_k_split(monkeypatch):
    """K = 256, B = 64, 79 vocab tiles: the one-range backward (a workgroup per tile) needs
    more than 160 KiB of LDS, so the engine uses the 4-k-range shape (n_dpart < n_tiles)."""
    monkeypatch.setenv("GFEDNTM_FWD_STRIP", "0")
    fused, _ = _pair("prodLDA", V=5000, K=256, H=(50,), B=64)
    m = fused.engine._m
    assert m.n_dpart < m.n_tiles
    _oracle_step("prodLDA", 64, 150, 256, (50,), 5000)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("B,K", [(64, 50), (128, 50)])
def test_long_rows_match_oracle(model_type, B, K):
    """Rows of up to 400 non-zeros (several per lane in the row-wise loops)."""
    _oracle_step(model_type, B, 2 * B, K, (50, 50), 3000, nnz=400)


def _oracle_step(model_type, B, n_docs, K, H, V, nnz=40):
    fused, ref = _pair(model_type, V=V, K=K, H=H, B=B)
    if K == 200 and model_type == "prodLDA" and B == 64:
        assert fused.engine._m.stage_flags & 2     # batch matrices read from L2
    X = random_csr(n_docs, V, nnz, seed=1)
    data, plan = _bind(fused, X, B=B)
    e = fused.engine
    phases = e.phases()
    e.run_phases(phases[:-1])            # everything but Adam
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x = data.dense_rows(ids)
    eps = e.ws["eps"][:nb].clone()
    mask_h = e.ws["mask_h"][:nb].clone()
    mask_t = e.ws["mask_t"][:nb].clone()
    ref.model.train()
    ref.model.zero_grad()
    loss, kl, rl = avitm_loss_explicit(ref.model, x, eps, mask_h, mask_t)
    loss.backward()
    torch.testing.assert_close(e.ws["kl"][:nb], kl.detach(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(e.loss_hist[0], loss.detach(), rtol=1e-4, atol=1e-2)
    g = _grads_of(fused)
    _check_grads(g, ref)
    sd_f, sd_r = fused.model.state_dict(), ref.model.state_dict()
    for k in sd_r:
        if "running" in k or "num_batches" in k:
            torch.testing.assert_close(sd_f[k].float(), sd_r[k].float(), rtol=1e-4, atol=1e-5,
                                       msg=lambda m: f"{k}: {m}")
    # Adam, on identical gradients (a near-zero gradient's sign is rounding noise and
    # Adam's first step normalises it to +-lr, so compare the optimizer in isolation)
    for k, p in ref.model.named_parameters():
        p.grad.copy_(g[k])
    ref.optimizer.step()
    e.run_phases([abi.PH_ADAM])
    torch.cuda.synchronize()
    sd_f = fused.model.state_dict()
    for k, p in ref.model.named_parameters():
        torch.testing.assert_close(sd_f[k], p.detach(), rtol=1e-4, atol=1e-5,
                                   msg=lambda m: f"{k}: {m}")
    assert int(e.d_step.item()) == 1 and int(e.adam_t.item()) == 1
    assert float(e.grad.abs().max().item()) == 0.0   # consumed and cleared


class _SlopeAct(torch.nn.Module):
    """RReLU with given per-element slopes (one tensor per call, in call order: the
    input layer's activation, then each hidden layer's) -- the kernels' Philox draws."""

    def __init__(self, slopes):
        super().__init__()
        self.slopes, self.i = slopes, 0

    def forward(self, z):
        r = self.slopes[self.i]
        self.i += 1
        return torch.where(z > 0, z, z * r)


@pytest.mark.parametrize("activation", ["relu", "tanh", "elu", "selu", "sigmoid", "leakyrelu",
                                        "rrelu"])
def test_activations(activation):
    fused, ref = _pair("prodLDA", V=300, K=10, H=(16, 16, 8), B=32, activation=activation)
    X = random_csr(40, 300, 20, seed=3)
    data, plan = _bind(fused, X, B=32)
    e = fused.engine
    e.run_phases(e.phases()[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    if activation == "rrelu":
        # ws_z holds d act / d z for RReLU: 1, or the element's drawn slope in [1/8, 1/3]
        slopes = [e.ws[f"z{l}"][:nb].clone() for l in range(3)]
        neg = torch.cat([s[s != 1.0] for s in slopes])
        assert neg.numel() > 0 and float(neg.min()) >= 0.125 and float(neg.max()) <= 1 / 3 + 1e-6
        act = _SlopeAct(slopes)
        net = ref.model.inf_net
        net.activation = act
        for blk in net.hiddens:
            blk[1] = act
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x = data.dense_rows(ids)
    loss, _, _ = avitm_loss_explicit(ref.model, x, e.ws["eps"][:nb], e.ws["mask_h"][:nb],
                                     e.ws["mask_t"][:nb])
    ref.model.zero_grad()
    loss.backward()
    torch.testing.assert_close(e.loss_hist[0], loss.detach(), rtol=1e-4, atol=1e-2)
    g = _grads_of(fused)
    _check_grads(g, ref)


def test_graph_replay_matches_eager():
    torch.manual_seed(0)
    kw = dict(input_size=500, n_components=16, hidden_sizes=(32, 32), batch_size=64,
              verbose=False, device="cuda")
    a = AVITM(backend="fused", **kw)
    b = AVITM(backend="fused", **kw)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = a.engine.seed
    b.engine._m.seed = a.engine.seed
    X = random_csr(300, 500, 30, seed=5)
    _bind(a, X, n_steps=12)
    _bind(b, X, n_steps=12)
    b.engine.enable_graph(True)
    for s in range(12):
        a.engine.step(s)
        b.engine.step(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.engine.loss_hist, b.engine.loss_hist, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(a.flat.buffer, b.flat.buffer, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("B,K,H", [(64, 50, (50, 50)), (32, 20, (32,)), (16, 100, (24, 100, 24))])
def test_fused_update_matches_gradient_mode(B, K, H, model_type):
    """The Adam epilogues fused into prodlda_bwd / enc_head_bwd / win_update give the
    same parameters, moments and BN statistics as gradient mode + the generic Adam,
    over several steps, with the FedAvg pre-scale on."""
    torch.manual_seed(0)
    kw = dict(input_size=900, n_components=K, hidden_sizes=H, batch_size=B, verbose=False,
              device="cuda", model_type=model_type)
    a = AVITM(backend="fused", **kw)
    b = AVITM(backend="fused", **kw)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = a.engine.seed
    b.engine._m.seed = a.engine.seed
    b.engine.set_update_mode(UPDATE_GRAD)
    assert a.engine.update_mode == UPDATE_FUSED
    for e in (a.engine, b.engine):
        e.set_fedavg_scale(0.75)
    X = random_csr(3 * B, 900, 35, seed=2)
    _bind(a, X, n_steps=6, B=B)
    _bind(b, X, n_steps=6, B=B)
    for s in range(6):
        a.engine.step(s)
        b.engine.step(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.engine.loss_hist, b.engine.loss_hist, rtol=1e-4, atol=1e-2)
    # the two paths inline the same Adam arithmetic into different kernels, so FP
    # contraction may differ by an ulp; tensors whose true gradient is 0 (rounding
    # noise, see _NOISE_KEYS) then diverge by up to lr per step after Adam.
    sa, sb = a.model.state_dict(), b.model.state_dict()
    lr_steps = 2 * a.engine.lr * 6
    for k in sb:
        if not sb[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        noisy = k in _NOISE_KEYS or k.startswith(("inf_net.f_mu_batchnorm.running_mean",
                                                   "inf_net.f_sigma_batchnorm.running_mean"))
        atol = lr_steps if noisy else 5e-5
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-3, atol=atol, msg=lambda m: f"{k}: {m}")


def test_training_decreases_loss():
    torch.manual_seed(0)
    from tests.helpers import tiny_corpus
    from gfedntm_amd.data.bow import BOWDataset
    c, terms, shards = tiny_corpus(V=800, K=10, n_docs=600, n_nodes=1, nwords=(80, 120))
    ds = BOWDataset(shards[0], {i: t for i, t in enumerate(terms)})
    m = AVITM(input_size=len(terms), n_components=10, hidden_sizes=(50, 50), num_epochs=15,
              verbose=False, backend="fused", device="cuda")
    data = m.device_data(ds)
    plan = BatchPlan.build(data.n_docs, 64, 10 * 15, seed=0)
    m.engine.bind_data(data, plan)
    for s in range(plan.n_steps):
        m.engine.step(s)
    h = m.engine.loss_hist.cpu().numpy()
    assert np.isfinite(h).all()
    assert h[-10:].mean() < 0.9 * h[:10].mean()


@pytest.mark.parametrize("inference_type,Cdim,V,K", [("combined", 96, 600, 20), ("combined", 100, 600, 20),
                                                     ("combined", 16, 600, 20), ("zeroshot", 96, 600, 20),
                                                     # the BASELINE CTM class at large V
                                                     ("combined", 768, 74000, 100)])
@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_ctm_step_matches_oracle(inference_type, Cdim, V, K, model_type):
    """CTM on the fused engine: CombinedTM's contextual path on ctx_fwd / ctx_bwd
    (csrc/ctx.hip, C split into chunks), ZeroShotTM's dense input layer in enc_in /
    win_update; compared with the explicit-noise oracle through the CTM encoder
    (gradient mode), up to CombinedTM K = 100, C = 768, V = 74k."""
    from gfedntm_amd.models import CombinedTM, ZeroShotTM
    if V > 10000 and model_type == "LDA":
        pytest.skip("large-V point: ProdLDA (the BASELINE CTM configuration)")
    cls = CombinedTM if inference_type == "combined" else ZeroShotTM
    H, B, n_docs = (32, 24), 64, 150
    torch.manual_seed(0)
    kw = dict(input_size=V, contextual_size=Cdim, n_components=K, model_type=model_type,
              hidden_sizes=H, batch_size=B, verbose=False, device="cuda")
    fused = cls(backend="fused", **kw)
    assert fused.backend == "fused"
    ref = cls(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    X = random_csr(n_docs, V, 40, seed=1)
    ctx = np.random.default_rng(2).standard_normal((n_docs, Cdim)).astype(np.float32)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    plan = BatchPlan.build(data.n_docs, B, 3, seed=0)
    e = fused.engine
    assert e.update_mode == UPDATE_FUSED
    if inference_type == "combined":
        # (C split over the CUs' slots: one chunk of <= 256 at large V, more at small V)
        assert e._m.ctx_fused == 1 and e._m.ctx_kb * e._m.ctx_ckb >= Cdim
        assert (e._m.ctx_kb > 1) == (Cdim > 16) or V > 50000
    else:
        assert e._m.ctx_fused == 2           # dense input layer in enc_in / win_update
    e.set_update_mode(UPDATE_GRAD)
    e.bind_data(data, plan)
    phases = e.phases()
    ctx_ph = (abi.PH_CTXF_FWD, abi.PH_CTXF_BWD) if inference_type == "combined" else ()
    assert phases[-1] == abi.PH_ADAM and all(p in phases for p in ctx_ph)
    assert not any(p in abi.HOST_PHASES for p in phases)
    e.run_phases(phases[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x, xc = data.dense_rows(ids), data.contextual[ids]
    eps = e.ws["eps"][:nb].clone()
    mask_h = e.ws["mask_h"][:nb].clone()
    mask_t = e.ws["mask_t"][:nb].clone()
    ref.model.train()
    ref.model.zero_grad()
    net = ref.model.inf_net
    x_enc = torch.cat([x, net.adapt_bert(xc)], 1) if inference_type == "combined" else xc
    kw_ = float(ref.weights.get("beta", 1.0))
    loss, kl, rl = avitm_loss_explicit(ref.model, x, eps, mask_h, mask_t, kl_weight=kw_,
                                       x_enc=x_enc)
    loss.backward()
    torch.testing.assert_close(e.ws["kl"][:nb], kl.detach(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=1e-4, atol=1e-2)
    _check_grads(_grads_of(fused), ref)
    e.run_phases([abi.PH_ADAM])
    torch.cuda.synchronize()
    assert float(e.grad.abs().max().item()) == 0.0


@pytest.mark.parametrize("inference_type", ["combined", "zeroshot"])
@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_ctm_fused_update_matches_gradient_mode(model_type, inference_type):
    """CTM: Adam fused into ctx_bwd (adapt_bert) and win_update's contextual tiles (the
    input layer; ZeroShotTM: the whole dense layer) == gradient mode + the generic Adam,
    with the FedAvg pre-scale."""
    from gfedntm_amd.models import CombinedTM, ZeroShotTM
    cls = CombinedTM if inference_type == "combined" else ZeroShotTM
    V, K, B, Cdim, n_docs = 700, 30, 64, 136, 200
    torch.manual_seed(0)
    kw = dict(input_size=V, contextual_size=Cdim, n_components=K, hidden_sizes=(48, 40),
              batch_size=B, verbose=False, device="cuda", backend="fused", model_type=model_type)
    a, b = cls(**kw), cls(**kw)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    b.engine.set_update_mode(UPDATE_GRAD)
    X = random_csr(n_docs, V, 40, seed=3)
    ctx = np.random.default_rng(4).standard_normal((n_docs, Cdim)).astype(np.float32)
    for t in (a, b):
        t.engine.set_fedavg_scale(0.75)
        t.engine.bind_data(DeviceCSR(X, "cuda", contextual=ctx), BatchPlan.build(n_docs, B, 5, seed=0))
    for s in range(5):
        a.engine.step(s)
        b.engine.step(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.engine.loss_hist, b.engine.loss_hist, rtol=1e-4, atol=1e-2)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    lr_steps = 2 * a.engine.lr * 5
    for k in sb:
        if not sb[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        noisy = k in _NOISE_KEYS or k.startswith(("inf_net.f_mu_batchnorm.running_mean",
                                                   "inf_net.f_sigma_batchnorm.running_mean"))
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-3, atol=lr_steps if noisy else 5e-5,
                                   msg=lambda m: f"{k}: {m}")


def test_ctm_graph_training():
    from gfedntm_amd.models import CombinedTM
    V, K, B, Cdim, n_docs = 500, 10, 64, 64, 400
    torch.manual_seed(0)
    tm = CombinedTM(input_size=V, contextual_size=Cdim, n_components=K, hidden_sizes=(50, 50),
                    batch_size=B, verbose=False, device="cuda", backend="fused")
    X = random_csr(n_docs, V, 40, seed=3)
    ctx = np.random.default_rng(4).standard_normal((n_docs, Cdim)).astype(np.float32)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    plan = BatchPlan.build(data.n_docs, B, 200, seed=0)
    e = tm.engine
    e.bind_data(data, plan)
    e.enable_graph(True)
    for s in range(200):
        e.step(s)
    h = e.loss_hist[:200].cpu().numpy()
    assert np.isfinite(h).all() and h[-20:].mean() < h[:20].mean()


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_steps_are_bitwise_deterministic(model_type):
    """No atomics anywhere: two runs from the same state give identical bits."""
    X = random_csr(300, 900, 60, seed=5)
    outs = []
    for _ in range(2):
        torch.manual_seed(3)
        tm = AVITM(input_size=900, n_components=30, model_type=model_type, hidden_sizes=(40, 40),
                   batch_size=64, verbose=False, device="cuda", backend="fused")
        _bind(tm, X, n_steps=12)
        for s in range(12):
            tm.engine.step(s)
        torch.cuda.synchronize()
        outs.append((tm.flat.buffer.clone(), tm.engine.loss_hist[:12].clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA", "ctm"])
@pytest.mark.parametrize("mode", [UPDATE_FUSED, UPDATE_GRAD])
def test_fedavg_prescale_covers_every_shared_tensor(model_type, mode):
    """One step with the FedAvg pre-scale w must leave w x (the unscaled step) in EVERY
    shared float tensor -- parameters and batch-norm running statistics alike -- or the
    all-reduce would not be the sample-weighted average (server.py:477-487)."""
    torch.manual_seed(0)
    kw = dict(input_size=700, n_components=20, hidden_sizes=(32, 24), batch_size=64,
              verbose=False, device="cuda", model_type=model_type)
    X = random_csr(150, 700, 40, seed=1)
    if model_type == "ctm":           # CombinedTM (adapt_bert + contextual input half)
        from gfedntm_amd.models import CombinedTM
        kw.update(model_type="prodLDA", contextual_size=80)
        a, b = CombinedTM(backend="fused", **kw), CombinedTM(backend="fused", **kw)
        ctx = np.random.default_rng(4).standard_normal((150, 80)).astype(np.float32)
        bind = lambda t: t.engine.bind_data(DeviceCSR(X, "cuda", contextual=ctx),  # noqa: E731
                                            BatchPlan.build(150, 64, 1, seed=0))
    else:
        a, b = AVITM(backend="fused", **kw), AVITM(backend="fused", **kw)
        bind = lambda t: _bind(t, X, n_steps=1)  # noqa: E731
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    for e in (a.engine, b.engine):
        e.set_update_mode(mode)
    a.engine.set_fedavg_scale(0.25)
    bind(a)
    bind(b)
    a.engine.step(0)
    b.engine.step(0)
    torch.cuda.synchronize()
    sa, sb = a.model.state_dict(), b.model.state_dict()
    for k in a.shared_keys:
        if k in sb and sb[k].is_floating_point():
            torch.testing.assert_close(sa[k], 0.25 * sb[k], rtol=1e-5, atol=1e-7,
                                       msg=lambda m: f"{k}: {m}")


def _bf(x):
    return x.to(torch.bfloat16).float()


@pytest.mark.parametrize("K,V", [(50, 2000), (200, 40000), (120, 9000), (200, 80000)])
def test_bf16_decoder_matches_emulated_oracle(K, V):
    """matmul_dtype='bf16': theta_d.beta, theta_d^T.dlogit and dlogit.beta^T take bf16
    operands on the matrix cores with fp32 accumulation.  Oracle: the fp32 PyTorch step
    with theta_d and beta rounded to bf16 before the logits GEMM (the backward GEMMs'
    extra rounding of dlogit is inside the gradient tolerance).  The forward is the bf16
    strip kernel (32-k steps: 8, 16 or 32 pairs, a ring of 8); V = 80k: waves with a
    second strip (the ring's cross-strip slots).  At V = 40k / 80k the backward is the
    pipelined kernel, whose GEMMs keep fp32 operands in bf16 mode (HBM-bound)."""
    from gfedntm_amd.models.functional import encoder_forward
    from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
    import torch.nn.functional as F
    from gfedntm_amd.ops.engine import STAGE_FWD_STRIP
    fused, ref = _pair("prodLDA", V=V, K=K, H=(50, 50), B=64, matmul_dtype="bf16")
    assert fused.engine._m.mm_bf16 == 1 and fused.engine._m.stage_flags & STAGE_FWD_STRIP
    X = random_csr(150, V, 60, seed=1)
    data, plan = _bind(fused, X, B=64)
    e = fused.engine
    e.run_phases(e.phases()[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x = data.dense_rows(ids)
    model = ref.model
    model.train()
    model.zero_grad()
    mu, ls = encoder_forward(model.inf_net, x, e.ws["mask_h"][:nb])
    theta = F.softmax(mu + e.ws["eps"][:nb] * torch.exp(0.5 * ls), dim=1)
    thetad = theta * e.ws["mask_t"][:nb]
    bf_round = lambda t: t + (_bf(t) - t).detach()      # noqa: E731  rounded forward, identity grad
    bb = model.beta_batchnorm
    logits = F.batch_norm(bf_round(thetad) @ bf_round(model.beta), bb.running_mean,
                          bb.running_var, training=True, momentum=bb.momentum, eps=bb.eps)
    wd = F.softmax(logits, dim=1)
    kl = kl_terms(model.prior_mean, model.prior_variance, mu, torch.exp(ls), ls, K)
    rl = reconstruction_terms(x, wd)
    loss = (kl + rl).sum()
    loss.backward()
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=2e-4, atol=5e-2)
    torch.testing.assert_close(e.loss_hist[0], loss.detach(), rtol=2e-4, atol=5e-2)
    g = _grads_of(fused)
    for k, p in model.named_parameters():
        if k in _NOISE_KEYS:
            continue
        scale = p.grad.abs().max().item() + 1e-6
        torch.testing.assert_close(g[k], p.grad, rtol=3e-2, atol=2e-2 * scale,
                                   msg=lambda m: f"{k}: {m}")


def test_bf16_training_tracks_fp32():
    """300 graph-replayed steps: the bf16-GEMM decoder's loss curve stays within 1 % of
    the fp32 one (same init, same data, same noise)."""
    curves = []
    X = random_csr(1000, 3000, 80, seed=4)
    for dt in ("fp32", "bf16"):
        torch.manual_seed(0)
        tm = AVITM(input_size=3000, n_components=50, hidden_sizes=(50, 50), batch_size=64,
                   verbose=False, device="cuda", backend="fused", matmul_dtype=dt)
        tm.engine.seed = tm.engine._m.seed = 1234
        _bind(tm, X, n_steps=300)
        tm.engine.enable_graph(True)
        for s in range(300):
            tm.engine.step(s)
        torch.cuda.synchronize()
        curves.append(tm.engine.loss_hist[:300].cpu().numpy())
    a, b = (c[-50:].mean() for c in curves)
    assert np.isfinite(curves[1]).all()
    assert abs(a - b) / a < 0.01, (a, b)


@pytest.mark.parametrize("inference_type", ["combined", "zeroshot"])
@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_ctm_label_head_matches_oracle(inference_type, model_type):
    """CTM label head on the fused engine (reference ctm decoding_network.py:84-85,156-159,
    ctm.py:292-296): labels appended to the encoder input, Linear(K -> L) on theta_d,
    batch-mean cross-entropy against argmax(labels) added to the summed KL + RL.  Loss,
    every gradient (classifier, input layer's label block) vs the PyTorch oracle."""
    import torch.nn.functional as F
    from gfedntm_amd.models import CombinedTM, ZeroShotTM
    from gfedntm_amd.models.functional import decoder_forward, encoder_forward
    from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
    cls = CombinedTM if inference_type == "combined" else ZeroShotTM
    V, K, H, B, n_docs, C, L = 600, 20, (32, 24), 64, 150, 48, 7
    torch.manual_seed(0)
    kw = dict(input_size=V, contextual_size=C, n_components=K, model_type=model_type,
              hidden_sizes=H, batch_size=B, verbose=False, device="cuda", label_size=L)
    fused = cls(backend="fused", **kw)
    assert fused.backend == "fused" and fused.engine._m.lab_on == 1
    ref = cls(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    X = random_csr(n_docs, V, 40, seed=1)
    rng = np.random.default_rng(2)
    ctx = rng.standard_normal((n_docs, C)).astype(np.float32)
    lab = np.eye(L, dtype=np.float32)[rng.integers(0, L, n_docs)]
    data = DeviceCSR(X, "cuda", contextual=ctx, labels=lab)
    plan = BatchPlan.build(data.n_docs, B, 3, seed=0)
    e = fused.engine
    e.set_update_mode(UPDATE_GRAD)
    e.bind_data(data, plan)
    e.run_phases(e.phases()[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x, xc, lb = data.dense_rows(ids), data.contextual[ids], data.labels[ids]
    model = ref.model
    model.train()
    model.zero_grad()
    net = model.inf_net
    x_enc = torch.cat([x, net.adapt_bert(xc), lb], 1) if inference_type == "combined" else \
        torch.cat([xc, lb], 1)
    mu, ls = encoder_forward(net, x_enc, e.ws["mask_h"][:nb])
    _, thetad, wd = decoder_forward(model, mu, ls, e.ws["eps"][:nb], e.ws["mask_t"][:nb])
    kl = kl_terms(model.prior_mean, model.prior_variance, mu, torch.exp(ls), ls, K)
    rl = reconstruction_terms(x, wd)
    ce = F.cross_entropy(model.label_classification(thetad), torch.argmax(lb, 1))
    loss = (kl + rl).sum() + ce
    loss.backward()
    torch.testing.assert_close(e.ws["ce"][:nb].sum(), ce.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(e.loss_hist[0], loss.detach(), rtol=1e-4, atol=1e-2)
    _check_grads(_grads_of(fused), ref)
    e.run_phases([abi.PH_ADAM])
    torch.cuda.synchronize()
    # inference encodes the labels too (the fused model's own, updated parameters)
    tm_theta = fused.engine.theta_infer(data, moments=True)
    fused.model.eval()
    with torch.no_grad():
        xa = torch.from_numpy(X.toarray()).cuda()
        mu_all, ls_all = fused.model.inf_net(xa, data.contextual, data.labels)
    torch.testing.assert_close(tm_theta[:, 0], mu_all, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(tm_theta[:, 1], ls_all, rtol=1e-4, atol=1e-4)


def test_ctm_label_head_fused_update_trains():
    """Fused Adam epilogues for the classifier and the label block, with graph replay:
    the label loss falls (log 4 = 1.39 at chance)."""
    from gfedntm_amd.models import CombinedTM
    V, K, C, L = 500, 16, 32, 4
    torch.manual_seed(0)
    tm = CombinedTM(input_size=V, contextual_size=C, n_components=K, hidden_sizes=(32, 32),
                    batch_size=64, verbose=False, device="cuda", backend="fused", label_size=L)
    assert tm.engine.update_mode == UPDATE_FUSED
    rng = np.random.default_rng(3)
    n = 512
    y = rng.integers(0, L, n)
    ctx = (np.eye(L)[y] @ rng.standard_normal((L, C)) + 0.1 * rng.standard_normal((n, C))).astype(np.float32)
    data = DeviceCSR(random_csr(n, V, 30, seed=5), "cuda", contextual=ctx,
                     labels=np.eye(L, dtype=np.float32)[y])
    tm.engine.bind_data(data, BatchPlan.build(n, 64, 400, seed=1))
    tm.engine.enable_graph(True)
    ce = []
    for s in range(400):
        tm.engine.step(s)
        if s in (0, 399):
            torch.cuda.synchronize()
            ce.append(float(tm.engine.ws["ce"][:64].sum()))
    assert np.isfinite(ce).all() and ce[1] < 0.85 * ce[0], ce


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_ctm_host_gemm_fallback_matches_oracle(model_type):
    """C % 4 != 0 is outside the fused contextual kernels' plan: the engine says why, runs
    adapt_bert / the contextual input half as host GEMMs between its kernels (gradient
    mode + generic optimizer), and the step still matches the fp32 oracle."""
    from gfedntm_amd.models import CombinedTM
    V, K, H, B, n_docs, Cdim = 500, 20, (32, 24), 64, 150, 30
    torch.manual_seed(0)
    kw = dict(input_size=V, contextual_size=Cdim, n_components=K, model_type=model_type,
              hidden_sizes=H, batch_size=B, verbose=False, device="cuda")
    fused = CombinedTM(backend="fused", **kw)
    ref = CombinedTM(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    e = fused.engine
    assert not e.ctx_fused and e.host_gemm_fallback and e.update_mode == UPDATE_GRAD
    assert "multiple of 4" in e.ctx_fallback_reason
    X = random_csr(n_docs, V, 40, seed=1)
    ctx = np.random.default_rng(2).standard_normal((n_docs, Cdim)).astype(np.float32)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    plan = BatchPlan.build(data.n_docs, B, 3, seed=0)
    e.bind_data(data, plan)
    phases = e.phases()
    assert abi.PH_CTX_FWD in phases and abi.PH_CTX_BWD in phases and phases[-1] == abi.PH_ADAM
    e.run_phases(phases[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x, xc = data.dense_rows(ids), data.contextual[ids]
    eps, mask_h, mask_t = (e.ws[k][:nb].clone() for k in ("eps", "mask_h", "mask_t"))
    ref.model.train()
    ref.model.zero_grad()
    net = ref.model.inf_net
    x_enc = torch.cat([x, net.adapt_bert(xc)], 1)
    loss, kl, rl = avitm_loss_explicit(ref.model, x, eps, mask_h, mask_t,
                                       kl_weight=float(ref.weights.get("beta", 1.0)), x_enc=x_enc)
    loss.backward()
    torch.testing.assert_close(e.ws["kl"][:nb], kl.detach(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=1e-4, atol=1e-2)
    _check_grads(_grads_of(fused), ref)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("B,n_docs,K,H,V", [(64, 80, 50, (50, 50), 3000), (128, 200, 20, (64,), 9000),
                                            (32, 45, 20, (30, 20), 20000),
                                            (128, 160, 20, (32,), 300)])   # > 512 entries per tile: list passes
def test_sparse_win_tiles_match_oracle(monkeypatch, model_type, B, n_docs, K, H, V):
    """W_in tiles as entry lists (GFEDNTM_WIN_SPARSE=1 forces the large-vocabulary path,
    csrc/update.hip win_tile_sparse) give the oracle's input-layer gradient."""
    monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    from gfedntm_amd.ops.engine import STAGE_WIN_SPARSE
    fused, _ = _pair(model_type, V=V, K=K, H=H, B=B)
    assert fused.engine._m.stage_flags & STAGE_WIN_SPARSE
    _oracle_step(model_type, B, n_docs, K, H, V)


@pytest.mark.parametrize("rs", ["1", "0"])
@pytest.mark.parametrize("Cdim,V", [(96, 600), (768, 9000), (100, 5000), (260, 3000), (768, 40000),
                                    (96, 69600), (260, 69600)])
def test_ctm_full_tile_forward_matches_oracle(monkeypatch, Cdim, V, rs):
    """ctx_fwd with all batch rows per vocab tile (stage_flags bit 5, the large-V shape;
    GFEDNTM_CTX_FULL=1 forces it at small V): the register-streamed kernel (bit 15, rs = 1:
    column ranges of 16-column units not aligned to the 64-column tiles, a partial last
    256-float phase at C = 96 / 100 / 260; V = 69.6k: 17 units in some workgroups, the last
    split over the helper waves' phases, one or two phases) or one workgroup per tile
    (rs = 0)."""
    from gfedntm_amd.ops.engine import STAGE_CTX_FULL, STAGE_CTX_RS
    monkeypatch.setenv("GFEDNTM_CTX_FULL", "1")
    monkeypatch.setenv("GFEDNTM_CTX_RS", rs)
    from gfedntm_amd.models import CombinedTM
    torch.manual_seed(0)
    tm = CombinedTM(input_size=V, contextual_size=Cdim, n_components=20, hidden_sizes=(32, 24),
                    batch_size=64, verbose=False, device="cuda", backend="fused")
    sf = tm.engine._m.stage_flags
    assert sf & STAGE_CTX_FULL and bool(sf & STAGE_CTX_RS) == (rs == "1")
    test_ctm_step_matches_oracle("combined", Cdim, V, 20, "prodLDA")


def test_ctm_v99k_step_matches_oracle():
    """The BASELINE CombinedTM class on its default kernels (C = 768: three 256-float x
    phases; V = 99k: 24-25 units per workgroup, the 25th split by phase) vs the oracle."""
    test_ctm_step_matches_oracle("combined", 768, 99000, 100, "prodLDA")


@pytest.mark.parametrize("Cdim,V", [(96, 600), (768, 9000)])
def test_ctm_sparse_win_tiles_match_oracle(monkeypatch, Cdim, V):
    """CombinedTM with the sparse W_in tiles (GFEDNTM_WIN_SPARSE=1 forces the large-V
    path): the bag-of-words half as entry-list tiles and the contextual half as dense
    A^T dz0 tiles of the same launch (csrc/update.hip win_tile_ctx) give the oracle's
    input-layer gradient (both halves)."""
    monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    test_ctm_step_matches_oracle("combined", Cdim, V, 20, "prodLDA")


def test_ctm_sparse_win_tiles_fused_update(monkeypatch):
    """The same tiles in the fused update mode (Adam + FedAvg pre-scale in win_tile_ctx's
    epilogue) == gradient mode + the generic Adam."""
    monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    from gfedntm_amd.ops.engine import STAGE_WIN_SPARSE
    from gfedntm_amd.models import CombinedTM
    torch.manual_seed(0)
    kw = dict(input_size=900, contextual_size=64, n_components=30, hidden_sizes=(48, 40),
              batch_size=64, verbose=False, device="cuda", backend="fused")
    a, b = CombinedTM(**kw), CombinedTM(**kw)
    assert a.engine._m.stage_flags & STAGE_WIN_SPARSE
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    b.engine.set_update_mode(UPDATE_GRAD)
    X = random_csr(200, 900, 40, seed=3)
    ctx = np.random.default_rng(4).standard_normal((200, 64)).astype(np.float32)
    for t in (a, b):
        t.engine.set_fedavg_scale(0.75)
        t.engine.bind_data(DeviceCSR(X, "cuda", contextual=ctx), BatchPlan.build(200, 64, 5, seed=0))
    for s in range(5):
        a.engine.step(s)
        b.engine.step(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.engine.loss_hist, b.engine.loss_hist, rtol=1e-4, atol=1e-2)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    lr_steps = 2 * a.engine.lr * 5
    for k in sb:
        if not sb[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        noisy = k in _NOISE_KEYS or k.startswith(("inf_net.f_mu_batchnorm.running_mean",
                                                   "inf_net.f_sigma_batchnorm.running_mean"))
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-3, atol=lr_steps if noisy else 5e-5,
                                   msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("bwdpp", ["1", "0"])
@pytest.mark.parametrize("Cdim,V", [(96, 600), (768, 9000), (100, 5000)])
def test_ctm_persistent_backward_matches_oracle(monkeypatch, Cdim, V, bwdpp):
    """ctx_bwd as one persistent workgroup per CU over equal ranges of (tile, 128-float C
    chunk) items, the next item's Wa state in flight (stage_flags bit 12, forced at small
    V), vs the (tile, chunk) grid (bwdpp = 0): the oracle's adapt_bert / input-layer
    gradients (C = 96 / 100: a partial last chunk; V = 5000: a partial last tile)."""
    monkeypatch.setenv("GFEDNTM_CTX_BWDPP", bwdpp)
    test_ctm_step_matches_oracle("combined", Cdim, V, 20, "prodLDA")


def test_ctm_persistent_backward_fused_update(monkeypatch):
    """The persistent backward's Adam epilogue (adapt_bert weight and bias, FedAvg
    pre-scale) == gradient mode + the generic Adam, over several steps."""
    monkeypatch.setenv("GFEDNTM_CTX_BWDPP", "1")
    from gfedntm_amd.ops.engine import STAGE_CTX_BWDPP
    from gfedntm_amd.models import CombinedTM
    torch.manual_seed(0)
    kw = dict(input_size=1900, contextual_size=136, n_components=30, hidden_sizes=(48, 40),
              batch_size=64, verbose=False, device="cuda", backend="fused")
    a, b = CombinedTM(**kw), CombinedTM(**kw)
    assert a.engine._m.stage_flags & STAGE_CTX_BWDPP
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    b.engine.set_update_mode(UPDATE_GRAD)
    X = random_csr(200, 1900, 40, seed=3)
    ctx = np.random.default_rng(4).standard_normal((200, 136)).astype(np.float32)
    for t in (a, b):
        t.engine.set_fedavg_scale(0.75)
        t.engine.bind_data(DeviceCSR(X, "cuda", contextual=ctx), BatchPlan.build(200, 64, 5, seed=0))
        t.engine.enable_graph(True)
    for s in range(5):
        a.engine.step(s)
        b.engine.step(s)
    torch.cuda.synchronize()
    torch.testing.assert_close(a.engine.loss_hist, b.engine.loss_hist, rtol=1e-4, atol=1e-2)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    lr_steps = 2 * a.engine.lr * 5
    for k in sb:
        if not sb[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        noisy = k in _NOISE_KEYS or k.startswith(("inf_net.f_mu_batchnorm.running_mean",
                                                   "inf_net.f_sigma_batchnorm.running_mean"))
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-3, atol=lr_steps if noisy else 5e-5,
                                   msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("B,K,V", [(64, 50, 4500), (64, 64, 3000), (32, 25, 7001), (16, 10, 700),
                                   (64, 50, 40000)])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_postfold_matches_separate_post_fwd(monkeypatch, B, K, V, dtype):
    """The strip forward with the posterior folded in (stage_flags GFK_FWD_POSTFOLD: BN of the
    heads, reparameterisation, softmax, dropout, KL, running statistics and the optimizer
    step counters computed in its theta_d staging; post_fwd not launched) matches the
    separate post_fwd kernel over several fused-update graph replays -- same workspace
    outputs for the backward, same counters, same trained state."""
    from gfedntm_amd.ops.engine import STAGE_FWD_POSTFOLD
    kw = dict(input_size=V, n_components=K, hidden_sizes=(50, 50), batch_size=B,
              verbose=False, device="cuda")
    if dtype == "bf16":
        kw["matmul_dtype"] = "bf16"
    tms = []
    for fold in ("1", "0"):
        monkeypatch.setenv("GFEDNTM_POSTFOLD", fold)
        torch.manual_seed(3)
        tm = AVITM(backend="fused", **kw)
        assert bool(tm.engine._m.stage_flags & STAGE_FWD_POSTFOLD) == (fold == "1")
        assert (abi.PH_POST_FWD in tm.engine.phases()) == (fold == "0")
        tms.append(tm)
    a, b = tms
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    X = random_csr(3 * B + 5, V, 40, seed=4)
    data = DeviceCSR(X, "cuda")
    plan = BatchPlan.build(data.n_docs, B, 5, seed=1)
    for tm in (a, b):
        tm.engine.set_fedavg_scale(0.5)
        tm.engine.bind_data(data, plan)
        tm.engine.enable_graph(True)
        for s in range(5):
            tm.engine.step(s)
    torch.cuda.synchronize()
    # (the folded statistics sum in another order: after five steps a few small-magnitude
    # heads of the tiny B = 16, K = 10 model differ at ~1e-5)
    for key in ("mu", "ls", "theta", "thetad", "kl", "bn_rstd"):
        torch.testing.assert_close(a.engine.ws[key], b.engine.ws[key], rtol=5e-4, atol=2e-5,
                                   msg=lambda m: f"ws[{key}]: {m}")
    assert int(a.engine.adam_t.item()) == int(b.engine.adam_t.item()) == 5
    torch.testing.assert_close(a.engine.adam_coef, b.engine.adam_coef, rtol=0, atol=0)
    torch.testing.assert_close(a.engine.loss_hist[:5], b.engine.loss_hist[:5], rtol=1e-5, atol=1e-3)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    for k in sa:
        if not sa[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        # (the heads' biases get a zero gradient in exact arithmetic -- batch norm removes
        # them -- so Adam steps them by +-lr on rounding noise, and the raw heads' running
        # means follow: compared at that scale)
        noisy = "bias" in k or k in _NOISE_KEYS or k.startswith((
            "inf_net.f_mu_batchnorm.running_mean", "inf_net.f_sigma_batchnorm.running_mean"))
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-4, atol=2e-3 if noisy else 5e-5,
                                   msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("V", [6000, 40000, 99000])
def test_ctm_bf16_contextual_matches_emulated_oracle(V):
    """matmul_dtype='bf16' on CombinedTM: the contextual GEMMs of ctx_fwd (A = x_ctx Wa^T + b
    and its input-layer term A Wc^T, register-streamed kernel, v_mfma_f32_16x16x32_bf16 with
    fp32 accumulation) and the decoder's theta_d beta take bf16 operands; master weights,
    Adam state and every other op stay fp32.  Oracle: the fp32 PyTorch step with exactly
    those operands rounded to bf16 (C = 768, K = 100; V = 6k / 40k / 99k -- the BASELINE
    CombinedTM class).  Reference: ctm inference_network.py:160-185."""
    import torch.nn.functional as F
    from gfedntm_amd.models import CombinedTM
    from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
    from gfedntm_amd.ops.engine import STAGE_CTX_RS
    K, Cdim, B, n_docs = 100, 768, 64, 150
    torch.manual_seed(0)
    kw = dict(input_size=V, contextual_size=Cdim, n_components=K, hidden_sizes=(50, 50),
              batch_size=B, verbose=False, device="cuda")
    fused = CombinedTM(backend="fused", matmul_dtype="bf16", **kw)
    ref = CombinedTM(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    e = fused.engine
    assert e._m.mm_bf16 == 1 and e._m.ctx_fused == 1 and e._m.stage_flags & STAGE_CTX_RS
    assert e.ctx_gemm_dtype == "bf16"
    X = random_csr(n_docs, V, 60, seed=1)
    ctx = np.random.default_rng(2).standard_normal((n_docs, Cdim)).astype(np.float32)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    plan = BatchPlan.build(data.n_docs, B, 3, seed=0)
    e.set_update_mode(UPDATE_GRAD)
    e.bind_data(data, plan)
    e.run_phases(e.phases()[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x, xc = data.dense_rows(ids), data.contextual[ids]
    model = ref.model
    model.train()
    model.zero_grad()
    net = model.inf_net
    bfr = lambda t: t + (_bf(t) - t).detach()      # noqa: E731  rounded forward, identity grad
    W = net.input_layer.weight                        # [H0, 2V]: BoW half | contextual half
    A = bfr(xc) @ bfr(net.adapt_bert.weight).t() + net.adapt_bert.bias
    z0 = x @ W[:, :V].t() + bfr(A) @ bfr(W[:, V:2 * V]).t() + net.input_layer.bias
    h = net.hiddens(net.activation(z0)) * e.ws["mask_h"][:nb]
    bn, bs = net.f_mu_batchnorm, net.f_sigma_batchnorm
    mu = F.batch_norm(net.f_mu(h), bn.running_mean, bn.running_var, training=True,
                      momentum=bn.momentum, eps=bn.eps)
    ls = F.batch_norm(net.f_sigma(h), bs.running_mean, bs.running_var, training=True,
                      momentum=bs.momentum, eps=bs.eps)
    theta = F.softmax(mu + e.ws["eps"][:nb] * torch.exp(0.5 * ls), dim=1)
    thetad = theta * e.ws["mask_t"][:nb]
    bb = model.beta_batchnorm
    logits = F.batch_norm(bfr(thetad) @ bfr(model.beta), bb.running_mean, bb.running_var,
                          training=True, momentum=bb.momentum, eps=bb.eps)
    wd = F.softmax(logits, dim=1)
    kl = kl_terms(model.prior_mean, model.prior_variance, mu, torch.exp(ls), ls, K)
    rl = reconstruction_terms(x, wd)
    w_kl = float(ref.weights.get("beta", 1.0))
    loss = (w_kl * kl + rl).sum()
    loss.backward()
    torch.testing.assert_close(e.ws["kl"][:nb], kl.detach(), rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=2e-4, atol=5e-2)
    # the adapted rows themselves: A (+ bias) per vocabulary tile in ws_actx [tile][b][64]
    act = e.ws["actx"].view(-1, B, 64)[:, :nb].permute(1, 0, 2).reshape(nb, -1)[:, :V]
    torch.testing.assert_close(act, A.detach(), rtol=1e-3, atol=1e-3)
    g = _grads_of(fused)
    for k, p in model.named_parameters():
        if k in _NOISE_KEYS:
            continue
        scale = p.grad.abs().max().item() + 1e-6
        torch.testing.assert_close(g[k], p.grad, rtol=3e-2, atol=2e-2 * scale,
                                   msg=lambda m: f"{k}: {m}")


@pytest.mark.parametrize("K,V", [(50, 2000), (100, 30000)])
def test_bf16_neurallda_matches_emulated_oracle(K, V):
    """matmul_dtype='bf16' on NeuralLDA: word_dist = theta_d beta_sm with bf16 theta_d and
    beta_sm (lda_row: per non-zero dot products, fp32 accumulation; the same bf16 beta_sm in
    d theta_d) and the backward's coefficient x theta_d product (lda_beta_bwd) on bf16
    operands.  Oracle: the fp32 step with theta_d and beta_sm rounded to bf16 before their
    product (reference decoder_network.py:127-132)."""
    import torch.nn.functional as F
    from gfedntm_amd.models.functional import encoder_forward
    from gfedntm_amd.models.networks import kl_terms, reconstruction_terms
    fused, ref = _pair("LDA", V=V, K=K, H=(50, 50), B=64, matmul_dtype="bf16")
    assert fused.engine._m.mm_bf16 == 1
    X = random_csr(150, V, 60, seed=1)
    data, plan = _bind(fused, X, B=64)
    e = fused.engine
    e.run_phases(e.phases()[:-1])
    torch.cuda.synchronize()
    nb = int(plan.size[0])
    ids = torch.from_numpy(plan.batch(0).astype(np.int64)).cuda()
    x = data.dense_rows(ids)
    model = ref.model
    model.train()
    model.zero_grad()
    mu, ls = encoder_forward(model.inf_net, x, e.ws["mask_h"][:nb])
    theta = F.softmax(mu + e.ws["eps"][:nb] * torch.exp(0.5 * ls), dim=1)
    thetad = theta * e.ws["mask_t"][:nb]
    bfr = lambda t: t + (_bf(t) - t).detach()      # noqa: E731
    bb = model.beta_batchnorm
    bnb = F.batch_norm(model.beta, bb.running_mean, bb.running_var, training=True,
                       momentum=bb.momentum, eps=bb.eps)
    wd = bfr(thetad) @ bfr(F.softmax(bnb, dim=1))
    kl = kl_terms(model.prior_mean, model.prior_variance, mu, torch.exp(ls), ls, K)
    rl = reconstruction_terms(x, wd)
    loss = (kl + rl).sum()
    loss.backward()
    torch.testing.assert_close(e.ws["rl"][:nb], rl.detach(), rtol=2e-4, atol=5e-2)
    g = _grads_of(fused)
    for k, p in model.named_parameters():
        if k in _NOISE_KEYS:
            continue
        scale = p.grad.abs().max().item() + 1e-6
        torch.testing.assert_close(g[k], p.grad, rtol=3e-2, atol=2e-2 * scale,
                                   msg=lambda m: f"{k}: {m}")
