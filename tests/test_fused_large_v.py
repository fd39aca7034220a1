"""The production (fused-update) step at large vocabularies vs gradient mode + the generic
optimizer kernel.

The oracle tests (test_fused_kernels.py) run every kernel in gradient mode, and the
fused-vs-gradient check there uses V = 900, a shape that never selects the large-V
kernels.  Here the engines take exactly the production kernel selections of the BASELINE
large configurations:

* ``prodlda_bwd_pipe_kernel`` (bwd_pre = 3: buffer-descriptor pipelined backward, Adam +
  the FedAvg pre-scale fused, beta row padding, dropped out-of-range rows / stores);
* ``bwd_pre = 2`` at B = 32;
* the sparse W_in tiles (STAGE_WIN_SPARSE; fused mode: the second moment in LDS, gradient
  mode: in registers);
* odd K and V % 64 != 0 (padding columns and a partial last vocabulary tile);
* CombinedTM K = 100, C = 768, V = 74k (ctx_fwd full tiles, ctx_bwd Adam epilogue).

Several graph-replayed steps with the FedAvg pre-scale on; parameters, moments and batch-
norm buffers must agree, and beta's padding columns (and their Adam moments) must stay
exactly 0.  Reference math: avitm.py:141-143 (Adam, betas = (momentum, 0.99)), :225 (loss);
decoder_network.py:121-126 (ProdLDA decoder).
"""
import numpy as np
import pytest
import torch

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
from gfedntm_amd.models import AVITM
from gfedntm_amd.ops.engine import STAGE_WIN_SPARSE, UPDATE_FUSED, UPDATE_GRAD
from tests.helpers import random_csr

pytestmark = pytest.mark.gpu

_NOISE_KEYS = ("inf_net.f_mu.bias", "inf_net.f_sigma.bias", "prior_mean")
N_STEPS = 6


def _twins(cls, kw):
    torch.manual_seed(0)
    a, b = cls(backend="fused", **kw), cls(backend="fused", **kw)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    assert a.engine.update_mode == UPDATE_FUSED
    b.engine.set_update_mode(UPDATE_GRAD)
    return a, b


def _run(tms, data, plan):
    for tm in tms:
        tm.engine.set_fedavg_scale(0.75)
        tm.engine.bind_data(data, plan)
        tm.engine.enable_graph(True)
    for s in range(plan.n_steps):
        for tm in tms:
            tm.engine.step(s)
    torch.cuda.synchronize()


def _compare(a, b, n_steps):
    torch.testing.assert_close(a.engine.loss_hist[:n_steps], b.engine.loss_hist[:n_steps],
                               rtol=1e-4, atol=1e-2)
    # the same Adam arithmetic inlined into two kernels may differ by an ulp (FP
    # contraction); tensors whose true gradient is 0 (rounding noise) then drift by up to
    # lr per step after Adam's normalisation
    sa, sb = a.model.state_dict(), b.model.state_dict()
    lr_steps = 2 * a.engine.lr * n_steps
    for k in sb:
        if not sb[k].is_floating_point():
            assert torch.equal(sa[k], sb[k]), k
            continue
        noisy = k in _NOISE_KEYS or k.startswith(("inf_net.f_mu_batchnorm.running_mean",
                                                   "inf_net.f_sigma_batchnorm.running_mean"))
        torch.testing.assert_close(sa[k], sb[k], rtol=1e-3, atol=lr_steps if noisy else 5e-5,
                                   msg=lambda m: f"{k}: {m}")
    for buf in ("exp_avg", "exp_avg_sq"):
        for k in ("beta", "inf_net.input_layer.weight"):
            fa = a.engine.view_like(getattr(a.engine, buf), k)
            fb = b.engine.view_like(getattr(b.engine, buf), k)
            scale = float(fb.abs().max()) + 1e-12
            torch.testing.assert_close(fa, fb, rtol=1e-2, atol=1e-4 * scale,
                                       msg=lambda m: f"{buf}[{k}]: {m}")


def _assert_beta_padding_zero(tm):
    e = tm.engine
    s = e.flat.slots["beta"]
    if not s.ld or s.ld == s.shape[1]:
        return
    V = s.shape[1]
    for buf in (e.flat.buffer, e.exp_avg, e.exp_avg_sq):
        raw = e.raw_like(buf, "beta")
        pad = raw[:, V:]
        assert pad.numel() > 0
        assert int(torch.count_nonzero(pad)) == 0, "beta padding columns were written"


@pytest.mark.parametrize("B,K,V,win", [
    (64, 200, 40000, "dense"),       # bwd_pre = 3, dense W_in tiles (the auto choice here)
    (64, 200, 112000, "auto"),       # the BASELINE large config: sparse W_in tiles (LDS v)
    (32, 200, 40000, "sparse"),      # B = 32: bwd_pre = 2
    (64, 199, 40001, "sparse"),      # odd K, V % 64 != 0: padded rows, partial last tile
])
def test_large_v_fused_matches_gradient_mode(monkeypatch, B, K, V, win):
    if win == "dense":
        monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "0")
    elif win == "sparse":
        monkeypatch.setenv("GFEDNTM_WIN_SPARSE", "1")
    kw = dict(input_size=V, n_components=K, hidden_sizes=(50, 50), batch_size=B,
              verbose=False, device="cuda")
    a, b = _twins(AVITM, kw)
    for tm in (a, b):
        m = tm.engine._m
        assert m.n_dpart < m.n_tiles, "expected the persistent k-range backward"
        assert m.bwd_pre == (3 if B == 64 else 2), m.bwd_pre
        sparse = bool(m.stage_flags & STAGE_WIN_SPARSE)
        assert sparse == (win != "dense"), win
    n_docs = 3 * B + 7
    X = random_csr(n_docs, V, 60, seed=2)
    data = DeviceCSR(X, "cuda")
    plan = BatchPlan.build(n_docs, B, N_STEPS, seed=0)
    _run((a, b), data, plan)
    assert np.isfinite(a.engine.loss_hist[:N_STEPS].cpu().numpy()).all()
    _compare(a, b, N_STEPS)
    _assert_beta_padding_zero(a)
    _assert_beta_padding_zero(b)


@pytest.mark.parametrize("rs,V", [("0", 74000), ("1", 74000), ("1", 69600)])
def test_ctm_large_v_fused_matches_gradient_mode(monkeypatch, rs, V):
    """CombinedTM K = 100, C = 768, V = 74k (the BASELINE CTM class): ctx_fwd full tiles,
    Adam in ctx_bwd (adapt_bert) and win_update (both input-layer halves) vs gradient mode;
    rs = 1: the register-streamed forward (18-19 units per workgroup on 256 CUs: waves with
    two; V = 69.6k: 16-17, the 17th unit split by phase over three helper waves); rs = 0: one
    workgroup per tile."""
    from gfedntm_amd.models import CombinedTM
    from gfedntm_amd.ops.engine import STAGE_CTX_FULL, STAGE_CTX_RS
    monkeypatch.setenv("GFEDNTM_CTX_RS", rs)
    K, Cdim, B = 100, 768, 64
    kw = dict(input_size=V, contextual_size=Cdim, n_components=K, hidden_sizes=(50, 50),
              batch_size=B, verbose=False, device="cuda")
    a, b = _twins(CombinedTM, kw)
    assert a.engine._m.ctx_fused == 1 and a.engine._m.stage_flags & STAGE_CTX_FULL
    assert bool(a.engine._m.stage_flags & STAGE_CTX_RS) == (rs == "1")
    n_docs = 2 * B + 5
    X = random_csr(n_docs, V, 60, seed=3)
    ctx = np.random.default_rng(4).standard_normal((n_docs, Cdim)).astype(np.float32)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    plan = BatchPlan.build(n_docs, B, 4, seed=0)
    _run((a, b), data, plan)
    _compare(a, b, 4)
    fa = a.engine.view_like(a.engine.exp_avg, "inf_net.adapt_bert.weight")
    fb = b.engine.view_like(b.engine.exp_avg, "inf_net.adapt_bert.weight")
    torch.testing.assert_close(fa, fb, rtol=1e-2, atol=1e-4 * (float(fb.abs().max()) + 1e-12))
    _assert_beta_padding_zero(a)
