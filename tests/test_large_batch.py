"""The fused engine's large-batch plan, 128 < batch_size <= 512 (csrc/gfk_common.h GFK_LB;
ops/engine.py FusedEngine._plan_large_batch).  The reference takes any batch_size
(avitm.py:84-85, SURVEY.md item 4 of round 4's verdict); up to 128 rows the fused kernels keep
the batch in LDS, above it the row-parallel kernels read the batch matrices from L2, the weight
jobs and NeuralLDA's beta backward stage 128-row chunks.  ProdLDA's decoder at B = 256, K <= 256
runs on two hand-written MFMA kernels (csrc/prodlda.hip prodlda_lb_fwd / prodlda_lb_bwd: the
logits GEMM + column batch-norm; the logit gradient + dbeta + d theta_d); elsewhere (B = 512,
K > 256, or GFEDNTM_LB_GEMM=1) its products are hipBLASLt GEMMs around two HIP kernels (column
batch-norm / logit gradient).

Oracle: the same PyTorch fp32 functional step as tests/test_fused_kernels.py (loss, KL, RL,
every gradient, BN running statistics, the optimizer step) at B in {256, 512} x K in {50, 200}
x V in {5k, 112k}, ProdLDA and NeuralLDA, plus a partial batch, a graph-replayed run, and
K in (256, 512] (ProdLDA: the same plan at the batch's own size) with θ inference.
"""
import numpy as np
import pytest
import torch

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
from gfedntm_amd.models import AVITM
from gfedntm_amd.ops import kernel_abi as abi
from gfedntm_amd.ops.engine import STAGE_LB, UPDATE_FUSED
from tests.helpers import random_csr
from tests.test_fused_kernels import _oracle_step

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
@pytest.mark.parametrize("B", [256, 512])
@pytest.mark.parametrize("K", [50, 200])
@pytest.mark.parametrize("V", [5000, 112000])
def test_large_batch_step_matches_oracle(model_type, B, K, V):
    _oracle_step(model_type, B, B + 37, K, (50, 50), V)


@pytest.mark.parametrize("K,V", [(100, 9000), (128, 5000), (7, 3001)])
def test_large_batch_mfma_decoder_shapes_match_oracle(K, V):
    """The MFMA decoder kernels' other instances: K in (64, 128] (16 waves, 8 k tiles), a
    partial last k tile and vocabulary tile (K = 7, V = 3001)."""
    torch.manual_seed(0)
    tm = AVITM(backend="fused", input_size=V, n_components=K, hidden_sizes=(50, 50),
               batch_size=256, verbose=False, device="cuda")
    assert tm.engine._m.lb_fused & 3 == 3
    _oracle_step("prodLDA", 256, 256 + 37, K, (50, 50), V)


@pytest.mark.parametrize("K,V", [(50, 5000), (200, 40000)])
def test_large_batch_fused_beta_adam_matches_gradient_mode(K, V):
    """B = 256 by default runs beta's Adam step (+ the FedAvg pre-scale) in prodlda_lb_bwd's
    epilogue and the rest in the generic optimizer pass (GfkModel.lb_fused bit 2); an explicit
    gradient mode materialises beta's gradient too.  Several graph-replayed steps: the same
    parameters, moments and losses."""
    from tests.test_fused_large_v import _compare, _run
    from gfedntm_amd.ops.engine import UPDATE_GRAD
    torch.manual_seed(0)
    kw = dict(input_size=V, n_components=K, hidden_sizes=(50, 50), batch_size=256,
              verbose=False, device="cuda")
    a, b = AVITM(backend="fused", **kw), AVITM(backend="fused", **kw)
    b.model.load_state_dict(a.model.state_dict())
    b.engine.seed = b.engine._m.seed = a.engine.seed
    b.engine.set_update_mode(UPDATE_GRAD)
    assert a.engine._m.lb_fused == 7 and b.engine._m.lb_fused == 3
    n_docs = 2 * 256 + 37
    X = random_csr(n_docs, V, 60, seed=4)
    data = DeviceCSR(X, "cuda")
    _run((a, b), data, BatchPlan.build(n_docs, 256, 4, seed=0))
    _compare(a, b, 4)


@pytest.mark.parametrize("K,V", [(50, 5000), (200, 40000)])
def test_large_batch_gemm_path_matches_oracle(monkeypatch, K, V):
    """B = 256 with the library-GEMM decoder forced (GFEDNTM_LB_GEMM=1): the same oracle."""
    monkeypatch.setenv("GFEDNTM_LB_GEMM", "1")
    torch.manual_seed(0)
    tm = AVITM(backend="fused", input_size=V, n_components=K, hidden_sizes=(50, 50),
               batch_size=256, verbose=False, device="cuda")
    assert tm.engine._m.lb_fused == 0 and abi.PH_LB_GEMM_FWD in tm.engine.phases()
    _oracle_step("prodLDA", 256, 256 + 37, K, (50, 50), V)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_large_batch_partial_batch_matches_oracle(model_type):
    """Fewer documents than bmax: rows >= nb are masked out of every column statistic and
    product (nb = 300 of bmax = 512)."""
    _oracle_step(model_type, 512, 300, 50, (50, 50), 7000)


def test_large_batch_plan_and_record():
    torch.manual_seed(0)
    tm = AVITM(backend="fused", input_size=5000, n_components=50, hidden_sizes=(50, 50),
               batch_size=256, verbose=False, device="cuda")
    e = tm.engine
    assert e.large_batch and e.bmax == 256 and e._m.stage_flags & STAGE_LB
    assert e.update_mode != UPDATE_FUSED
    # B = 256, K = 50: the decoder on the MFMA kernels, no library GEMM phase, one d theta_d
    # slab per persistent workgroup
    ph = e.phases()
    assert e._m.lb_fused == 7 and abi.PH_LB_GEMM_FWD not in ph and abi.PH_LB_GEMM_BWD not in ph
    assert e._m.n_dpart == e._m.dec_grid
    assert tm.engine_info["engine"] == "fused" and "large-batch" in tm.engine_info["plan"]
    assert "hipBLASLt" not in tm.engine_info["plan"]
    # B = 512: the library GEMMs around the HIP kernels
    tm2 = AVITM(backend="fused", input_size=5000, n_components=50, hidden_sizes=(50, 50),
                batch_size=512, verbose=False, device="cuda")
    ph = tm2.engine.phases()
    assert tm2.engine._m.lb_fused == 0 and tm2.engine.host_gemm_fallback
    assert ph.index(abi.PH_LB_GEMM_FWD) < ph.index(abi.PH_PRODLDA_FWD)
    assert ph.index(abi.PH_PRODLDA_BWD) < ph.index(abi.PH_LB_GEMM_BWD) < ph.index(abi.PH_POST_BWD)
    with pytest.raises(ValueError):
        e.set_update_mode(UPDATE_FUSED)


@pytest.mark.parametrize("model_type", ["prodLDA", "LDA"])
def test_large_batch_graph_training_tracks_torch(model_type):
    """30 graph-replayed steps (batch prep, the host GEMMs and the kernels in one hipGraph)
    against the PyTorch engine from the same initial weights: the loss curves agree (the
    dropout / reparameterisation draws differ, so per-step losses are compared as a trend)
    and the trained state stays finite."""
    kw = dict(input_size=3000, n_components=50, hidden_sizes=(50, 50), batch_size=256,
              model_type=model_type, verbose=False, device="cuda")
    torch.manual_seed(1)
    fused = AVITM(backend="fused", **kw)
    ref = AVITM(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    X = random_csr(256 * 4, 3000, 60, seed=3)
    losses = []
    for tm in (fused, ref):
        data = DeviceCSR(X, "cuda")
        plan = BatchPlan.build(data.n_docs, 256, 30, seed=0)
        tm.engine.bind_data(data, plan)
        if tm is fused:
            tm.engine.enable_graph(True)
        for s in range(30):
            tm.engine.step(s)
        torch.cuda.synchronize()
        losses.append(tm.engine.loss_hist[:30].detach().cpu().numpy())
    lf, lr_ = losses
    assert np.isfinite(lf).all()
    assert torch.isfinite(fused.flat.buffer).all()
    # both decrease, to within a few percent of each other
    assert lf[-5:].mean() < lf[:5].mean() and lr_[-5:].mean() < lr_[:5].mean()
    np.testing.assert_allclose(lf[-5:].mean(), lr_[-5:].mean(), rtol=0.05)


@pytest.mark.parametrize("B,K", [(64, 300), (256, 512), (100, 512)])
def test_large_k_matches_oracle(B, K):
    """K in (256, 512] (ProdLDA, bag of words) runs the large-batch plan at the batch's own
    row count (round 5 padded a smaller batch to 256 rows): same oracle."""
    from gfedntm_amd.ops.engine import BMAX_CHOICES
    torch.manual_seed(0)
    tm = AVITM(backend="fused", input_size=5000, n_components=K, hidden_sizes=(50, 50),
               batch_size=B, verbose=False, device="cuda")
    assert tm.engine.large_batch and tm.engine.bmax == next(x for x in BMAX_CHOICES if x >= B)
    _oracle_step("prodLDA", B, B + 37, K, (50, 50), 5000)


def test_large_k_theta_inference_matches_eval_encoder():
    """θ inference at K = 512 (csrc/infer.hip's 8-topics-per-lane instance): the posterior
    moments equal the eval-mode encoder's."""
    torch.manual_seed(0)
    tm = AVITM(backend="fused", input_size=3000, n_components=512, hidden_sizes=(50, 50),
               batch_size=64, verbose=False, device="cuda")
    X = random_csr(300, 3000, 40, seed=1)
    data = DeviceCSR(X, "cuda")
    tm.engine.bind_data(data, BatchPlan.build(300, 64, 5, seed=0))
    for s in range(5):
        tm.engine.step(s)
    torch.cuda.synchronize()
    mom = tm.engine.theta_infer(data, moments=True)
    tm.model.eval()
    with torch.no_grad():
        mu, ls = tm.model.inf_net(torch.from_numpy(X.toarray()).cuda())
    torch.testing.assert_close(mom[:, 0], mu, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(mom[:, 1], ls, rtol=1e-4, atol=1e-4)
