"""Every solver the reference offers (avitm.py:141-153: adam, sgd, adagrad, adadelta,
rmsprop) on the fused engine: the kernels write gradients and the generic optimizer
kernel (csrc/gfk_common.h adam_block, GFK_SOLVER_*) applies the update rule; the
result is compared with the torch optimizer the reference constructs, fed the same
gradients, over two steps (so the optimizer state is exercised), and the engine's
state_dict is checked against the torch optimizer's layout.
"""
import numpy as np
import pytest
import torch

from gfedntm_amd.federation import wire
from gfedntm_amd.models.engine import make_optimizer

SOLVERS = ["sgd", "adagrad", "adadelta", "rmsprop", "adam"]


@pytest.mark.parametrize("solver", SOLVERS)
def test_wire_codec_accepts_every_solver_state(solver):
    """The reference OptUpdate message is Adam's: other solvers' param groups still
    encode (their per-tensor state is not carried)."""
    p = torch.nn.Parameter(torch.randn(6))
    opt = make_optimizer([p], solver, 2e-3, 0.99)
    p.grad = torch.randn(6)
    opt.step()
    msg = wire.adam_update_from_state_dict(opt.state_dict())
    assert abs(msg.adamUpdate.paramGroups.lr - 2e-3) < 1e-9
    assert len(msg.adamUpdate.state.contentState) == (1 if solver == "adam" else 0)


@pytest.mark.parametrize("solver", SOLVERS)
def test_fused_param_group_matches_torch(solver):
    """The fused engine's optimizer param group has the installed torch optimizer's keys
    and the reference's hyperparameters (avitm.py:141-153)."""
    from types import SimpleNamespace
    from gfedntm_amd.ops.engine import FusedAdamState, solver_hparams

    hp = solver_hparams(solver, 0.99)
    e = SimpleNamespace(solver=solver, lr=2e-3, weight_decay=0.0, **hp)
    pg = FusedAdamState(e).param_groups[0]
    p = torch.nn.Parameter(torch.zeros(3))
    tg = make_optimizer([p], solver, 2e-3, 0.99).param_groups[0]
    assert set(pg) == set(tg) - {"params"}
    for k, v in tg.items():
        if k != "params":
            assert pg[k] == pytest.approx(v) if isinstance(v, float) else pg[k] == v, k


@pytest.mark.gpu
@pytest.mark.parametrize("model_type", ["prodLDA", "LDA", "combined", "zeroshot"])
@pytest.mark.parametrize("solver", SOLVERS)
def test_fused_solver_matches_torch_optimizer(solver, model_type):
    from gfedntm_amd.models import AVITM, CombinedTM, ZeroShotTM
    from gfedntm_amd.ops import kernel_abi as abi
    from gfedntm_amd.ops.engine import UPDATE_FUSED, UPDATE_GRAD
    from tests.helpers import random_csr
    from gfedntm_amd.data.bow import BatchPlan, DeviceCSR

    torch.manual_seed(0)
    kw = dict(input_size=700, n_components=20, model_type=model_type, hidden_sizes=(32, 24),
              batch_size=64, solver=solver, lr=2e-3, momentum=0.99, verbose=False,
              device="cuda", reduce_on_plateau=True)
    ctx = None
    if model_type in ("combined", "zeroshot"):
        cls = CombinedTM if model_type == "combined" else ZeroShotTM
        kw.update(model_type="prodLDA", contextual_size=96)
        ctx = np.random.default_rng(4).standard_normal((200, 96)).astype(np.float32)
    else:
        cls = AVITM
    fused = cls(backend="fused", **kw)
    assert fused.backend == "fused"
    ref = cls(backend="torch", **kw)
    ref.model.load_state_dict(fused.model.state_dict())
    e = fused.engine
    assert type(e).__name__ == "FusedEngine"
    expect_mode = UPDATE_FUSED if solver == "adam" else UPDATE_GRAD
    assert e.update_mode == expect_mode
    if solver != "adam":
        with pytest.raises(ValueError):
            e.set_update_mode(UPDATE_FUSED)
    e.set_update_mode(UPDATE_GRAD)
    X = random_csr(200, 700, 40, seed=1)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    e.bind_data(data, BatchPlan.build(data.n_docs, 64, 3, seed=0))
    phases = e.phases()
    assert phases[-1] == abi.PH_ADAM
    for _ in range(2):
        e.run_phases(phases[:-1])
        torch.cuda.synchronize()
        for k, p in ref.model.named_parameters():
            p.grad = e.gradient(k).detach().clone()
        ref.optimizer.step()
        e.run_phases([abi.PH_ADAM])
        torch.cuda.synchronize()
        sd_f = fused.model.state_dict()
        for k, p in ref.model.named_parameters():
            torch.testing.assert_close(sd_f[k], p.detach(), rtol=1e-4, atol=1e-5,
                                       msg=lambda m: f"{solver} {k}: {m}")
        # keep both sides on identical parameters (BN statistics included)
        ref.model.load_state_dict(fused.model.state_dict())
    assert float(e.grad.abs().max().item()) == 0.0
    # state_dict: torch layout of the same solver, values equal to torch's state
    sd_e, sd_t = e.optimizer_state_dict(), ref.optimizer.state_dict()
    assert set(sd_e["param_groups"][0]) == set(sd_t["param_groups"][0])
    for i, st in sd_t["state"].items():
        assert set(sd_e["state"][i]) == set(st), (solver, set(sd_e["state"][i]), set(st))
        for key, val in st.items():
            if key == "step":
                assert float(sd_e["state"][i][key]) == float(val)
                continue
            # ulp-level differences in sqrt / division order, amplified on the
            # near-zero gradients of the rounding-noise tensors (test_fused_kernels)
            atol = 1e-5 * float(val.abs().max()) + 1e-6
            torch.testing.assert_close(sd_e["state"][i][key], val, rtol=1e-3, atol=atol,
                                       msg=lambda m: f"{solver} state {i}.{key}: {m}")
    # torch -> engine round trip (checkpoint resume)
    ref.optimizer.load_state_dict(sd_e)
    e.load_optimizer_state_dict(sd_t)
    sd_back = e.optimizer_state_dict()
    for i, st in sd_e["state"].items():
        for key, val in st.items():
            if key != "step":
                torch.testing.assert_close(sd_back["state"][i][key], sd_t["state"][i][key],
                                           rtol=0, atol=0)
    assert np.isclose(sd_back["param_groups"][0]["lr"], 2e-3)
