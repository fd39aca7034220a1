"""Every single-engine stage_flags bit, forced on, in the FUSED update mode (Adam and the
FedAvg pre-scale inside the kernels' epilogues) vs gradient mode + the generic optimizer
kernel -- gradient mode being what the oracle tests (test_fused_kernels.py) check against
the explicit-noise PyTorch reference.  docs/DESIGN.md "Stage bits and knobs" maps every
bit and environment knob to its test; the batched-launch bits (9, 20) are forced in
tests/test_federation_gpu.py::test_batched_large_round_variants_match_branch_round, the
large-batch plan (bit 19, gradient mode by design) in tests/test_large_batch.py.

Reference math: avitm.py:141-143 (Adam), :225 (loss); decoder_network.py:121-126.
"""
import numpy as np
import pytest

from gfedntm_amd.data.bow import BatchPlan, DeviceCSR
from gfedntm_amd.ops import engine as E
from tests.helpers import random_csr
from tests.test_fused_large_v import _compare, _run, _twins

pytestmark = pytest.mark.gpu

N_STEPS = 4

# id -> (the bit, model class name, its constructor arguments, environment, a bit that must
# be clear)
CASES = {
    "plan_weights_in_lds": (1, "AVITM", dict(input_size=2000, n_components=50), {}, 2),
    "plan_batch_from_l2": (2, "AVITM", dict(input_size=3000, n_components=200), {}, 0),
    "fwd_strip": (E.STAGE_FWD_STRIP, "AVITM", dict(input_size=5000, n_components=50), {}, 0),
    "win_sparse": (E.STAGE_WIN_SPARSE, "AVITM", dict(input_size=3000, n_components=50),
                   {"GFEDNTM_WIN_SPARSE": "1"}, 0),
    "ctx_full": (E.STAGE_CTX_FULL, "CombinedTM", dict(input_size=3000, n_components=20),
                 {"GFEDNTM_CTX_FULL": "1", "GFEDNTM_CTX_RS": "0"}, E.STAGE_CTX_RS),
    "ctx_rs": (E.STAGE_CTX_RS, "CombinedTM", dict(input_size=3000, n_components=20),
               {"GFEDNTM_CTX_FULL": "1"}, 0),
    "ctx_bwdpp": (E.STAGE_CTX_BWDPP, "CombinedTM", dict(input_size=3000, n_components=20),
                  {"GFEDNTM_CTX_BWDPP": "1"}, 0),
    "fwd_postfold": (E.STAGE_FWD_POSTFOLD, "AVITM", dict(input_size=5000, n_components=50),
                     {"GFEDNTM_POSTFOLD": "1"}, 0),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_stage_bit_fused_update_matches_gradient_mode(monkeypatch, case):
    from gfedntm_amd import models
    bit, cls_name, kw, env, clear = CASES[case]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    cls = getattr(models, cls_name)
    ctm = cls_name == "CombinedTM"
    kw = dict(kw, hidden_sizes=(50, 50), batch_size=64, verbose=False, device="cuda")
    if ctm:
        kw["contextual_size"] = 96
    a, b = _twins(cls, kw)
    sf = int(a.engine._m.stage_flags)
    assert a.engine.update_mode == E.UPDATE_FUSED
    assert sf & bit, f"{case}: stage_flags {sf:#x} lack {bit:#x}"
    assert not sf & clear, f"{case}: stage_flags {sf:#x} carry {clear:#x}"
    n_docs = 2 * 64 + 9                   # a partial last batch
    V = kw["input_size"]
    X = random_csr(n_docs, V, 50, seed=11)
    ctx = (np.random.default_rng(12).standard_normal((n_docs, 96)).astype(np.float32)
           if ctm else None)
    data = DeviceCSR(X, "cuda", contextual=ctx)
    _run((a, b), data, BatchPlan.build(n_docs, 64, N_STEPS, seed=0))
    assert np.isfinite(a.engine.loss_hist[:N_STEPS].cpu().numpy()).all()
    _compare(a, b, N_STEPS)
