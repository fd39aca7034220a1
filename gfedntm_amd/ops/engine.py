"""Fused HIP engine: the MI355X local step.

One local step (reference federated_avitm.py:51-83: zero_grad -> forward ->
loss -> backward -> Adam) runs as a short chain of hand-written CDNA4 kernels
launched from C++ (csrc/step.cpp) on the current HIP stream:

  ProdLDA:   enc_in -> post_fwd -> prodlda_fwd -> row_loss -> prodlda_bwd
             -> row_bwd -> post_bwd -> win_update
  NeuralLDA: lda_beta_fwd -> enc_in -> post_fwd -> lda_row_loss_bwd -> row_bwd
             -> post_bwd -> lda_beta_bwd -> win_update

In the fused update mode (AVITM default) there is no optimizer kernel: every
tensor's Adam update (and the FedAvg pre-scale w_i = n_i / sum n of the shared
tensors) is applied in the epilogue of the kernel that completes its gradient
(beta in prodlda_bwd / lda_beta_bwd; W_in and the small MLP tensors -- as batch-reduction
GEMM tiles and column sums -- in win_update).  The gradient mode writes gradients into a flat buffer instead and
appends the generic multi-segment Adam kernel (used by NeuralLDA, by the tests
as the oracle of the fused epilogues, and by gradient-sharing variants).

Everything the step reads or writes is device resident: the CSR shard, the
batch plan, the step / Adam counters and bias-correction powers (advanced by
the kernels themselves), the Philox RNG (keyed by seed and step), the loss
history.  That makes the whole step capturable once into a hipGraph and
replayed with no host work at all.

Parameters live in the model's :class:`FlatState` buffer (views back to the
reference-keyed nn.Module); gradients and Adam moments use the same layout, so
kernels reach a parameter's moments at a fixed offset and the FedAvg
collective is one contiguous all-reduce of ``flat.shared``.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..data.bow import BatchPlan, DeviceCSR
from ..models.engine import EngineBase
from ..utils.flat import ALIGN, slot_view
from ..utils.misc import graph_capture
from . import kernel_abi as abi
from . import native

BMAX_CHOICES = (16, 32, 64, 128, 256, 512)
# batch sizes above this run the large-batch plan (csrc/gfk_common.h GFK_LB)
LB_MIN_BMAX = 256
LDS_LIMIT = 160 * 1024
VB = 64
# stage_flags plans, fastest first: bit 0 = MLP weights staged in LDS (enc_in,
# post_bwd); bit 1 = the posterior kernels read the [B, K] batch matrices from L2
# instead of staging them (large K).  Plan 3 (weights staged, batch matrices from L2)
# is the large-K plan: the head weights [K, H] feed post_bwd's GEMVs from LDS instead
# of one dependent L2 round trip per pass
STAGE_PLANS = (1, 0, 3, 2)
STAGE_FWD_STRIP = 4               # bit 2: ProdLDA strip forward (csrc/prodlda.hip)
STAGE_WIN_SPARSE = 16             # bit 4: sparse W_in tiles (csrc/update.hip win_tile_sparse)
STAGE_CTX_FULL = 32               # bit 5: CombinedTM forward, one workgroup per tile (csrc/ctx.hip)
STAGE_WIN_BATCH8 = 512            # bit 9: batched launches: win_update's 8-wave tile shape
STAGE_CTX_BWDPP = 4096            # bit 12: CombinedTM backward, persistent pipelined shape (csrc/ctx.hip)
STAGE_CTX_RS = 32768              # bit 15: CombinedTM forward, Wa register-streamed (csrc/ctx.hip)
STAGE_FWD_POSTFOLD = 65536        # bit 16: the strip forward computes post_fwd (csrc/prodlda.hip FP)
STAGE_LB = 524288                 # bit 19: the large-batch plan (bmax 256 / 512, csrc/gfk_common.h)
STAGE_POST_ROWS2 = 1048576        # bit 20: batched post_bwd, two rows per workgroup; its batch-level
                                  #         workgroup in row_bwd (csrc/posterior.hip)
# (removed in round 6, measured not faster: bits 3 / 8 the strip forward's 8-wave whole-block
# prefetch vs its ring (now the only variant), bit 6 the plain rolling prefetch, 7 the split W_in update, 10 the sparse tile's register second moment
# as a knob, 11 / 13 the LDS-DMA balanced CombinedTM forwards, 14 the persistent Wc update,
# 17 the moved batch-level workgroup on its own, 18 the one-range backward walking tiles)


def engine_bmax(tm) -> int:
    """Rows the engine's workspaces are sized for: the batch size rounded up to a kernel
    instance.  (K > 256 runs the large-batch plan at the batch's own size since round 6;
    round 5 padded it to 256 rows.)"""
    return next(x for x in BMAX_CHOICES if x >= tm.batch_size)


def uses_large_batch_plan(tm, bmax: int) -> bool:
    """The large-batch plan (csrc/gfk_common.h GFK_LB): 256 / 512 rows, or K > 256 (its
    posterior / decoder shapes take K <= 512) at any batch size."""
    return bmax >= LB_MIN_BMAX or tm.n_components > 256


def _explain(ok: bool, why: str, explain: bool) -> bool:
    if not ok and explain:
        raise RuntimeError(f"fused engine unsupported: {why}")
    return ok


def supports(tm, explain: bool = False) -> bool:
    """Whether the fused kernels cover this model configuration."""
    dev = getattr(tm, "device", torch.device("cpu"))
    checks = [
        (dev.type == "cuda", "needs a GPU device"),
        (native.kernels_available(), "kernel library not built"),
        (tm.solver in abi.SOLVER_CODES, f"solver {tm.solver} not fused"),
        (tm.activation in abi.ACT_CODES, f"activation {tm.activation} not fused"),
        (tm.batch_size <= BMAX_CHOICES[-1], f"batch_size > {BMAX_CHOICES[-1]}"),
        (tm.n_components <= 512, "n_components > 512"),
        (max(tm.hidden_sizes) <= 512 and len(tm.hidden_sizes) <= abi.MAX_LAYERS,
         "hidden layers too wide / too many"),
        (getattr(tm, "label_size", 0) <= 256, "label_size > 256"),
    ]
    # reduce_on_plateau needs nothing here: the reference builds ReduceLROnPlateau
    # (avitm.py:156-157) but never calls scheduler.step(), so the lr never changes
    for ok, why in checks:
        if not _explain(ok, why, explain):
            return False
    bmax = engine_bmax(tm)
    if tm.n_components > 256 and (tm.kind == "ctm" or tm.model_type.lower() != "prodlda"):
        return _explain(False, "n_components > 256 needs the large-batch plan: ProdLDA, bag-of-words",
                        explain)
    if uses_large_batch_plan(tm, bmax):
        # the large-batch plan: bag-of-words AVITM, the sparse W_in tiles (H0 <= 64), the
        # [bmax, ldb] logit matrix addressed with 32-bit buffer offsets
        lb = [(tm.kind != "ctm", "batch_size > 128 needs a bag-of-words AVITM model"),
              (tm.hidden_sizes[0] <= 64, "batch_size > 128 needs hidden_sizes[0] <= 64"),
              (4 * bmax * beta_ld(tm.input_size) < (1 << 31), "batch_size x vocabulary too large")]
        for ok, why in lb:
            if not _explain(ok, why, explain):
                return False
    need = lds_required(tm, bmax)
    return _explain(need <= LDS_LIMIT, f"LDS budget exceeded ({need} B)", explain)


UPDATE_GRAD, UPDATE_FUSED = 0, 1


def theta_stride(K: int) -> int:
    """Row stride of the dropped-out theta workspace: K rounded up to 2 x odd, so the
    decoder MFMAs' A-role reads (16 rows x 2 k per half-wave, ds_read_b32: bank =
    dword % 32) land on 32 distinct banks (B * kt stays a multiple of 4 for LDS-DMA)."""
    kt = -(-K // 2) * 2
    return kt + 2 if (kt // 2) % 2 == 0 else kt


# beta rows padded to whole 64-column tiles (256 B) from this vocabulary size on
# (utils/flat.py): the large-V kernels' RMW tiles never split a cache line with another
# tile, and a tile's columns past V are row padding (prodlda_bwd_pipe_kernel stores there)
BETA_PAD_MIN_V = 8192
BETA_PAD = 64                     # whole 64-column tiles (the pipelined backward's stores rely on it)


def beta_ld(V: int) -> int:
    """beta's row stride in the fused engine's flat layout."""
    return -(-V // BETA_PAD) * BETA_PAD if V >= BETA_PAD_MIN_V else V


def _shape_model(tm, bmax: int) -> "abi.GfkModel":
    m = abi.GfkModel()
    hs = list(tm.hidden_sizes)
    m.bmax, m.V, m.K, m.n_hidden = bmax, tm.input_size, tm.n_components, len(hs)
    m.ldb = beta_ld(m.V)
    for i, h in enumerate(hs):
        m.H[i] = h
    m.kind = abi.KIND_PRODLDA if tm.model_type.lower() == "prodlda" else abi.KIND_LDA
    m.mm_bf16 = int(getattr(tm, "matmul_dtype", "fp32") == "bf16")
    m.kt = theta_stride(m.K)
    m.vb, m.n_tiles = VB, -(-m.V // VB)
    m.n_dpart = m.n_tiles if m.kind == abi.KIND_PRODLDA else 1
    return m


def _force_k_split(lib, m) -> bool:
    """ProdLDA backward at large K with few vocab tiles: the one-range shape (a workgroup
    per tile, all K topics of theta_d and the beta tile in LDS) exceeds the LDS at
    K = 256, B >= 64.  Then use the 4-k-range shape anyway (persistent, n_dpart < n_tiles
    slabs; ~71 KB at K = 256).  Returns True when it set n_dpart so."""
    if m.kind != abi.KIND_PRODLDA or m.n_tiles < 2 or -(-m.K // 16) < 4:
        return False
    m.n_dpart = m.n_tiles
    if lib.gfk_smem_required(C.byref(m), 1) <= LDS_LIMIT:
        return False
    m.n_dpart = m.n_tiles - 1
    return True


def lds_required(tm, bmax: int) -> int:
    """Largest dynamic LDS any fused kernel needs for this model (weights unstaged),
    as computed by the kernel library itself."""
    m = abi.GfkModel()
    hs = list(tm.hidden_sizes)
    m.bmax, m.V, m.K, m.n_hidden = bmax, tm.input_size, tm.n_components, len(hs)
    m.ldb = beta_ld(m.V)
    for i, h in enumerate(hs):
        m.H[i] = h
    m.kind = abi.KIND_PRODLDA if tm.model_type.lower() == "prodlda" else abi.KIND_LDA
    m.mm_bf16 = int(getattr(tm, "matmul_dtype", "fp32") == "bf16")
    m.kt = theta_stride(m.K)
    m.vb, m.n_tiles = VB, -(-m.V // VB)
    m.n_dpart = m.n_tiles if m.kind == abi.KIND_PRODLDA else 1
    lib = native.kernels()
    which = (0, 1) if m.kind == abi.KIND_PRODLDA else (2, 3)
    if uses_large_batch_plan(tm, bmax):
        need = 0
        for win in (0, STAGE_WIN_SPARSE):        # (either W_in tile shape)
            m.stage_flags, m.n_dpart = 2 | STAGE_LB | win, 1
            need = max(need, int(max(lib.gfk_smem_required(C.byref(m), w) for w in which + (4, 5, 7))))
        return need
    _force_k_split(lib, m)
    need = 0
    for flags in (0, 2):                 # weights unstaged; batch matrices in LDS, then in L2
        m.stage_flags = flags
        need = int(max(lib.gfk_smem_required(C.byref(m), w) for w in which + (4, 5, 7)))
        if need <= LDS_LIMIT:
            break
    return need


# Per solver: hyperparameters as the reference constructs the torch optimizer
# (avitm.py:141-153: Adam betas=(momentum, 0.99), SGD / RMSprop momentum=momentum,
# torch defaults otherwise), and the torch state names of the two flat state buffers.
SOLVER_STATE = {
    "adam": (("exp_avg", "exp_avg"), ("exp_avg_sq", "exp_avg_sq")),
    "sgd": (("momentum_buffer", "exp_avg"),),
    "adagrad": (("sum", "exp_avg_sq"),),
    "adadelta": (("square_avg", "exp_avg_sq"), ("acc_delta", "exp_avg")),
    "rmsprop": (("square_avg", "exp_avg_sq"), ("momentum_buffer", "exp_avg")),
}


def solver_hparams(solver: str, momentum: float) -> Dict[str, float]:
    """beta1 / beta2 / eps of the generic optimizer kernel for ``solver``."""
    return {"adam": dict(beta1=momentum, beta2=0.99, eps=1e-8),
            "sgd": dict(beta1=momentum, beta2=0.0, eps=0.0),
            "adagrad": dict(beta1=0.0, beta2=0.0, eps=1e-10),
            "adadelta": dict(beta1=0.0, beta2=0.9, eps=1e-6),
            "rmsprop": dict(beta1=momentum, beta2=0.99, eps=1e-8)}[solver]


class FusedAdamState:
    """torch.optim-compatible view of the flat optimizer state (for checkpoints and
    the reference OptUpdate wire message): the state_dict has the keys and
    param_group fields of the torch optimizer of the same solver."""

    def __init__(self, engine: "FusedEngine"):
        self.e = engine
        self.param_groups = [self._group()]

    def _group(self):
        e = self.e
        # the installed torch optimizer's defaults give the exact key set of its
        # param groups (it changes across torch versions); our values override
        from ..models.engine import make_optimizer
        dummy = torch.nn.Parameter(torch.zeros(1))
        base = dict(make_optimizer([dummy], e.solver, e.lr, e.beta1 or 0.0).defaults)
        common = {"lr": e.lr, "weight_decay": e.weight_decay}
        extra = {
            "adam": {"betas": (e.beta1, e.beta2), "eps": e.eps, "amsgrad": False,
                     "capturable": False, "fused": None},
            "sgd": {"momentum": e.beta1, "dampening": 0, "nesterov": False, "fused": None},
            "adagrad": {"lr_decay": 0, "initial_accumulator_value": 0, "eps": e.eps,
                        "fused": None},
            "adadelta": {"rho": e.beta2, "eps": e.eps, "capturable": False},
            "rmsprop": {"alpha": e.beta2, "eps": e.eps, "momentum": e.beta1,
                        "centered": False, "capturable": False},
        }[e.solver]
        return {**base, **common, **{k: v for k, v in extra.items() if k in base}}

    def state_dict(self):
        e = self.e
        t = int(e.adam_t.item())
        state = {}
        if t > 0:
            for i, (name, _) in enumerate(e.param_order):
                st = {} if e.solver == "sgd" else {"step": torch.tensor(float(t))}
                for key, buf in SOLVER_STATE[e.solver]:
                    st[key] = e.view_like(getattr(e, buf), name).detach().clone()
                state[i] = st
        pg = dict(self.param_groups[0])
        pg["params"] = list(range(len(e.param_order)))
        return {"state": state, "param_groups": [pg]}

    def load_state_dict(self, sd):
        e = self.e
        pg = sd["param_groups"][0]
        e.lr = float(pg.get("lr", e.lr))
        if e.solver == "adam":
            e.beta1, e.beta2 = (float(x) for x in pg.get("betas", (e.beta1, e.beta2)))
        e.beta1 = float(pg.get("momentum", e.beta1))
        e.beta2 = float(pg.get("rho", pg.get("alpha", e.beta2)))
        e.eps = float(pg.get("eps", e.eps))
        e.weight_decay = float(pg.get("weight_decay", e.weight_decay))
        self.param_groups = [self._group()]
        e.exp_avg.zero_()
        e.exp_avg_sq.zero_()
        t = int(e.adam_t.item()) if e.solver == "sgd" else 0
        for i, (name, _) in enumerate(e.param_order):
            st = sd["state"].get(i, sd["state"].get(str(i)))
            if not st:
                continue
            for key, buf in SOLVER_STATE[e.solver]:
                if st.get(key) is not None:
                    e.view_like(getattr(e, buf), name).copy_(torch.as_tensor(st[key]))
            if "step" in st:
                step = st["step"]
                t = int(step.item() if isinstance(step, torch.Tensor) else step)
        e.set_adam_t(t)
        e._rebuild_adam()

    def zero_grad(self, set_to_none: bool = False):
        self.e.grad.zero_()


class FusedEngine(EngineBase):
    """Fused-kernel local step for AVITM (ProdLDA / NeuralLDA) and CTM encoders."""

    def __init__(self, tm):
        super().__init__(tm.model, tm.flat, float(tm.weights.get("beta", 1)))
        self.tm = tm
        self.kind = tm.kind
        self.lib = native.kernels()
        dev = self.device
        self.grad = torch.zeros_like(self.flat.buffer)
        self.exp_avg = torch.zeros_like(self.flat.buffer)
        self.exp_avg_sq = torch.zeros_like(self.flat.buffer)
        self.d_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.adam_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.adam_pow = torch.ones(2, dtype=torch.float64, device=dev)     # beta1^t, beta2^t
        self.adam_coef = torch.zeros(2, dtype=torch.float32, device=dev)   # see csrc/gfk_common.h
        # CTM contextual path on the fused kernels: CombinedTM (ctx_fwd / ctx_bwd) and
        # ZeroShotTM (dense input layer in enc_in / win_update).  _plan_ctx may fall back
        # to host-issued GEMMs for shapes outside the kernels' plan; that path runs in
        # gradient mode with the generic optimizer kernel
        self.ctx_fused = tm.kind == "ctm"
        self.ctx_fallback_reason: Optional[str] = None
        # Adam runs in the kernels' epilogues; the other solvers in gradient mode
        # (kernels write gradients, the generic optimizer kernel applies the rule)
        self.solver = tm.solver
        self.update_mode = (UPDATE_FUSED if (tm.kind != "ctm" or self.ctx_fused)
                            and self.solver == "adam" else UPDATE_GRAD)
        hp = solver_hparams(self.solver, float(tm.momentum))
        self.lr, self.beta1, self.beta2 = float(tm.lr), hp["beta1"], hp["beta2"]
        self.eps, self.weight_decay = hp["eps"], 0.0
        self.fedavg_scale: Optional[float] = None
        self.bmax = engine_bmax(tm)
        # the large-batch plan (bmax 256 / 512): library GEMMs for the decoder products,
        # gradient mode (the kernels write gradients; the generic optimizer kernel follows)
        self.large_batch = uses_large_batch_plan(tm, self.bmax)
        if self.large_batch:
            self.update_mode = UPDATE_GRAD
        self.param_order: List[Tuple[str, torch.nn.Parameter]] = list(self.model.named_parameters())
        self.optimizer = FusedAdamState(self)
        self.seed = int(torch.randint(0, 2**62, (1,)).item())
        self._host_step = 0
        self.graph_enabled = False
        self._graph = None
        self._graphs_k = {}
        self.graph_gen = 0
        self._graph_key = None
        self._comm = None
        self._m = abi.GfkModel()
        self._a = abi.GfkAdam()
        self._u = abi.GfkUpdate()
        # the kernels read the model / update descriptors from device memory (one entry per
        # client of a batched launch: csrc gfk_dev / gfk_grid); this engine's own copies,
        # uploaded whenever the host structs change (_sync_dev)
        self._dev_m = torch.zeros(C.sizeof(abi.GfkModel), dtype=torch.uint8, device=self.device)
        self._dev_u = torch.zeros(C.sizeof(abi.GfkUpdate), dtype=torch.uint8, device=self.device)
        self._dev_bytes = (None, None)
        self._m.dev, self._m.dev_upd, self._m.n_batch = (self._dev_m.data_ptr(),
                                                         self._dev_u.data_ptr(), 1)
        self._phases = None
        self._nb_int = {}
        self._fill_static()
        self._rebuild_adam()

    # ------------------------------------------------------------------ layout
    def view_like(self, buf: torch.Tensor, key: str) -> torch.Tensor:
        """The slot of ``key`` inside another flat-layout buffer (grad, m, v)."""
        return slot_view(buf, self.flat.slots[key])

    def gradient(self, key: str) -> torch.Tensor:
        """The pending gradient of parameter ``key`` (gradient mode, before Adam
        consumes it)."""
        if self.update_mode != UPDATE_GRAD:
            raise RuntimeError("gradients are only materialised in gradient mode")
        return self.view_like(self.grad, key)

    def set_update_mode(self, mode: int):
        """UPDATE_FUSED: optimizer in the kernel epilogues; UPDATE_GRAD: kernels write
        gradients and the generic Adam kernel follows."""
        if mode == UPDATE_FUSED and self.kind == "ctm" and not self.ctx_fused:
            raise ValueError("the fused update mode needs the fused contextual path")
        if mode == UPDATE_FUSED and self.large_batch:
            raise ValueError("the large-batch plan runs in gradient mode")
        if mode == UPDATE_FUSED and self.solver != "adam":
            raise ValueError(f"the fused update mode is Adam only (solver {self.solver})")
        self.update_mode = mode
        self._m.update_mode = mode
        if self.large_batch and mode == UPDATE_GRAD:
            # an explicit gradient mode materialises every gradient, beta's included (the
            # oracle tests, --agg grads): beta's Adam leaves the large-batch backward
            self._m.lb_fused &= ~4
        self._rebuild_adam()

    def set_adam_t(self, t: int):
        """Set the optimizer step count and the device bias-correction state."""
        self.adam_t.fill_(t)
        p1, p2 = float(self.beta1) ** t, float(self.beta2) ** t
        self.adam_pow.copy_(torch.tensor([p1, p2], dtype=torch.float64))
        if t > 0:
            self.adam_coef.copy_(torch.tensor([self.lr / (1.0 - p1), 1.0 / np.sqrt(1.0 - p2)],
                                              dtype=torch.float32))

    def _ptr(self, buf, key):
        if key not in self.flat.slots:
            return None
        return buf.data_ptr() + 4 * self.flat.slots[key].offset

    def _fill_static(self):
        tm, m, model = self.tm, self._m, self.model
        net = model.inf_net
        hs = list(tm.hidden_sizes)
        m.bmax, m.V, m.K, m.n_hidden = self.bmax, tm.input_size, tm.n_components, len(hs)
        # beta's row stride (a padded slot: rows start on 128-B lines, utils/flat.py)
        bs = self.flat.slots.get("beta")
        m.ldb = int(bs.ld or bs.shape[1]) if bs is not None else int(m.V)
        for i, h in enumerate(hs):
            m.H[i] = h
        m.act = abi.ACT_CODES[tm.activation]
        m.mm_bf16 = int(getattr(tm, "matmul_dtype", "fp32") == "bf16")
        m.kind = abi.KIND_PRODLDA if model.is_prodlda else abi.KIND_LDA
        if self.kind == "ctm":
            m.input = abi.IN_COMBINED if tm.inference_type == "combined" else abi.IN_CONTEXTUAL
            m.C = tm.contextual_size
        else:
            m.input = abi.IN_BOW
        # CTM label head: the labels are the last L inputs of input_layer (CombinedTM
        # [BoW | adapted | labels], ZeroShotTM [contextual | labels])
        m.L = int(getattr(tm, "label_size", 0) or 0)
        m.lab_on = int(m.L > 0)
        if m.lab_on:
            m.lab_off = 2 * tm.input_size if m.input == abi.IN_COMBINED else m.C
        props = torch.cuda.get_device_properties(self.device)
        if self.ctx_fused:
            self._plan_ctx(props.multi_processor_count)
        m.vb = VB
        m.n_tiles = -(-m.V // VB)
        m.dec_grid = int(min(m.n_tiles, 2 * props.multi_processor_count))
        m.learn_priors = int(tm.learn_priors)
        m.kt = theta_stride(m.K)
        m.n_dpart = m.n_tiles if m.kind == abi.KIND_PRODLDA else 1
        m.drop_enc = float(net.dropout_enc.p)
        m.drop_theta = float(model.drop_theta.p)
        m.bn_momentum = float(model.beta_batchnorm.momentum)
        m.bn_eps = float(model.beta_batchnorm.eps)
        m.kl_weight = float(self.beta_weight)
        m.seed = self.seed
        if m.lab_on:
            P0 = self.flat.buffer
            m.w_cls = self._ptr(P0, "label_classification.weight")
            m.b_cls = self._ptr(P0, "label_classification.bias")
            m.lab_in_enc = int(bool(self.ctx_fused))   # else the host hctx carries the labels
        P, G = self.flat.buffer, self.grad
        if tm.learn_priors:
            m.prior_mean, m.prior_var = self._ptr(P, "prior_mean"), self._ptr(P, "prior_variance")
            m.g_prior_mean = self._ptr(G, "prior_mean")
            m.g_prior_var = self._ptr(G, "prior_variance")
        else:
            m.prior_mean, m.prior_var = model.prior_mean.data_ptr(), model.prior_variance.data_ptr()
        m.beta, m.g_beta = self._ptr(P, "beta"), self._ptr(G, "beta")
        m.w_in, m.g_w_in = self._ptr(P, "inf_net.input_layer.weight"), \
            self._ptr(G, "inf_net.input_layer.weight")
        m.b_in, m.g_b_in = self._ptr(P, "inf_net.input_layer.bias"), \
            self._ptr(G, "inf_net.input_layer.bias")
        for l in range(len(hs) - 1):
            for attr, suffix in (("w_h", "weight"), ("b_h", "bias")):
                k = f"inf_net.hiddens.l_{l}.0.{suffix}"
                getattr(m, attr)[l] = self._ptr(P, k)
                getattr(m, "g_" + attr)[l] = self._ptr(G, k)
        for attr, k in (("w_mu", "inf_net.f_mu.weight"), ("b_mu", "inf_net.f_mu.bias"),
                        ("w_s", "inf_net.f_sigma.weight"), ("b_s", "inf_net.f_sigma.bias")):
            setattr(m, attr, self._ptr(P, k))
            setattr(m, "g_" + attr, self._ptr(G, k))
        for attr, k in (("mu_rm", "inf_net.f_mu_batchnorm.running_mean"),
                        ("mu_rv", "inf_net.f_mu_batchnorm.running_var"),
                        ("s_rm", "inf_net.f_sigma_batchnorm.running_mean"),
                        ("s_rv", "inf_net.f_sigma_batchnorm.running_var"),
                        ("beta_rm", "beta_batchnorm.running_mean"),
                        ("beta_rv", "beta_batchnorm.running_var")):
            setattr(m, attr, self._ptr(P, k))
        m.nbt_mu = net.f_mu_batchnorm.num_batches_tracked.data_ptr()
        m.nbt_s = net.f_sigma_batchnorm.num_batches_tracked.data_ptr()
        m.nbt_beta = model.beta_batchnorm.num_batches_tracked.data_ptr()
        m.step, m.adam_t = self.d_step.data_ptr(), self.adam_t.data_ptr()
        if m.ctx_fused == 1:
            m.w_a, m.b_a = self._ptr(P, "inf_net.adapt_bert.weight"), self._ptr(P, "inf_net.adapt_bert.bias")
        # optimizer (fused epilogues + generic Adam)
        m.update_mode = self.update_mode
        m.flat_base = P.data_ptr()
        m.n_shared = self.flat.n_shared
        m.off_m = (self.exp_avg.data_ptr() - P.data_ptr()) // 4
        m.off_v = (self.exp_avg_sq.data_ptr() - P.data_ptr()) // 4
        m.off_g = (self.grad.data_ptr() - P.data_ptr()) // 4
        m.adam_pow, m.adam_coef = self.adam_pow.data_ptr(), self.adam_coef.data_ptr()
        self._sync_opt_fields()
        if self.large_batch:
            self._plan_large_batch(props.multi_processor_count)
            self._alloc_workspace()
            rc = self.lib.gfk_setup(C.byref(m))
            if rc:
                raise RuntimeError(f"gfk_setup failed ({rc})")
            return
        which = (0, 1) if m.kind == abi.KIND_PRODLDA else (2, 3)
        k_split = _force_k_split(self.lib, m)
        need = lambda: max(self.lib.gfk_smem_required(C.byref(m), w)  # noqa: E731
                           for w in which + (4, 5, 7, 8))
        for flags in STAGE_PLANS:         # first plan that fits the 160 KiB of LDS
            m.stage_flags = flags
            if need() <= LDS_LIMIT:
                break
        else:
            raise RuntimeError(f"fused step needs {need()} B of LDS (> {LDS_LIMIT})")
        if m.kind == abi.KIND_PRODLDA:
            # persistent decoder forward: one workgroup per resident slot (16-wave
            # workgroups: 2 per CU when the LDS allows), each looping over its vocab
            # tiles with theta_d staged once and its row-LSE partials merged
            cu = props.multi_processor_count
            sm = self.lib.gfk_smem_required(C.byref(m), 0)
            m.dec_grid = int(min(m.n_tiles, (2 if 2 * sm <= LDS_LIMIT else 1) * cu))
            # strip forward (prodlda_fwd_strip_kernel, stage_flags bit 2): each wave owns
            # 16 columns x all rows, beta straight into registers, batch norm without
            # barriers.  The default wherever it applies (fp32, B <= 64): interleaved A/B
            # vs the tile kernel (profiles/r2/ab_strip_forward.txt) K=50 headline 0.0583
            # vs 0.0589 ms, K=50 V=28k 0.092 vs 0.101, K=200 V=112k 0.342 vs 0.349, CTM /
            # ZeroShotTM K=100 neutral.  GFEDNTM_FWD_STRIP=0 selects the tile kernel
            strip = os.environ.get("GFEDNTM_FWD_STRIP", "auto")
            # (bf16 GEMMs: the ring variant with v_mfma_f32_16x16x32_bf16, 32-k steps)
            fits = (m.bmax <= 64 and m.K <= 256 and m.K * m.ldb < (1 << 29))
            if fits and strip in ("1", "auto"):
                m.stage_flags |= STAGE_FWD_STRIP
                # the rolling prefetch: the next strip's k pair loaded into the registers
                # its MFMAs just consumed, through a ring of <= 13 pairs (K > 104: 128 VGPRs,
                # 16 waves per CU; K = 200 V = 112k forward 39.7 -> 36.5 us, round 0.2794 ->
                # 0.2751 ms).  Rounds 5-6 removed the other strip variants: the plain rolling
                # one, the non-prefetching one and the 8-wave whole-block prefetch, measured
                # slower (profiles/r3, r4, r6/ab_strip_pf_vs_ring.txt)
                m.dec_grid = int(min(m.n_tiles, cu))
                # the batch-coupled posterior (BN of the heads, reparameterisation, softmax,
                # dropout, KL) inside the ring forward's theta_d staging: post_fwd is not
                # launched (K <= 64, no label head; csrc/gfk_common.h gfk_postfold).  Where it
                # pays: batched launches of several clients (BatchedSteps, sim8 strip forward
                # + post_fwd 27.4 -> 20.5 us); for ONE client the redundant per-workgroup
                # statistics lengthen the forward's critical path more than the launch they
                # save (interleaved, one box: 0.0601 vs 0.0597 ms per round,
                # profiles/r5/ab_fold.txt).  GFEDNTM_POSTFOLD=1 forces it here, =0 everywhere
                self._fold_ok = bool(m.K <= 64 and not m.lab_on)
                if self._fold_ok and os.environ.get("GFEDNTM_POSTFOLD", "auto") == "1":
                    m.stage_flags |= STAGE_FWD_POSTFOLD
            # backward: one workgroup per tile while the tiles fit the resident slots;
            # else persistent, n_dpart d theta_d slabs: with >= 4 k tiles the topics
            # are split over 4 workgroups per slab (csrc/prodlda.hip, 8 waves each, two
            # per CU when their LDS allows), otherwise one 16-wave workgroup per CU
            m.n_dpart = m.n_tiles
            sb = self.lib.gfk_smem_required(C.byref(m), 1)      # one tile per workgroup
            if m.n_tiles <= (2 if 2 * sb <= LDS_LIMIT else 1) * cu and not k_split:
                m.n_dpart = m.n_tiles
            elif -(-m.K // 16) >= 4:
                m.n_dpart = min(cu // 2, m.n_tiles - 1)
                if 2 * self.lib.gfk_smem_required(C.byref(m), 1) > LDS_LIMIT:
                    m.n_dpart = min(cu // 4, m.n_tiles - 1)
            else:
                m.n_dpart = cu
            # the persistent k-range backward (4 workgroups per vocab tile) takes its
            # logit-gradient tiles precomputed once per tile by prodlda_dlogit instead of
            # recomputing them in each range workgroup; GFEDNTM_BWD_PRE=0 selects the
            # recomputing variant
            kq4 = m.n_dpart < m.n_tiles and -(-m.K // 16) >= 4
            # (2: two per CU; 3, the default: two per CU, software-pipelined -- the next
            # tile's loads in flight during this tile's compute and stores -- where it
            # applies: fp32, B = 64.  Round 6 removed the 80-VGPR three-per-CU shape and the
            # split beta Adam pass, both measured slower: profiles/r2, profiles/r4)
            pre = os.environ.get("GFEDNTM_BWD_PRE", "3")
            m.bwd_pre = int(pre) if kq4 and m.bmax <= 64 and pre in ("2", "3") else 0
            if (m.bwd_pre == 3 and m.bmax == 64 and m.ldb % 64 == 0
                    and m.K * m.ldb * 4 < 0x7FFF0000):
                pass
            elif m.bwd_pre:
                m.bwd_pre = 2            # two per CU, no register cap
        # W_in tiles as entry lists instead of dense x^T MFMA tiles where a 64-word tile
        # holds few non-zeros (large vocabularies, the 8-wave update shape: more tiles than
        # two rounds of workgroups); GFEDNTM_WIN_SPARSE=0 keeps the dense tiles
        cu_n = props.multi_processor_count
        # CombinedTM at large V: ctx_fwd with all batch rows per vocab tile (each Wa block
        # staged once instead of once per 16-row block); GFEDNTM_CTX_FULL=0 / 1 overrides
        cf_env = os.environ.get("GFEDNTM_CTX_FULL", "auto")
        # (matmul_dtype = "bf16": the register-streamed forward at any V -- the variant with
        # bf16 operands on the matrix cores; the other shapes keep fp32 GEMMs)
        if m.ctx_fused == 1 and m.bmax <= 64 and (
                cf_env == "1" or (cf_env == "auto" and (m.n_tiles > 2 * cu_n or m.mm_bf16))):
            m.stage_flags |= STAGE_CTX_FULL
            # ... as the register-streamed persistent kernel: one 16-wave workgroup per CU
            # owns an equal range of 16-column units (at most 32: V <= 131k on 256 CUs), Wa
            # streamed from global memory into registers as the MFMA A operand, x_ctx staged
            # once per workgroup in 256-float phases; each workgroup leaves one contextual z0
            # partial (ctx_parts for enc_in).  V = 99k, interleaved: ctx_fwd 134 -> 122 us,
            # round 0.7386 -> 0.7287 ms (profiles/r4/ab_s8).  GFEDNTM_CTX_RS=0 keeps the
            # one-workgroup-per-tile kernel.  (Round 6 removed the LDS-DMA balanced shapes,
            # bits 11 / 13, measured slower than this one.)
            n_units = -(-int(m.V) // 16)
            if (os.environ.get("GFEDNTM_CTX_RS", "1") != "0" and int(m.H[0]) <= 64
                    and -(-n_units // min(m.n_tiles, cu_n)) <= 32
                    and m.V * m.C * 4 < (1 << 31) and 4 * self.flat.n_total < (1 << 31)):
                m.stage_flags |= STAGE_CTX_RS
                m.ctx_parts = int(min(m.n_tiles, cu_n))
        # CombinedTM backward as one persistent workgroup per CU walking equal ranges of the
        # (tile, C chunk) items with the next item's Wa state in flight (csrc/ctx.hip
        # gfk_ctx_bwd_pp_k); GFEDNTM_CTX_BWDPP=0 keeps the (tile, chunk) grid
        if (m.ctx_fused == 1 and m.bmax <= 64 and int(m.H[0]) <= 64
                and os.environ.get("GFEDNTM_CTX_BWDPP", "auto") in ("1", "auto")
                and (os.environ.get("GFEDNTM_CTX_BWDPP", "auto") == "1" or m.n_tiles > 2 * cu_n)):
            m.stage_flags |= STAGE_CTX_BWDPP
            m.ctx_bgrid = int(cu_n)
        ws_env = os.environ.get("GFEDNTM_WIN_SPARSE", "auto")
        # (fused CombinedTM too: its bag-of-words half as sparse tiles, the contextual half
        # as dense tiles of the same launch -- csrc/update.hip win_tile_ctx; B <= 64)
        comb = m.input == abi.IN_COMBINED and m.ctx_fused == 1 and m.bmax <= 64
        if (m.input == abi.IN_BOW or comb) and int(m.H[0]) <= 64 and m.bmax <= 128 and (
                ws_env == "1" or (ws_env == "auto" and m.n_tiles > 4 * cu_n)):
            m.stage_flags |= STAGE_WIN_SPARSE
            # fused CombinedTM: the contextual half (Wc) as dense tiles of the same launch.
            # (Round 6 removed three opt-in variants measured slower: Wc as a persistent
            # kernel -- V = 99k, 0.7389 vs 0.7309 ms; the sparse tile's second moment in
            # registers instead of LDS -- profiles/r3/win_vl/; the split W_in update, the
            # words outside the batch on a side stream -- K=200 V=112k 0.320 vs 0.294 ms,
            # profiles/r3/win_split.md)
        self._alloc_workspace()
        rc = self.lib.gfk_setup(C.byref(m))
        if rc:
            raise RuntimeError(f"gfk_setup failed ({rc})")

    def _plan_large_batch(self, cu: int):
        """The large-batch plan, 128 < batch_size <= 512 (csrc/gfk_common.h GFK_LB; reference
        avitm.py:84-85 takes any batch_size).  The row-parallel kernels (enc_in, post_fwd,
        row_loss, row_bwd, post_bwd) run as for small batches with the [B, K] batch matrices
        read from L2 (bit 1), W_in's gradient on the sparse tiles (bit 4), the weight jobs and
        NeuralLDA's beta backward in 128-row chunks.  ProdLDA's decoder: logits = theta_d beta,
        dbeta = theta_d^T dlogit and d theta_d = dlogit beta^T are hipBLASLt GEMMs on the step's
        stream (PH_LB_GEMM_FWD / _BWD: at B >= 256 they are large enough to run near the
        matrix cores' fp32 peak) around prodlda_lb_colbn (column batch-norm, BN'ed tiles, row
        sum-exp partials) and prodlda_lb_dlogit (the logit gradient) -- one slab of d theta_d,
        the [B, ldb] logit / logit-gradient matrix in ws["dt"].  Gradient mode: the generic
        optimizer kernel updates every tensor (as the CTM host-GEMM path)."""
        m = self._m
        # W_in's gradient: the sparse entry-list tiles where a 64-word tile holds few of the
        # batch's non-zeros (more tiles than 4 rounds of the CUs, as for small batches), else
        # the dense tiles in 128-row chunks (csrc/update.hip win_tile_dense_ch);
        # GFEDNTM_WIN_SPARSE=1 / 0 forces either
        ws_env = os.environ.get("GFEDNTM_WIN_SPARSE", "auto")
        sparse = ws_env == "1" or (ws_env == "auto" and m.n_tiles > 4 * cu)
        m.stage_flags = 2 | STAGE_LB | (STAGE_WIN_SPARSE if sparse else 0)
        m.dec_grid = int(min(m.n_tiles, 2 * cu))
        m.n_dpart = 1
        m.bwd_pre = 0
        # ProdLDA's decoder on the matrix cores (csrc/prodlda.hip prodlda_lb_fwd / _bwd) at
        # bmax 256, K <= 208: one 16-wave workgroup per CU, persistent over the tiles, the
        # backward's d theta_d in one slab per workgroup.  Elsewhere (bmax 512, K > 208) and
        # with GFEDNTM_LB_GEMM=1: the library GEMMs around the HIP kernels.
        m.lb_fused = 0
        if (m.kind == abi.KIND_PRODLDA and int(m.K) <= 208 and self.bmax == 256
                and os.environ.get("GFEDNTM_LB_GEMM", "0") != "1"):
            # (+ bit 2: beta's Adam step in prodlda_lb_bwd's epilogue -- the generic optimizer
            # pass then skips beta, 80 % of the parameters at K = 200, V = 112k)
            m.lb_fused = 3 | (4 if self.solver == "adam" else 0)
            m.dec_grid = int(min(m.n_tiles, cu))
            if m.lb_fused & 2:
                m.n_dpart = m.dec_grid
        which = (0, 1) if m.kind == abi.KIND_PRODLDA else (2, 3)
        need = max(self.lib.gfk_smem_required(C.byref(m), w) for w in which + (4, 5, 7))
        if need > LDS_LIMIT:
            raise RuntimeError(f"large-batch plan needs {need} B of LDS (> {LDS_LIMIT})")

    def _lb_views(self):
        """(theta_d [B, K], beta [K, ldb], beta's gradient [K, ldb], the logit matrix
        [B, ldb], d theta_d slab 0 [B, K]) for the large-batch GEMMs."""
        if getattr(self, "_lbv", None) is None:
            B, K = self.bmax, int(self._m.K)
            self._lbv = (self.ws["thetad"][:, :K], self.raw_like(self.flat.buffer, "beta"),
                         self.raw_like(self.grad, "beta"), self.ws["dt"].view(B, int(self._m.ldb)),
                         self.ws["dthetad"][: B * K].view(B, K))
        return self._lbv

    def _lb_gemm_fwd(self):
        th, beta, _, dt, _ = self._lb_views()
        torch.mm(th, beta, out=dt)                       # logits [B, ldb]

    def _lb_gemm_bwd(self):
        th, beta, gbeta, dt, dth = self._lb_views()
        torch.mm(th.t(), dt, out=gbeta)                  # dbeta = theta_d^T dlogit
        torch.mm(dt, beta.t(), out=dth)                  # d theta_d = dlogit beta^T

    def _plan_ctx(self, cu: int):
        """Fused CombinedTM contextual kernels (csrc/ctx.hip).  The forward runs one
        workgroup per (vocab tile, 16-row block); the backward splits C into chunks
        of 16k <= 256 floats, enough of them that n_tiles x chunks covers the CUs
        once (one 16-wave workgroup per CU).  Falls back to the host GEMMs when a shape is outside
        the kernels' assumptions (C % 4, H0 <= 512, LDS)."""
        m = self._m
        if m.input == abi.IN_CONTEXTUAL:
            # ZeroShotTM: the [C, H0] input layer is gathered densely by enc_in and its
            # gradient + Adam are ceil(C / 64) extra win_update tiles
            m.ctx_fused = 2 if int(m.H[0]) <= 512 else 0
            if not m.ctx_fused:
                self._ctx_fallback(f"H0 = {int(m.H[0])} > 512")
            return
        n_tiles, Cs = -(-int(m.V) // VB), int(m.C)
        k = max(1, min(cu // n_tiles, -(-Cs // 16)))      # one round, one workgroup per CU
        m.ctx_ckb = min(256, -(-(-(-Cs // k)) // 16) * 16)
        m.ctx_kb = -(-Cs // m.ctx_ckb)
        m.ctx_fused = 1
        aligned = self.flat.slots["inf_net.adapt_bert.weight"].offset % 4 == 0
        why = [w for ok, w in (
            (self.lib.gfk_smem_required(C.byref(m), 8) <= LDS_LIMIT, "LDS plan exceeds 160 KiB"),
            (int(m.H[0]) <= 512, f"H0 = {int(m.H[0])} > 512"),
            (Cs % 4 == 0, f"contextual_size = {Cs} is not a multiple of 4"),
            (aligned, "adapt_bert is not 16-byte aligned in the flat buffer")) if not ok]
        if why:
            m.ctx_fused, m.ctx_kb = 0, 0
            self._ctx_fallback("; ".join(why))

    def _ctx_fallback(self, why: str):
        """Leave the fused contextual kernels for host-issued hipBLASLt GEMMs (gradient
        mode + the generic optimizer kernel).  Logged, and visible as
        ``ctx_fallback_reason`` (the bench records it): the GEMMs are launched between
        the fused kernels on the step's stream, and cost several extra dispatches and the
        [B, V] adapted matrix's round trip through HBM per step."""
        import logging
        self.ctx_fused = False
        self.update_mode = UPDATE_GRAD
        self.ctx_fallback_reason = why
        logging.getLogger("gfedntm_amd.engine").warning(
            "CTM contextual path on host GEMMs (fused ctx kernels unavailable: %s)", why)

    def _alloc_workspace(self):
        m, dev = self._m, self.device
        B, K, V = self.bmax, m.K, m.V
        hs = [m.H[i] for i in range(m.n_hidden)]
        def f(*shape):
            # 16 floats of zeroed slack: LDS-DMA copies whole 16-byte chunks
            n = int(np.prod(shape))
            return torch.zeros(n + 16, dtype=torch.float32, device=dev)[:n].view(*shape)

        ws: Dict[str, torch.Tensor] = {
            "doc": torch.zeros(B, dtype=torch.int32, device=dev),
            "nb": torch.zeros(1, dtype=torch.int32, device=dev),
            "hd": f(B, hs[-1]), "mask_h": f(B, hs[-1]),
            "mu_raw": f(B, K), "ls_raw": f(B, K), "mu": f(B, K), "ls": f(B, K),
            "bn_rstd": f(2 * K), "eps": f(B, K), "theta": f(B, K), "thetad": f(B, m.kt),
            "mask_t": f(B, K), "kl": f(B), "rl": f(B), "lse": f(max(B, K)), "s": f(B),
            "zn": f(m.n_tiles * B * VB if m.kind == abi.KIND_PRODLDA else V * K),
            "col_rstd": f(m.n_tiles * VB),
            "row_part": f(max(m.n_tiles * 4 * B, m.dec_grid * K) * 2),
            "dthetad": f((m.n_dpart + m.lab_on) * B * K),     # + the label head's slab
            "dmr": f(B, K), "dlr": f(B, K), "dmu": f(B, K), "dls": f(B, K),
            "dbsm": f(1), "ck": f(K),        # LDA: per-non-zero coefficients, sized in bind_data
            "hctx": f(B, hs[0]),
            "tstart": torch.zeros(B * (m.n_tiles + 1), dtype=torch.int32, device=dev),
            "erange": torch.zeros(2 * B, dtype=torch.int32, device=dev),
            "next": torch.zeros(1 + 3 * B, dtype=torch.int32, device=dev),
            # fused CombinedTM: the adapted rows per vocab tile and their contextual
            # pre-activation partials (csrc/ctx.hip)
            "actx": f(m.n_tiles * B * 64 if m.ctx_fused == 1 else 1),
            "hpart": f(m.n_tiles * B * hs[0] if m.ctx_fused == 1 else 1),
            # precomputed logit-gradient tiles [n_tiles][B][66] (bwd_pre; + the pipelined
            # backward's store sinks, 64 floats per workgroup)
            # (the large-batch plan: the [B, ldb] logit / logit-gradient matrix)
            "dt": f(B * int(m.ldb) if m.stage_flags & STAGE_LB and (m.lb_fused & 3) != 3 else
                    m.n_tiles * B * 66 + 64 * (4 * m.n_dpart + 32) if m.bwd_pre else 1),
            # the large-batch plan's posterior column statistics (6 x 2K floats)
            "colstat": f(12 * K if m.stage_flags & STAGE_LB else 1),
        }
        Lb = max(int(m.L), 1)
        ws.update(lab=f(B, Lb), dlab=f(B, Lb), ce=f(B), thd=f(B, K))   # label head
        for i, h in enumerate(hs):
            ws[f"z{i}"] = f(B, h)
            ws[f"a{i}"] = f(B, h)
        ws["dtheta"] = f(B, K)            # the reduced d theta_d (row_bwd)
        for i, h in enumerate(hs):
            ws[f"dz{i}"] = f(B, h)
        self.ws = ws
        self._alloc_ctx()
        for k, t in ws.items():
            if k[0] in "za" and k[1:].isdigit():
                getattr(m, "ws_" + k[0])[int(k[1:])] = t.data_ptr()
            elif k.startswith("dz") and k[2:].isdigit():
                m.ws_dz[int(k[2:])] = t.data_ptr()
            else:
                setattr(m, "ws_" + k, t.data_ptr())
        self._build_update_jobs()

    def _build_update_jobs(self):
        """The small-tensor gradient / update jobs of win_update (csrc/update.hip):
        64 x 64 GEMM tiles for the hidden / head weights, batch column sums for the
        biases, the priors' gradient (from post_bwd)."""
        u, ws, P = self._u, self.ws, self.flat.buffer
        hs = list(self.tm.hidden_sizes)
        K = self._m.K
        wj = []
        for l in range(len(hs) - 1):
            wj.append((f"inf_net.hiddens.l_{l}.0.weight", ws[f"dz{l + 1}"], ws[f"a{l}"], hs[l + 1], hs[l]))
        wj.append(("inf_net.f_mu.weight", ws["dmr"], ws["hd"], K, hs[-1]))
        wj.append(("inf_net.f_sigma.weight", ws["dlr"], ws["hd"], K, hs[-1]))
        L = int(self._m.L)
        if L:
            # label head: the classifier [L, K] (d est x theta_d) and the input layer's
            # label block [L, H0] of the transposed weight (labels x d z0)
            wj.append(("label_classification.weight", ws["dlab"], ws["thd"], L, K))
            lab_block = self._ptr(P, "inf_net.input_layer.weight") + 4 * int(self._m.lab_off) * hs[0]
            wj.append((lab_block, ws["lab"], ws["dz0"], L, hs[0]))
        n = 0
        for key, dz, a, rows, cols in wj:
            for j0 in range(0, rows, 64):
                for i0 in range(0, cols, 64):
                    if n >= abi.MAX_WJOBS:
                        raise RuntimeError("too many weight tiles for the fused update")
                    J = u.w[n]
                    J.param = key if isinstance(key, int) else self._ptr(P, key)
                    J.dz, J.a = dz.data_ptr(), a.data_ptr()
                    J.rows, J.cols, J.j0, J.i0 = rows, cols, j0, i0
                    n += 1
        u.n_w = n
        vj = [("inf_net.input_layer.bias", ws["dz0"], hs[0])]
        for l in range(len(hs) - 1):
            vj.append((f"inf_net.hiddens.l_{l}.0.bias", ws[f"dz{l + 1}"], hs[l + 1]))
        vj += [("inf_net.f_mu.bias", ws["dmr"], K), ("inf_net.f_sigma.bias", ws["dlr"], K)]
        if self.tm.learn_priors:
            vj += [("prior_mean", None, K), ("prior_variance", None, K)]
        if L:
            vj.append(("label_classification.bias", ws["dlab"], L))
        for i, (key, src, nn_) in enumerate(vj):
            V = u.v[i]
            V.param, V.src, V.n = self._ptr(P, key), (src.data_ptr() if src is not None else None), nn_
        u.n_v = len(vj)

    def _sync_opt_fields(self):
        m = self._m
        m.lr, m.beta1, m.beta2 = self.lr, self.beta1, self.beta2
        m.adam_eps, m.weight_decay = self.eps, self.weight_decay
        m.fed_scale_on = int(self.fedavg_scale is not None)
        m.fed_scale = 1.0 if self.fedavg_scale is None else float(self.fedavg_scale)

    def _fill_adam(self, a, keys=None, keep_grad: bool = False):
        """Segment table of a GfkAdam: [start, end) float ranges of parameters (all,
        or the slots of ``keys``) with ADAM, plus SCALE on the shared prefix.
        Batch-norm running statistics are scaled by the kernels that update them.
        Returns the number of workgroups (abi.ADAM_CHUNK float4 each)."""
        a.p, a.g = self.flat.buffer.data_ptr(), self.grad.data_ptr()
        a.m, a.v = self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr()
        a.lr, a.beta1, a.beta2 = self.lr, self.beta1, self.beta2
        a.eps, a.weight_decay = self.eps, self.weight_decay
        a.solver = abi.SOLVER_CODES[self.solver]
        a.scale = 1.0 if self.fedavg_scale is None else float(self.fedavg_scale)
        a.t = self.adam_t.data_ptr()
        a.coef = self.adam_coef.data_ptr()
        up = lambda x: -(-x // ALIGN) * ALIGN  # noqa: E731
        n_total = self.flat.n_total
        shared_end = up(self.flat.n_shared) if self.fedavg_scale is not None else 0
        if keys is None and getattr(self, "large_batch", False) and self._m.lb_fused & 4:
            # beta's Adam runs in the large-batch backward's epilogue (csrc/prodlda.hip)
            keys = [k for k in self.flat.slots if k != "beta"
                    and any(k == n for n, _ in self.param_order)]
        if keys is None:
            pr = [(s0, up(s1)) for s0, s1 in self.flat.param_ranges()]
        else:
            pr = [(self.flat.slots[k].offset, up(self.flat.slots[k].offset + self.flat.slots[k].numel))
                  for k in keys]
        cuts = sorted({0, n_total, shared_end} | {x for r in pr for x in r})
        segs: List[List[int]] = []
        for x0, x1 in zip(cuts[:-1], cuts[1:]):
            if x1 <= x0 or not any(s0 <= x0 and x1 <= s1 for s0, s1 in pr):
                continue
            flags = abi.SEG_ADAM | (abi.SEG_SCALE if x1 <= shared_end else 0) | \
                (abi.SEG_KEEP_GRAD if keep_grad else 0)
            if segs and segs[-1][1] == x0 and segs[-1][2] == flags:
                segs[-1][1] = x1
            else:
                segs.append([x0, x1, flags])
        if len(segs) > abi.MAX_SEGS:
            raise RuntimeError("too many Adam segments")
        a.n_seg = len(segs)
        nblk = 0
        for i, (s0, s1, fl) in enumerate(segs):
            a.seg_start[i], a.seg_end[i], a.seg_flags[i] = s0, s1, fl
            a.seg_first_block[i] = nblk
            nblk += -(-((s1 - s0) // 4) // abi.ADAM_CHUNK)
        return nblk

    def _rebuild_adam(self):
        self._sync_opt_fields()
        self.adam_grid = int(max(1, self._fill_adam(self._a)))
        self._invalidate_graph()

    @property
    def ctx_gemm_dtype(self) -> Optional[str]:
        """Operand precision of CombinedTM's contextual GEMMs (adapt_bert and its input-layer
        term) in the forward: "bf16" where matmul_dtype = "bf16" runs the register-streamed
        kernel (csrc/ctx.hip gfk_ctx_fwd_rs_k<BF>), else "fp32"; None without them."""
        m = self._m
        if not self.ctx_fused or m.ctx_fused != 1:
            return None
        rs = STAGE_CTX_FULL | STAGE_CTX_RS
        return "bf16" if m.mm_bf16 and (m.stage_flags & rs) == rs else "fp32"

    @property
    def launch_plan(self) -> str:
        """The launch plan in one phrase (recorded in bench / metrics records)."""
        if self.large_batch:
            if self._m.kind == abi.KIND_PRODLDA and (self._m.lb_fused & 3) != 3:
                return ("large-batch: HIP kernels + hipBLASLt decoder GEMMs"
                        + (" (backward)" if self._m.lb_fused else "") + ", gradient mode")
            return "large-batch: HIP kernels, gradient mode"
        return "fused kernels" + (" (fused optimizer epilogues)" if self.update_mode == UPDATE_FUSED else "")

    def set_fedavg_scale(self, w: Optional[float]):
        """Pre-scale the shared state by w after the update (None disables)."""
        if w != self.fedavg_scale:
            self.fedavg_scale = w
            self._rebuild_adam()

    def set_lr(self, lr: float):
        self.lr = float(lr)
        self.optimizer.param_groups[0]["lr"] = self.lr
        self._rebuild_adam()

    # ------------------------------------------------------------------ data
    def bind_data(self, data: DeviceCSR, plan: BatchPlan):
        super().bind_data(data, plan)
        m, dev = self._m, self.device
        self._plan_dev = {
            "order": torch.from_numpy(plan.order).to(dev),
            "start": torch.from_numpy(plan.start).to(dev),
            "size": torch.from_numpy(plan.size).to(dev),
        }
        m.indptr, m.indices, m.values = (data.indptr.data_ptr(), data.indices.data_ptr(),
                                         data.values.data_ptr())
        if m.kind == abi.KIND_LDA:      # g = -x / (wd + eps) per CSR non-zero (lda_row -> lda_beta_bwd)
            nnz = int(data.indices.numel())
            if self.ws["dbsm"].numel() < nnz:
                self.ws["dbsm"] = torch.zeros(nnz + 16, dtype=torch.float32, device=dev)
            m.ws_dbsm = self.ws["dbsm"].data_ptr()
        m.ctx = data.contextual.data_ptr() if data.contextual is not None else None
        if m.stage_flags & STAGE_CTX_RS and data.contextual is not None \
                and 4 * data.contextual.numel() >= (1 << 31):
            # the register-streamed forward addresses x_ctx with 32-bit buffer offsets
            m.stage_flags &= ~STAGE_CTX_RS
            m.ctx_parts = 0
        if m.lab_on:
            if data.labels is None or data.labels.shape[1] != m.L:
                raise ValueError(f"the model has a label head of size {m.L}: bind data with "
                                 f"labels [n_docs, {m.L}]")
            m.labels = data.labels.data_ptr()
        # the next batch's rows in fixed slots (prepare_next_batch -> enc_in / row_loss)
        cap = max(16, -(-int(data.row_len_max) // 16) * 16)
        if self.ws.get("sidx") is None or self.ws["sidx"].numel() < self.bmax * cap:
            self.ws["sidx"] = torch.zeros(self.bmax * cap + 16, dtype=torch.int32, device=dev)
            self.ws["sval"] = torch.zeros(self.bmax * cap + 16, dtype=torch.float32, device=dev)
        m.slot_cap = cap
        m.ws_sidx, m.ws_sval = self.ws["sidx"].data_ptr(), self.ws["sval"].data_ptr()
        m.plan_order = self._plan_dev["order"].data_ptr()
        m.plan_start = self._plan_dev["start"].data_ptr()
        m.plan_size = self._plan_dev["size"].data_ptr()
        m.loss_hist = self.loss_hist.data_ptr()
        m.kl_hist = self.kl_hist.data_ptr() if self.terms_on else None
        m.rl_hist = self.rl_hist.data_ptr() if self.terms_on else None
        m.n_steps = plan.n_steps
        self.d_step.zero_()
        self._host_step = 0
        self._invalidate_graph()
        self._launch([abi.PH_BATCH_PREP])

    def record_terms(self, on: bool = True):
        """The batch-level workgroup (csrc/posterior.hip post_term_hist) writes the step's mean
        KL and RL next to loss_hist while on (two more block sums at the end of the step)."""
        super().record_terms(on)
        if self.kl_hist is not None:
            self._m.kl_hist = self.kl_hist.data_ptr() if self.terms_on else None
            self._m.rl_hist = self.rl_hist.data_ptr() if self.terms_on else None
            self._invalidate_graph()

    def phases(self) -> List[int]:
        if self._m.kind == abi.KIND_LDA:
            ph = [p for p in abi.LDA_STEP if p != abi.PH_ADAM] + \
                ([abi.PH_ADAM] if self.update_mode == UPDATE_GRAD else [])
        else:
            ph = abi.PRODLDA_STEP + ([abi.PH_ADAM] if self.update_mode == UPDATE_GRAD else [])
            if self.large_batch:                    # the decoder's GEMMs around its kernels
                if not self._m.lb_fused & 1:
                    ph.insert(ph.index(abi.PH_PRODLDA_FWD), abi.PH_LB_GEMM_FWD)
                if not self._m.lb_fused & 2:
                    ph.insert(ph.index(abi.PH_PRODLDA_BWD) + 1, abi.PH_LB_GEMM_BWD)
            if self._m.stage_flags & STAGE_FWD_POSTFOLD:
                ph.remove(abi.PH_POST_FWD)          # computed by the strip forward
        if self.ctx_fused:
            if self._m.ctx_fused == 1:
                ph.insert(ph.index(abi.PH_ENC_FWD), abi.PH_CTXF_FWD)
                ph.insert(ph.index(abi.PH_ENC_BWD), abi.PH_CTXF_BWD)
        elif self.kind == "ctm":
            ph.insert(ph.index(abi.PH_ENC_FWD), abi.PH_CTX_FWD)
            ph.insert(ph.index(abi.PH_ENC_BWD) + 1, abi.PH_CTX_BWD)
        if self._comm is not None and self._comm["mode"] == "graph":
            if "beta" in self._comm:
                last = abi.PH_PRODLDA_BWD if abi.PH_PRODLDA_BWD in ph else abi.PH_LDA_BETA_BWD
                ph.insert(ph.index(last) + 1, abi.PH_FEDAVG_BETA)
            if "wa" in self._comm:
                ph.insert(ph.index(abi.PH_CTXF_BWD) + 1, abi.PH_FEDAVG_WA)
            ph.append(abi.PH_FEDAVG_END)
        return ph

    # ------------------------------------------------------------------ FedAvg
    def attach_fedavg(self, group=None, method: Optional[str] = None, wire: str = "fp32") -> str:
        """Make the round's FedAvg all-reduce part of :meth:`step` (collective: call on
        every rank, after the shared state is pre-scaled).

        With the custom xGMI all-reduce the collectives are kernels on the step's
        streams and are captured in the step's graph; in fused ProdLDA mode beta is
        final after prodlda_bwd (Adam + pre-scale in its epilogue), so its all-reduce
        runs on a side stream while row_bwd / post_bwd / win_update proceed, and only
        the encoder part stays on the critical path.  Otherwise (RCCL) the all-reduce
        follows the step eagerly.  ``wire="bf16delta"``: the opt-in reduced-byte FedAvg
        (parallel/aggregator.py; this engine's pre-scale is the rank's weight).  Returns the
        method in use."""
        from ..parallel.aggregator import CollectiveAggregator
        self._comm = None
        shared = self.flat.shared
        parts = {k: shared[a:b] for k, (a, b) in self.fedavg_parts().items()}
        if wire != "fp32" and self.fedavg_scale is None:
            raise ValueError("bf16delta FedAvg needs the FedAvg pre-scale (set_fedavg_scale)")
        aggs = {k: CollectiveAggregator(group, method=method, wire=wire, weight=self.fedavg_scale)
                for k in parts}
        # large parts (beta at V ~ 100k: 90 MB) are all-reduced in place: the xGMI kernel
        # maps the state itself into the peers instead of copying it into a stage first
        # (2 S of local HBM traffic per round saved, one extra hand-off)
        big = int(float(os.environ.get("GFEDNTM_XGMI_INPLACE_MB", "8")) * (1 << 20))
        methods = {k: aggs[k].prepare(v, inplace=4 * v.numel() >= big) for k, v in parts.items()}
        # setup cost of the data plane (IPC mapping, validation, RCCL-vs-xGMI timing)
        self.fedavg_attach = {"s": round(sum(a.setup_s for a in aggs.values()), 4),
                              "bytes": {k: 4 * v.numel() for k, v in parts.items()},
                              "tuning": {k: a.tuning for k, a in aggs.items() if a.tuning},
                              # per part: method, in-place, uncached flags (csrc/comm.hip
                              # gfk_comm_alloc) or why it is not on the xGMI kernel
                              "plane": {k: a.describe() for k, a in aggs.items()}}
        if all(m == "xgmi" for m in methods.values()):
            c = {"mode": "graph", **{k: (aggs[k], parts[k]) for k in parts}}
            if len(parts) > 1:
                c["stream"] = torch.cuda.Stream(self.device)
                c["ev_fork"] = torch.cuda.Event()
                c["ev_fork_wa"] = torch.cuda.Event()
                c["ev_join"] = torch.cuda.Event()
            self._comm = c
            used = "xgmi" + ("+overlap" if len(parts) > 1 else "")
        else:
            for a in aggs.values():
                if a.xgmi is not None:
                    a.xgmi.close()
            agg = CollectiveAggregator(group, method="rccl", wire=wire, weight=self.fedavg_scale)
            agg.set_reference(shared)
            self._comm = {"mode": "eager", "rest": (agg, shared)}
            used = agg.active
        self._invalidate_graph()
        return used

    def fedavg_parts(self) -> Dict[str, Tuple[int, int]]:
        """The shared state's FedAvg parts as (start, end) offsets, each with its own
        collective: in the fused update mode beta is final after the decoder backward
        and CombinedTM's adapt_bert after ctx_bwd (their Adam + pre-scale epilogues), so
        those all-reduces run on a side stream while the rest of the step proceeds; the
        rest of the state follows win_update.  (The layout puts them last: topic_model
        FUSED_SHARED_LAST.)"""
        flat = self.flat
        keys = flat.shared_keys
        n = flat.n_shared
        if not (self.update_mode == UPDATE_FUSED and keys and keys[-1] == "beta" and len(keys) > 1):
            return {"rest": (0, n)}
        b0 = flat.slots["beta"].offset
        wa = ["inf_net.adapt_bert.weight", "inf_net.adapt_bert.bias"]
        if self._m.ctx_fused == 1 and len(keys) > 3 and keys[-3:-1] == wa:
            w0 = flat.slots[wa[0]].offset
            return {"rest": (0, w0), "wa": (w0, b0), "beta": (b0, n)}
        return {"rest": (0, b0), "beta": (b0, n)}

    def fedavg_set_reference(self):
        """bf16delta: the current shared state becomes every part's last averaged state
        (after a checkpoint was loaded into it)."""
        if self._comm is None:
            return
        for k in ("rest", "beta", "wa"):
            if k in self._comm:
                agg, buf = self._comm[k]
                agg.set_reference(buf)

    def detach_fedavg(self, close: bool = True):
        """Remove the in-step all-reduce (returns it for :meth:`restore_fedavg` when
        ``close`` is False; otherwise frees the xGMI buffers)."""
        c, self._comm = self._comm, None
        self._invalidate_graph()
        if c is not None and close:
            for k in ("rest", "beta", "wa"):
                if k in c and c[k][0].xgmi is not None:
                    c[k][0].xgmi.close()
                    c[k][0].xgmi = None
            return None
        return c

    def restore_fedavg(self, c):
        self._comm = c
        self._invalidate_graph()

    def fedavg_error(self) -> int:
        """Non-zero if an xGMI all-reduce wait timed out (synchronises)."""
        if self._comm is None:
            return 0
        err = 0
        for k in ("rest", "beta", "wa"):
            if k in self._comm and self._comm[k][0].xgmi is not None:
                err = err or self._comm[k][0].xgmi.error()
        return err

    def fedavg_debug(self) -> dict:
        """Per-part diagnostics of the xGMI all-reduces (epochs, lagging flags)."""
        out = {}
        for k in ("rest", "beta", "wa"):
            if self._comm is not None and k in self._comm and self._comm[k][0].xgmi is not None:
                out[k] = self._comm[k][0].xgmi.debug_state()
        return out

    def fedavg_error_async(self):
        """Start a non-blocking read of the xGMI error words (behind the enqueued rounds);
        :meth:`fedavg_error_poll` returns it once the copies have landed."""
        if self._comm is None or self._comm["mode"] != "graph":
            return
        c = self._comm
        if "err_host" not in c:
            c["err_host"] = torch.zeros(3, dtype=torch.int32, pin_memory=True)
            c["err_ev"] = torch.cuda.Event()
        for i, k in enumerate(("rest", "beta", "wa")):
            if k in c and c[k][0].xgmi is not None:
                c[k][0].xgmi.error_async(c["err_host"][i:i + 1])
        c["err_ev"].record()
        c["err_pending"] = True

    def fedavg_error_poll(self) -> int:
        """The error word of the last :meth:`fedavg_error_async` if it has landed, else 0
        (not known yet); never synchronises."""
        c = self._comm
        if not c or not c.get("err_pending") or not c["err_ev"].query():
            return 0
        c["err_pending"] = False
        return int(c["err_host"].max().item())

    def _fedavg_beta(self):
        c = self._comm
        cur = torch.cuda.current_stream(self.device)
        c["ev_fork"].record(cur)
        side = c["stream"]
        side.wait_event(c["ev_fork"])
        with torch.cuda.stream(side):
            agg, buf = c["beta"]
            agg.allreduce_(buf)
        c["ev_join"].record(side)

    def _fedavg_wa(self):
        c = self._comm
        cur = torch.cuda.current_stream(self.device)
        c["ev_fork_wa"].record(cur)
        side = c["stream"]
        side.wait_event(c["ev_fork_wa"])          # (behind beta's on the same side stream)
        with torch.cuda.stream(side):
            agg, buf = c["wa"]
            agg.allreduce_(buf)
        c["ev_join"].record(side)

    def _fedavg_end(self):
        c = self._comm
        agg, buf = c["rest"]
        agg.allreduce_(buf)
        if "beta" in c or "wa" in c:
            torch.cuda.current_stream(self.device).wait_event(c["ev_join"])

    # ------------------------------------------------------------------ CTM
    def _alloc_ctx(self):
        """Buffers of the CTM contextual path (reference ctm inference_network.py:97-193)
        when it runs on host-issued GEMMs.  The default path is the fused kernels
        (_plan_ctx: CombinedTM's ctx_fwd / ctx_bwd in csrc/ctx.hip, ZeroShotTM's dense
        input layer in enc_in / win_update); these buffers serve (a) the fallback for
        shapes outside the kernels' plan (C % 4, H0 > 512, LDS, alignment -- logged by
        _ctx_fallback), where adapt_bert [B,C]x[C,V], the contextual half of
        input_layer [B,V]x[V,H0] and their weight gradients are hipBLASLt GEMMs on the
        step's stream between the fused kernels (CTX_FWD fills ws_hctx, CTX_BWD turns
        d z0 into the contextual gradients, the generic optimizer kernel follows), and
        (b) the dense contextual term of theta inference (_ctx_dense)."""
        self._ctx = None
        if self.kind != "ctm":
            return
        m, dev = self._m, self.device
        B, V, C, H0 = self.bmax, m.V, int(m.C), int(m.H[0])
        z = lambda *sh: torch.zeros(*sh, dtype=torch.float32, device=dev)  # noqa: E731
        c = {"docs": torch.zeros(B, dtype=torch.int64, device=dev),
             "rows": torch.arange(B, dtype=torch.int32, device=dev),
             "valid": torch.zeros(B, dtype=torch.bool, device=dev),
             "xc": z(B, C), "dzm": z(B, H0)}
        kw = "inf_net.input_layer.weight"
        w_in, g_in = self.flat.raw(kw), self.raw_like(self.grad, kw)     # [n_in, H0]
        if m.input == abi.IN_COMBINED:
            c.update(a=z(B, V), da=z(B, V),
                     Wa=self.flat.view("inf_net.adapt_bert.weight"),          # [V, C]
                     ba=self.flat.view("inf_net.adapt_bert.bias"),
                     gWa=self.view_like(self.grad, "inf_net.adapt_bert.weight"),
                     gba=self.view_like(self.grad, "inf_net.adapt_bert.bias"),
                     Wc=w_in[V:2 * V], gWc=g_in[V:2 * V])
        else:
            c.update(W=w_in[:C], gW=g_in[:C])                                   # [C, H0]
        if m.lab_on:                 # the label block [L, H0] (its gradient: a win_update job)
            c.update(Wl=w_in[int(m.lab_off): int(m.lab_off) + int(m.L)],
                     lb=z(B, int(m.L)))
        self._ctx = c

    def raw_like(self, buf: torch.Tensor, key: str) -> torch.Tensor:
        return slot_view(buf, self.flat.slots[key], storage=True)

    def _ctx_fwd(self):
        c, ws = self._ctx, self.ws
        if self.data is None or self.data.contextual is None:
            raise RuntimeError("CTM needs contextual embeddings in the bound data")
        c["docs"].copy_(ws["next"][1: 1 + self.bmax])        # this step's rows (batch prep)
        torch.index_select(self.data.contextual, 0, c["docs"], out=c["xc"])
        if "Wa" in c:
            torch.addmm(c["ba"], c["xc"], c["Wa"].t(), out=c["a"])
            torch.mm(c["a"], c["Wc"], out=ws["hctx"])
        else:
            torch.mm(c["xc"], c["W"], out=ws["hctx"])
        if "Wl" in c:                # labels' contribution (enc_in adds hctx)
            torch.index_select(self.data.labels, 0, c["docs"], out=c["lb"])
            ws["hctx"].addmm_(c["lb"], c["Wl"])

    def _ctx_bwd(self):
        c, ws = self._ctx, self.ws
        torch.lt(c["rows"], ws["nb"], out=c["valid"])         # rows >= nb hold stale d z0
        torch.mul(ws["dz0"], c["valid"].unsqueeze(1), out=c["dzm"])
        if "Wa" in c:
            torch.mm(c["a"].t(), c["dzm"], out=c["gWc"])
            torch.mm(c["dzm"], c["Wc"].t(), out=c["da"])
            torch.mm(c["da"].t(), c["xc"], out=c["gWa"])
            torch.sum(c["da"], 0, out=c["gba"])
        else:
            torch.mm(c["xc"].t(), c["dzm"], out=c["gW"])

    # ------------------------------------------------------------------ inference
    def _ctx_dense(self, data: DeviceCSR, d0: int, d1: int) -> torch.Tensor:
        """Dense contextual contribution to the input layer for documents [d0, d1):
        adapt_bert + the contextual half of input_layer (CombinedTM) or the whole
        input layer (ZeroShotTM) -- library GEMMs, as in the step's CTX_FWD."""
        c = self._ctx
        x = data.contextual[d0:d1]
        h = torch.addmm(c["ba"], x, c["Wa"].t()) @ c["Wc"] if "Wa" in c else x @ c["W"]
        if "Wl" in c:                # CTM label head: the labels are encoder inputs too
            if data.labels is None:
                raise ValueError("this model encodes labels: inference data needs them")
            h = h + data.labels[d0:d1] @ c["Wl"]
        return h

    @torch.no_grad()
    def theta_infer(self, data: DeviceCSR, n_samples: int = 20, seed: int = 0,
                    postprocess: bool = False, threshold: float = 3e-3, moments: bool = False,
                    chunk: Optional[int] = None) -> torch.Tensor:
        """Document-topic distribution of every document of ``data`` (csrc/infer.hip):
        the mean over ``n_samples`` draws of softmax(mu + eps * sigma) with the encoder
        in eval mode (running batch-norm statistics, no dropout), evaluated ONCE per
        document with the draws made in registers (the reference re-runs the encoder
        for every sample, avitm.py:470-523).  ``postprocess`` fuses the theta
        threshold + L1 normalisation (federated_model.py:170-173); ``moments`` returns
        the posterior [D, 2, K] = (mu, log sigma^2) instead.  The draws are keyed by
        (seed, document index), so the chunking does not change the result."""
        m, K, n = self._m, int(self._m.K), int(data.n_docs)
        out = torch.empty(n, 2 * K if moments else K, dtype=torch.float32, device=self.device)
        if n:
            ctx = m.input != abi.IN_BOW
            if ctx and data.contextual is None:
                raise RuntimeError("CTM inference needs the contextual embeddings")
            if chunk is None:       # the CombinedTM adapt_bert output is [chunk, V]: <= 1 GiB
                chunk = (1 << 16) if not ctx else max(256, min(1 << 16, (1 << 28) // max(m.V, 1)))
            cu = torch.cuda.get_device_properties(self.device).multi_processor_count
            stream = torch.cuda.current_stream(self.device).cuda_stream
            for d0 in range(0, n, chunk):
                d1 = min(n, d0 + chunk)
                hctx = self._ctx_dense(data, d0, d1).contiguous() if ctx else None
                p = abi.GfkInfer()
                p.indptr = data.indptr.data_ptr() + 4 * d0
                p.indices, p.values = data.indices.data_ptr(), data.values.data_ptr()
                p.hctx = hctx.data_ptr() if hctx is not None else None
                p.out = out.data_ptr() + 4 * d0 * out.shape[1]
                p.n_docs, p.n_samples = d1 - d0, int(n_samples)
                p.flags = (abi.INFER_POSTPROCESS if postprocess else 0) | \
                    (abi.INFER_MOMENTS if moments else 0)
                p.thr, p.seed, p.doc0 = float(threshold), int(seed) % (1 << 64), d0
                p.grid = int(max(1, min(-(-(d1 - d0) // 8), 4 * cu)))   # 8 waves (docs) per WG
                self._sync_dev()
                rc = self.lib.gfk_theta_infer(C.byref(m), C.byref(p), stream)
                if rc:
                    raise RuntimeError(f"gfk_theta_infer failed ({rc})")
        return out.view(n, 2, K) if moments else out

    # ------------------------------------------------------------------ step
    def _launch(self, phases):
        if any(p in abi.HOST_PHASES for p in phases):
            run: List[int] = []
            for p in list(phases) + [None]:
                if p is None or p in abi.HOST_PHASES:
                    if run:
                        self._launch_native(run)
                        run = []
                    if p == abi.PH_CTX_FWD:
                        self._ctx_fwd()
                    elif p == abi.PH_CTX_BWD:
                        self._ctx_bwd()
                    elif p == abi.PH_FEDAVG_BETA:
                        self._fedavg_beta()
                    elif p == abi.PH_FEDAVG_WA:
                        self._fedavg_wa()
                    elif p == abi.PH_FEDAVG_END:
                        self._fedavg_end()
                    elif p == abi.PH_LB_GEMM_FWD:
                        self._lb_gemm_fwd()
                    elif p == abi.PH_LB_GEMM_BWD:
                        self._lb_gemm_bwd()
                else:
                    run.append(p)
            return
        self._launch_native(phases)

    def _sync_dev(self):
        """Upload the model / update descriptors if the host structs changed (a stream-
        ordered copy; never inside a graph capture: captures sync first)."""
        bm, bu = bytes(self._m), bytes(self._u)
        if (bm, bu) == self._dev_bytes:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("fused engine descriptors changed inside a graph capture")
        self._dev_m.copy_(torch.frombuffer(bytearray(bm), dtype=torch.uint8))
        self._dev_u.copy_(torch.frombuffer(bytearray(bu), dtype=torch.uint8))
        self._dev_bytes = (bm, bu)

    def _launch_native(self, phases):
        self._sync_dev()
        arr, n = abi.phase_array(phases)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = self.lib.gfk_run(C.byref(self._m), C.byref(self._a), self.adam_grid,
                              C.byref(self._u), stream, arr, n)
        if rc:
            raise RuntimeError(f"gfk_run failed: code {rc}")

    def run_phases(self, phases):
        """Launch a subset of the step's kernels (tests inspect intermediates)."""
        self._launch(phases)

    def _invalidate_graph(self):
        # the generation lets external captures (LocalFederation's round graph) see that
        # the kernel arguments / buffers they baked in are stale
        self._graph = None
        self._graphs_k = {}
        self.graph_gen += 1

    @property
    def host_gemm_fallback(self) -> bool:
        """True when part of the step runs as host-issued library GEMMs: the CTM contextual
        path outside the fused ctx kernels' plan (_plan_ctx), or the large-batch plan's
        decoder (_plan_large_batch)."""
        return (self.kind == "ctm" and not self.ctx_fused) or self.large_batch

    def _warm_host_gemms(self):
        """hipBLASLt picks algorithms / workspaces on a shape's first call, which is not
        allowed while capturing: run the host GEMMs once eagerly (their outputs are fully
        rewritten by the next step before anything reads them)."""
        if self._ctx is not None and not self.ctx_fused:
            self._ctx_fwd()
            self._ctx_bwd()
        if self.large_batch and self._m.kind == abi.KIND_PRODLDA:
            if not self._m.lb_fused & 1:
                self._lb_gemm_fwd()
            if not self._m.lb_fused & 2:
                self._lb_gemm_bwd()
        torch.cuda.synchronize(self.device)

    def enable_graph(self, on: bool = True):
        self.graph_enabled = on
        self._invalidate_graph()

    def _capture(self, k: int = 1):
        # warm-up on a side stream is not needed: no lazy allocation in gfk_run
        if self.host_gemm_fallback:
            self._warm_host_gemms()
        self._sync_dev()
        g = torch.cuda.CUDAGraph()
        saved = (self.d_step.clone(), self.adam_t.clone(), self.adam_pow.clone(),
                 self.adam_coef.clone())
        with graph_capture(g):
            for _ in range(k):
                self._launch(self.phases())
        # capture does not execute; restore the device counters defensively
        self.d_step.copy_(saved[0])
        self.adam_t.copy_(saved[1])
        self.adam_pow.copy_(saved[2])
        self.adam_coef.copy_(saved[3])
        if k == 1:
            self._graph = g
        else:
            self._graphs_k[k] = g

    def warm_graph(self):
        """Capture the step graph now (no execution), so the first timed / collective
        step is a plain replay on every rank."""
        if self.graph_enabled and self._graph is None:
            self._capture()

    # ---- external capture (LocalFederation's round graph: all clients' steps and
    # the in-process FedAvg kernel in one hipGraph)
    def prepare_external_capture(self):
        """Run anything that must not happen for the first time inside a capture."""
        self._sync_dev()
        if self.host_gemm_fallback:
            self._warm_host_gemms()

    def launch_step_phases(self):
        """Enqueue one step's kernels on the current stream (no graph of its own;
        the device step counter advances itself, the host tracks it with
        :meth:`advance_host_step`)."""
        if self._comm is not None:
            raise RuntimeError("external capture is for in-process federations (no collective)")
        self._launch(self.phases())

    def advance_host_step(self, s: int):
        self._host_step = s + 1

    def sync_step_counter(self, s: int):
        if s != self._host_step:
            self.d_step.fill_(s)
            self._host_step = s
            self._launch([abi.PH_BATCH_PREP])   # the step's batch is prepared by the previous one

    @property
    def grad_buffer(self) -> torch.Tensor:
        return self.grad

    def compute_grads(self, s: int) -> torch.Tensor:
        """The step's kernels without the optimizer (gradient mode): the gradients are
        left in ``grad`` for an all-reduce before :meth:`apply_grads`."""
        if self.update_mode != UPDATE_GRAD or self.fedavg_scale is not None:
            raise RuntimeError("gradient aggregation needs gradient mode without the FedAvg pre-scale")
        if self.plan is None:
            raise RuntimeError("bind_data() first")
        self.sync_step_counter(s)
        self._launch([p for p in self.phases() if p not in (abi.PH_ADAM, abi.PH_FEDAVG_BETA,
                                                           abi.PH_FEDAVG_WA, abi.PH_FEDAVG_END)])
        self._host_step = s + 1
        return self.loss_hist[s]

    def apply_grads(self, s: int):
        self._launch([abi.PH_ADAM])

    def step(self, s: int) -> torch.Tensor:
        if self.plan is None:
            raise RuntimeError("bind_data() first")
        self.sync_step_counter(s)
        if self.graph_enabled:
            if self._graph is None:
                self._capture()
            self._graph.replay()
        else:
            self._launch(self.phases())
        if self._comm is not None and self._comm["mode"] == "eager":
            agg, buf = self._comm["rest"]
            agg.allreduce_(buf)
        self._host_step = s + 1
        return self.loss_hist[s]

    def steps_per_replay_ok(self) -> bool:
        """Several steps may share one graph replay (:meth:`step_k`): the graph is on and
        nothing runs on the host between steps (no eager all-reduce)."""
        return self.graph_enabled and not (self._comm is not None and self._comm["mode"] == "eager")

    def step_k(self, s: int, k: int) -> torch.Tensor:
        """Steps s .. s + k - 1 in one replay of a k-step graph (the step is device-driven:
        its batch, counter and in-graph all-reduce), the same work as k :meth:`step` calls
        without the graph-to-graph gaps."""
        if k <= 1:
            return self.step(s)
        if self.plan is None:
            raise RuntimeError("bind_data() first")
        if not self.steps_per_replay_ok():
            raise RuntimeError("step_k needs the step graph and no host-side collective")
        self.sync_step_counter(s)
        g = self._graphs_k.get(k)
        if g is None:
            self._capture(k)
            g = self._graphs_k[k]
        g.replay()
        self._host_step = s + k
        return self.loss_hist[s + k - 1]

    # ------------------------------------------------------------------ misc
    def optimizer_state_dict(self):
        return self.optimizer.state_dict()

    def load_optimizer_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)


# the GfkModel fields that fix a launch's grid, block and LDS: engines batched into one
# launch per phase must agree on all of them (their pointers and per-client values differ)
_BATCH_SHAPE_FIELDS = ("bmax", "V", "ldb", "K", "n_hidden", "act", "kind", "input", "C", "L", "vb", "ctx_parts",
                       "n_tiles", "dec_grid", "learn_priors", "stage_flags", "kt", "n_dpart",
                       "update_mode", "ctx_fused", "ctx_kb", "ctx_ckb", "mm_bf16",
                       "lab_on", "lab_off", "lab_in_enc", "bwd_pre")


class BatchedSteps:
    """One launch per phase for the local steps of several fused engines (clients).

    Every kernel reads its GfkModel / GfkUpdate from a device array indexed by blockIdx.z
    (csrc gfk_dev / gfk_grid), so M clients' step = the kernels of ONE client with
    gridDim.z = M: a K = 50 client fills ~70 of the 256 CUs per kernel, M of them fill the
    GPU in the same few microseconds, instead of M graph branches of small kernels
    competing for hardware queues.  Requirements: the same shapes (_BATCH_SHAPE_FIELDS),
    the same phase list, every phase native (no host GEMMs / host collectives)."""

    def __init__(self, engines: List["FusedEngine"]):
        self.validate(engines)
        self.engines = list(engines)
        e0 = engines[0]
        self.device = e0.device
        M = len(engines)
        self._arr_m = torch.zeros(M * C.sizeof(abi.GfkModel), dtype=torch.uint8, device=self.device)
        self._arr_u = torch.zeros(M * C.sizeof(abi.GfkUpdate), dtype=torch.uint8, device=self.device)
        self._blob = None
        self._host = None
        self._phases = e0.phases()
        self._cu = torch.cuda.get_device_properties(self.device).multi_processor_count
        self._fold = None                 # abi.GfkFold when the FedAvg runs in the epilogues
        self._fold_left = None            # its device table of leftover pieces

    @staticmethod
    def possible(engines) -> bool:
        try:
            BatchedSteps.validate(engines)
            return True
        except (ValueError, AttributeError):
            return False

    @staticmethod
    def validate(engines):
        if len(engines) < 1:
            raise ValueError("no engines")
        e0 = engines[0]
        ph = e0.phases()
        if abi.PH_ADAM in ph:
            raise ValueError("batched launches run the fused update mode (no generic optimizer)")
        for e in engines:
            if e.device != e0.device:
                raise ValueError("batched engines must share a device")
            if e.phases() != ph:
                raise ValueError("batched engines must run the same phases")
            if any(p in abi.HOST_PHASES for p in ph) \
                    or e._comm is not None:
                raise ValueError("batched launches need native phases only")
            for f in _BATCH_SHAPE_FIELDS:
                a, b = getattr(e._m, f), getattr(e0._m, f)
                if (list(a) if hasattr(a, "__len__") else a) != (list(b) if hasattr(b, "__len__") else b):
                    raise ValueError(f"batched engines differ in {f}")
            if list(e._m.H) != list(e0._m.H) or e._u.n_w != e0._u.n_w or e._u.n_v != e0._u.n_v:
                raise ValueError("batched engines differ in their layer / job tables")

    def _refresh(self):
        M = len(self.engines)
        ms, us = [], []
        for e in self.engines:
            mm = abi.GfkModel.from_buffer_copy(bytes(e._m))
            mm.dev, mm.dev_upd, mm.n_batch = self._arr_m.data_ptr(), self._arr_u.data_ptr(), M
            # the strip forward: M clients' tiles in one launch of 16-wave workgroups (one per
            # CU).  The strips are grid-strided (a workgroup's wave group g takes tiles
            # g grid + x, so any grid works): where M clients' one-tile-per-workgroup grids
            # exceed one round of the CUs, each workgroup takes T whole tiles (one strip per
            # wave), T the FEWEST in 1..4 whose M ceil(n_tiles / T) workgroups still fit one
            # round -- T = 3 at M = 8, V = 4.7k: 192 workgroups of 12 busy waves instead of
            # 144 of 16; past 4 tiles the M clients share one round (dec_grid = CUs / M).
            # GFEDNTM_BATCH_STRIP=keep: the engines' own grids (rounds of the CUs).
            if (mm.stage_flags & STAGE_FWD_STRIP and M > 1 and M * mm.dec_grid > self._cu
                    and os.environ.get("GFEDNTM_BATCH_STRIP", "fill") != "keep"):
                t = next((t for t in (1, 2, 3, 4) if M * -(-mm.n_tiles // t) <= self._cu), None)
                mm.dec_grid = -(-mm.n_tiles // t) if t else max(1, self._cu // M)
            # NeuralLDA's decoder kernels (beta forward / backward, grid-strided over the
            # tiles) likewise: T tiles per workgroup so the M clients' workgroups fit one
            # round of the CUs -- the backward's theta_d staging is then paid once per T
            # tiles (8 clients, V = 4.7k: 0.1426 -> 0.1407 ms, same bits; one round of two
            # workgroups per CU measured 0.1497, profiles/r6/lda/ab_batch_fill.txt).
            # GFEDNTM_BATCH_STRIP=keep: the engines' own grids here too.
            if (mm.kind == abi.KIND_LDA and M > 1 and M * mm.dec_grid > self._cu
                    and os.environ.get("GFEDNTM_BATCH_STRIP", "fill") != "keep"):
                t = next((t for t in (1, 2, 3, 4) if M * -(-mm.n_tiles // t) <= self._cu), None)
                mm.dec_grid = -(-mm.n_tiles // t) if t else max(1, self._cu // M)
            # the posterior folded into the strip forward for M > 1 clients (the engines' own
            # plan keeps post_fwd for one client; GFEDNTM_POSTFOLD=0: never)
            if (M > 1 and getattr(e, "_fold_ok", False) and mm.stage_flags & STAGE_FWD_STRIP
                    and os.environ.get("GFEDNTM_POSTFOLD", "auto") != "0"):
                mm.stage_flags |= STAGE_FWD_POSTFOLD
            # post_bwd: M clients x (bmax + 1) workgroups of 16 waves with the batch matrices
            # in LDS (~93 KB: one per CU) run in three rounds at M = 8.  Two rows per
            # workgroup (the matrices, weights and column sums staged once for both) and the
            # batch-level workgroup moved into row_bwd: M bmax / 2 workgroups, one round
            # (M (bmax + 1) <= CUs: the one-row shape).  Round 6 removed the opt-in variants
            # measured slower: the matrices read from L2, and the persistent one-range
            # backward walking several tiles (profiles/r5/ab_batch.txt).
            if M > 1 and M * (mm.bmax + 1) > self._cu:
                mm.stage_flags |= STAGE_POST_ROWS2
            # CombinedTM: M clients' vocabulary tiles in one launch fill the CUs the way one
            # client's do at a large vocabulary, so the batched launch takes that plan -- the
            # forward with all batch rows per tile (each Wa block staged once) and the
            # persistent pipelined backward -- once M n_tiles > 2 CUs (V = 5k, 8 clients:
            # 0.5296 -> 0.5175 / 0.5137 ms each, profiles/r6/ctm_batched/).  The z0 partials
            # keep the per-tile layout (no register-streamed forward here).
            # GFEDNTM_CTX_FULL / GFEDNTM_CTX_BWDPP = 0: the engines' own plan.
            if (M > 1 and mm.ctx_fused == 1 and mm.bmax <= 64 and int(mm.H[0]) <= 64
                    and M * mm.n_tiles > 2 * self._cu):
                ctx_new = False
                if (not mm.stage_flags & STAGE_CTX_FULL
                        and os.environ.get("GFEDNTM_CTX_FULL", "auto") == "auto"):
                    mm.stage_flags |= STAGE_CTX_FULL
                    ctx_new = True
                if (not mm.stage_flags & STAGE_CTX_BWDPP
                        and os.environ.get("GFEDNTM_CTX_BWDPP", "auto") == "auto"):
                    mm.stage_flags |= STAGE_CTX_BWDPP
                    mm.ctx_bgrid = int(self._cu)
                    ctx_new = True
                if ctx_new:                  # (the new kernels' dynamic-LDS limit)
                    rc = e.lib.gfk_setup(C.byref(mm))
                    if rc:
                        raise RuntimeError(f"gfk_setup failed ({rc})")
            # win_update: all clients' W_in tiles in one launch -> the 8-wave tile shape once
            # they exceed two rounds of 16-wave workgroups
            if M * (mm.n_tiles + 8) > 2 * self._cu:
                mm.stage_flags |= STAGE_WIN_BATCH8
            ms.append(bytes(mm))
            us.append(bytes(e._u))
        # the phases of the batched plan: post_fwd out where the launch folds it, back in
        # where the launch dropped the engines' fold
        ph = list(self.engines[0].phases())
        folded = bool(abi.GfkModel.from_buffer_copy(ms[0]).stage_flags & STAGE_FWD_POSTFOLD)
        if folded and abi.PH_POST_FWD in ph:
            ph.remove(abi.PH_POST_FWD)
        elif not folded and abi.PH_PRODLDA_FWD in ph and abi.PH_POST_FWD not in ph:
            ph.insert(ph.index(abi.PH_PRODLDA_FWD), abi.PH_POST_FWD)
        self._phases = ph
        blob = b"".join(ms) + b"".join(us)
        if blob != self._blob:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("batched engine descriptors changed inside a graph capture")
            self._arr_m.copy_(torch.frombuffer(bytearray(b"".join(ms)), dtype=torch.uint8))
            self._arr_u.copy_(torch.frombuffer(bytearray(b"".join(us)), dtype=torch.uint8))
            self._blob = blob
        self._host = abi.GfkModel.from_buffer_copy(ms[0])
        if self._fold is not None:
            self._upload_fold_table()

    def prepare(self):
        """Upload the descriptors now (before a capture)."""
        self._refresh()

    # ---- the FedAvg in the update epilogues (csrc/prodlda.hip gfk_bwd_fold_k,
    #      csrc/update.hip gfk_win_fold_k) ----
    FOLD_PIECE = 1024                     # floats per leftover workgroup (256 threads x float4)

    def _fold_owned(self) -> Dict[int, str]:
        """Flat offsets of the shared slots the fold kernels' update jobs own (beta, W_in,
        every weight / vector job's parameter) -> key."""
        e0 = self.engines[0]
        base = e0.flat.buffer.data_ptr()
        by_off = {s.offset: k for k, s in e0.flat.slots.items()}
        owned = {}
        ptrs = [int(e0._m.beta), int(e0._m.w_in)]
        ptrs += [int(e0._u.w[i].param) for i in range(e0._u.n_w)]
        ptrs += [int(e0._u.v[i].param) for i in range(e0._u.n_v)]
        for p in ptrs:
            off = (p - base) // 4
            if (p - base) % 4 or off not in by_off:
                raise ValueError("an update job's parameter is not a slot of the flat buffer")
            owned[off] = by_off[off]
        return owned

    def fold_reason(self) -> Optional[str]:
        """Why the in-epilogue FedAvg cannot run this launch (None: it can).  The fold
        kernels cover the headline plan: ProdLDA, bag of words, fused Adam, fp32, bmax 64,
        K and every hidden layer <= 64, one d theta_d slab per tile, dense W_in tiles,
        every parameter in the shared prefix and pre-scaled."""
        e0 = self.engines[0]
        m = self._host if self._host is not None else e0._m
        if not hasattr(e0.lib, "gfk_bwd_fold_launch"):
            return "kernel library without the fold kernels"
        checks = [
            (m.kind == abi.KIND_PRODLDA, "ProdLDA only"),
            (m.input == abi.IN_BOW and not m.lab_on, "bag-of-words input without a label head"),
            (e0.update_mode == UPDATE_FUSED, "fused Adam epilogues only"),
            (not m.mm_bf16, "fp32 GEMM operands only"),
            (m.K <= 64 and m.bmax == 64, "K <= 64 and batch 64 only"),
            (max(int(m.H[i]) for i in range(m.n_hidden)) <= 64, "hidden layers <= 64 only"),
            (not m.bwd_pre and m.n_dpart == m.n_tiles,
             "the one-slab-per-tile backward only"),
            (not m.stage_flags & (STAGE_WIN_SPARSE | STAGE_LB),
             "dense W_in tiles only"),
            (m.kt % 2 == 0, "theta_d stride"),
            (all(e0._u.v[i].n <= 64 for i in range(e0._u.n_v)), "vector jobs <= 64 long"),
            (e0._u.n_w <= abi.FOLD_W and e0._u.n_v <= abi.FOLD_V, "too many update jobs"),
        ]
        for ok, why in checks:
            if not ok:
                return why
        for e in self.engines:
            fl = e.flat
            if any(s.offset + s.numel > fl.n_shared for s in fl.param_slots()):
                return "a parameter outside the shared prefix"
            if not e._m.fed_scale_on:
                return "no FedAvg pre-scale"
        try:
            owned = self._fold_owned()
        except ValueError as exc:
            return str(exc)
        fl = e0.flat
        for k in fl.shared_keys:
            s = fl.slots[k]
            if s.offset not in owned and s.is_param:
                return f"parameter {k} has no fold job"
        return None

    def set_fold(self, mode: Optional[int]):
        """mode abi.FOLD_ALL / FOLD_FIRST: replace prodlda_bwd and win_update by the fold
        kernels (the round's in-rank FedAvg inside their epilogues; every client's state must
        be the same at the start of each round -- the caller's invariant); None: off."""
        if mode is None:
            self._fold = None
            return
        why = self.fold_reason()
        if why is not None:
            raise ValueError(f"in-epilogue FedAvg not available: {why}")
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("set_fold inside a graph capture")
        e0 = self.engines[0]
        owned = self._fold_owned()
        pieces = []
        for k in e0.flat.shared_keys:
            s = e0.flat.slots[k]
            if s.offset in owned:
                continue
            for a in range(0, s.numel, self.FOLD_PIECE):
                pieces += [s.offset + a, min(self.FOLD_PIECE, s.numel - a)]
        if any(p % 4 for p in pieces[0::2]):
            raise ValueError("leftover pieces must start on 16-byte boundaries")
        self._fold_left = torch.tensor(pieces or [0, 0], dtype=torch.int64, device=self.device)
        M = len(self.engines)
        self._fold_cl = torch.zeros(M * C.sizeof(abi.GfkFoldClient), dtype=torch.uint8,
                                    device=self.device)
        self._fold_cl_bytes = None
        f = abi.GfkFold()
        f.models, f.upds = self._arr_m.data_ptr(), self._arr_u.data_ptr()
        f.left = self._fold_left.data_ptr()
        f.M, f.mode, f.n_left = M, int(mode), len(pieces) // 2
        f.nj = -(-int(e0._m.H[0]) // 16)
        f.cl = self._fold_cl.data_ptr()
        self._fold = f
        self._upload_fold_table()

    @staticmethod
    def _fold_client(e) -> "abi.GfkFoldClient":
        """One client's pointer table for the fold kernels (csrc GfkFoldClient)."""
        m, u = e._m, e._u
        c = abi.GfkFoldClient()
        base = int(m.flat_base)

        def moments(p):
            p = int(p)
            return p, p + 4 * int(m.off_m), p + 4 * int(m.off_v)

        def scale(p):
            return float(m.fed_scale) if (m.fed_scale_on and (int(p) - base) // 4 < int(m.n_shared)) else 1.0

        c.tstart, c.indices, c.values, c.nb = m.ws_tstart, m.indices, m.values, m.ws_nb
        c.coef, c.zn, c.thetad, c.lse, c.s, c.rstd = (m.adam_coef, m.ws_zn, m.ws_thetad, m.ws_lse,
                                                       m.ws_s, m.ws_col_rstd)
        c.beta, c.beta_m, c.beta_v = moments(m.beta)
        c.dthetad, c.dz0 = m.ws_dthetad, m.ws_dz[0]
        c.w_in, c.w_in_m, c.w_in_v = moments(m.w_in)
        c.flat = base
        c.beta_sc, c.win_sc = scale(m.beta), scale(m.w_in)
        c.b1, c.b2, c.eps, c.wd = m.beta1, m.beta2, m.adam_eps, m.weight_decay
        for j in range(u.n_w):
            J = u.w[j]
            c.wdz[j], c.wa[j] = J.dz, J.a
            c.wp[j], c.wm[j], c.wv[j] = moments(J.param)
            c.wsc[j] = scale(J.param)
        for j in range(u.n_v):
            J = u.v[j]
            c.vsrc[j] = J.src
            c.vp[j], c.vm[j], c.vv[j] = moments(J.param)
            c.vg[j] = int(J.param) + 4 * int(m.off_g)
            c.vsc[j] = scale(J.param)
        return c

    def _upload_fold_table(self):
        blob = b"".join(bytes(self._fold_client(e)) for e in self.engines)
        if blob != self._fold_cl_bytes:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("fold client table changed inside a graph capture")
            self._fold_cl.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
            self._fold_cl_bytes = blob

    @property
    def fold_mode(self) -> Optional[int]:
        return None if self._fold is None else int(self._fold.mode)

    def _run_fold(self, phase: int):
        e0 = self.engines[0]
        stream = torch.cuda.current_stream(self.device).cuda_stream
        if phase == abi.PH_FOLD_BWD:
            rc = e0.lib.gfk_bwd_fold_launch(C.byref(self._host), C.byref(self._fold), stream)
        else:
            rc = e0.lib.gfk_win_fold_launch(C.byref(self._host), C.byref(e0._u),
                                            C.byref(self._fold), stream)
        if rc:
            raise RuntimeError(f"fold kernel launch failed: code {rc} (phase {phase})")

    def _run(self, phases):
        e0 = self.engines[0]
        arr, n = abi.phase_array(phases)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        rc = e0.lib.gfk_run(C.byref(self._host), C.byref(e0._a), e0.adam_grid,
                            C.byref(e0._u), stream, arr, n)
        if rc:
            raise RuntimeError(f"gfk_run (batched) failed: code {rc}")

    def launch(self, after=None):
        """Enqueue one local step of every engine on the current stream.  ``after``:
        {phase: callable} called (on the host, while enqueuing) right after that phase's
        launch -- the multi-client rank round forks beta's FedAvg there."""
        self._refresh()
        after = dict(after or {})
        phases = list(self._phases)
        if self._fold is not None:
            swap = {abi.PH_PRODLDA_BWD: abi.PH_FOLD_BWD, abi.PH_ENC_BWD: abi.PH_FOLD_WIN}
            phases = [swap.get(p, p) for p in phases]
            after = {swap.get(p, p): f for p, f in after.items()}
        run: List[int] = []
        for p in phases + [None]:
            if p is not None and p not in (abi.PH_FOLD_BWD, abi.PH_FOLD_WIN):
                run.append(p)
                if p not in after:
                    continue
            if run:
                self._run(run)
                run = []
            if p in (abi.PH_FOLD_BWD, abi.PH_FOLD_WIN):
                self._run_fold(p)
            if p in after:
                after[p]()

    def wa_final_phase(self) -> Optional[int]:
        """The phase after which every client's adapt_bert (CombinedTM) is final in the
        fused update mode, or None."""
        e0 = self.engines[0]
        if e0.update_mode != UPDATE_FUSED or abi.PH_CTXF_BWD not in self._phases:
            return None
        return abi.PH_CTXF_BWD

    def beta_final_phase(self) -> Optional[int]:
        """The phase after which every client's beta is final in the fused update mode
        (Adam + the FedAvg pre-scale in its epilogue), or None."""
        e0 = self.engines[0]
        if e0.update_mode != UPDATE_FUSED:
            return None
        for p in (abi.PH_PRODLDA_BWD, abi.PH_LDA_BETA_BWD):
            if p in self._phases:
                return p
        return None
