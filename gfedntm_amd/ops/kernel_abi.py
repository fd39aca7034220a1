"""ctypes mirror of the C ABI in csrc/gfk_common.h and csrc/step.cpp.

Field order and types MUST match the C structs; :func:`declare` checks the
struct sizes against the library's own ``sizeof`` at load time.
"""
from __future__ import annotations

import ctypes as C

MAX_LAYERS = 8
MAX_SEGS = 48
P = C.c_void_p

# activation / model / input codes
ACT_CODES = {"softplus": 0, "relu": 1, "sigmoid": 2, "tanh": 3, "leakyrelu": 4, "elu": 5,
             "selu": 6, "rrelu": 7}
KIND_PRODLDA, KIND_LDA = 0, 1
IN_BOW, IN_COMBINED, IN_CONTEXTUAL = 0, 1, 2

# phase ids (csrc/step.cpp GfkPhase)
PH_BATCH_DOCS = 0
PH_ENC_FWD = 1
PH_POST_FWD = 2
PH_PRODLDA_FWD = 3
PH_PRODLDA_LOSS = 4
PH_PRODLDA_BWD = 5
PH_LDA_BETA_FWD = 6
PH_LDA_ROW = 7
PH_POST_BWD = 8
PH_LDA_BETA_BWD = 9
PH_ENC_BWD = 10
PH_ADAM = 11
PH_BATCH_PREP = 12
PH_CTXF_FWD = 13      # CombinedTM contextual forward on the fused kernels (ctx_fwd)
PH_CTXF_BWD = 14      # ... and its backward + adapt_bert updates (ctx_bwd)

# PH_ENC_FWD = enc_in (sparse gather, MLP, heads, random draws), PH_POST_FWD =
# post_fwd (batch-norm, reparameterisation, softmax, KL), PH_POST_BWD = row_bwd +
# post_bwd, PH_ENC_BWD = win_update (W_in tiles, small-tensor gradient tiles,
# fused updates, next-batch prep).  In fused-update mode the optimizer step lives
# in the kernel epilogues; gradient mode appends the generic Adam.
# host-side phases (CTM): the dense contextual GEMMs around the fused kernels,
# issued on the same stream (hipBLASLt through torch) and captured in the same graph
PH_CTX_FWD = 100
PH_CTX_BWD = 101
# host-side phases (multi-GPU): the FedAvg all-reduce of beta (on a side stream,
# overlapping the encoder backward) and of the rest of the shared state
PH_FEDAVG_BETA = 102
PH_FEDAVG_END = 103
# (104 - 106: round 5's split beta / W_in update phases, removed in round 6)
# CombinedTM (fused): adapt_bert's share of the FedAvg forked onto the side stream once
# ctx_bwd has finished it (overlapping win_update), behind beta's
PH_FEDAVG_WA = 107
# the large-batch plan (bmax 256 / 512): ProdLDA's decoder products as hipBLASLt GEMMs on the
# step's stream -- logits = theta_d beta before prodlda_lb_colbn (PH_PRODLDA_FWD), dbeta and
# d theta_d after prodlda_lb_dlogit (PH_PRODLDA_BWD)
PH_LB_GEMM_FWD = 108
PH_LB_GEMM_BWD = 109
# batched clients with the FedAvg in the update epilogues (ops/engine.py BatchedSteps.set_fold):
# csrc/prodlda.hip gfk_bwd_fold_k in place of PH_PRODLDA_BWD, csrc/update.hip gfk_win_fold_k
# in place of PH_ENC_BWD (launched by the batched plan, not by gfk_run)
PH_FOLD_BWD = 110
PH_FOLD_WIN = 111
HOST_PHASES = (PH_CTX_FWD, PH_CTX_BWD, PH_FEDAVG_BETA, PH_FEDAVG_END, PH_FEDAVG_WA, PH_LB_GEMM_FWD,
               PH_LB_GEMM_BWD)

PRODLDA_STEP = [PH_ENC_FWD, PH_POST_FWD, PH_PRODLDA_FWD, PH_PRODLDA_LOSS, PH_PRODLDA_BWD,
                PH_POST_BWD, PH_ENC_BWD]
LDA_STEP = [PH_LDA_BETA_FWD, PH_ENC_FWD, PH_POST_FWD, PH_LDA_ROW, PH_POST_BWD, PH_LDA_BETA_BWD,
            PH_ENC_BWD, PH_ADAM]

SEG_ADAM, SEG_SCALE, SEG_KEEP_GRAD = 1, 2, 4


class GfkModel(C.Structure):
    _fields_ = [
        ("bmax", C.c_int32), ("V", C.c_int32), ("K", C.c_int32), ("n_hidden", C.c_int32),
        ("H", C.c_int32 * MAX_LAYERS),
        ("act", C.c_int32), ("kind", C.c_int32), ("input", C.c_int32), ("C", C.c_int32),
        ("L", C.c_int32), ("vb", C.c_int32), ("n_tiles", C.c_int32), ("dec_grid", C.c_int32),
        ("learn_priors", C.c_int32), ("stage_flags", C.c_int32), ("kt", C.c_int32),
        ("scatter_chunks", C.c_int32), ("n_dpart", C.c_int32), ("n_steps", C.c_int32),
        ("drop_enc", C.c_float), ("drop_theta", C.c_float), ("bn_momentum", C.c_float),
        ("bn_eps", C.c_float), ("kl_weight", C.c_float), ("lb_fused", C.c_int32),
        ("seed", C.c_uint64),
        ("prior_mean", P), ("prior_var", P), ("beta", P), ("w_in", P), ("b_in", P),
        ("w_h", P * MAX_LAYERS), ("b_h", P * MAX_LAYERS),
        ("w_mu", P), ("b_mu", P), ("w_s", P), ("b_s", P),
        ("mu_rm", P), ("mu_rv", P), ("s_rm", P), ("s_rv", P), ("beta_rm", P), ("beta_rv", P),
        ("nbt_mu", P), ("nbt_s", P), ("nbt_beta", P),
        ("g_prior_mean", P), ("g_prior_var", P), ("g_beta", P), ("g_w_in", P), ("g_b_in", P),
        ("g_w_h", P * MAX_LAYERS), ("g_b_h", P * MAX_LAYERS),
        ("g_w_mu", P), ("g_b_mu", P), ("g_w_s", P), ("g_b_s", P),
        ("indptr", P), ("indices", P), ("values", P), ("ctx", P),
        ("plan_order", P), ("plan_start", P), ("plan_size", P),
        ("step", P), ("adam_t", P), ("loss_hist", P),
        ("ws_doc", P), ("ws_nb", P), ("ws_z", P * MAX_LAYERS), ("ws_a", P * MAX_LAYERS), ("ws_hd", P), ("ws_mask_h", P),
        ("ws_mu_raw", P), ("ws_ls_raw", P), ("ws_mu", P), ("ws_ls", P), ("ws_bn_rstd", P),
        ("ws_eps", P), ("ws_theta", P), ("ws_mask_t", P), ("ws_thetad", P),
        ("ws_kl", P), ("ws_rl", P), ("ws_lse", P), ("ws_s", P),
        ("ws_zn", P), ("ws_col_rstd", P), ("ws_row_part", P), ("ws_dthetad", P),
        ("ws_dz", P * MAX_LAYERS), ("ws_dmr", P), ("ws_dlr", P),
        ("ws_dmu", P), ("ws_dls", P),
        ("ws_dbsm", P), ("ws_ck", P), ("ws_hctx", P), ("ws_tstart", P), ("ws_erange", P),
        ("ws_next", P), ("dbg", P),
        ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("adam_eps", C.c_float),
        ("weight_decay", C.c_float), ("fed_scale", C.c_float), ("update_mode", C.c_int32),
        ("fed_scale_on", C.c_int32), ("flat_base", P), ("n_shared", C.c_int64),
        ("off_m", C.c_int64), ("off_v", C.c_int64), ("off_g", C.c_int64),
        ("adam_pow", P), ("adam_coef", P), ("ws_dtheta", P),
        ("w_a", P), ("b_a", P), ("ws_actx", P), ("ws_hpart", P),
        ("ctx_fused", C.c_int32), ("ctx_kb", C.c_int32), ("ctx_ckb", C.c_int32),
        ("slot_cap", C.c_int32), ("ws_sidx", P), ("ws_sval", P),
        ("mm_bf16", C.c_int32), ("ctx_parts", C.c_int32),
        ("lab_on", C.c_int32), ("lab_off", C.c_int32), ("labels", P), ("w_cls", P), ("b_cls", P),
        ("ws_lab", P), ("ws_dlab", P), ("ws_ce", P), ("ws_thd", P),
        ("lab_in_enc", C.c_int32), ("bwd_pre", C.c_int32), ("ws_dt", P),
        ("dev", P), ("dev_upd", P), ("n_batch", C.c_int32), ("ldb", C.c_int32),
        ("ctx_bgrid", C.c_int32), ("ws_colstat", P),
        ("kl_hist", P), ("rl_hist", P),
    ]


class GfkWJob(C.Structure):
    _fields_ = [("param", P), ("dz", P), ("a", P), ("rows", C.c_int32), ("cols", C.c_int32),
                ("j0", C.c_int32), ("i0", C.c_int32)]


class GfkVJob(C.Structure):
    _fields_ = [("param", P), ("src", P), ("n", C.c_int32), ("pad", C.c_int32)]


MAX_WJOBS, MAX_VJOBS = 40, 16


class GfkUpdate(C.Structure):
    _fields_ = [("n_w", C.c_int32), ("n_v", C.c_int32), ("w", GfkWJob * MAX_WJOBS),
                ("v", GfkVJob * MAX_VJOBS)]


# update rules of the generic optimizer kernel (csrc/gfk_common.h GFK_SOLVER_*)
ADAM_CHUNK = 256      # float4 per workgroup of the generic optimizer kernel (GFK_ADAM_CHUNK)
SOLVER_CODES = {"adam": 0, "sgd": 1, "adagrad": 2, "adadelta": 3, "rmsprop": 4}


class GfkAdam(C.Structure):
    _fields_ = [
        ("p", P), ("g", P), ("m", P), ("v", P),
        ("n_seg", C.c_int32), ("solver", C.c_int32),
        ("seg_start", C.c_int64 * MAX_SEGS), ("seg_end", C.c_int64 * MAX_SEGS),
        ("seg_flags", C.c_int32 * MAX_SEGS),
        ("lr", C.c_float), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
        ("weight_decay", C.c_float), ("scale", C.c_float),
        ("t", P), ("coef", P),
        ("seg_first_block", C.c_int32 * MAX_SEGS), ("dbg", P),
    ]


class GfkInfer(C.Structure):
    """theta-inference launch (csrc/infer.hip)."""
    _fields_ = [("indptr", P), ("indices", P), ("values", P), ("hctx", P), ("out", P),
                ("n_docs", C.c_int32), ("n_samples", C.c_int32), ("flags", C.c_int32),
                ("thr", C.c_float), ("seed", C.c_uint64), ("grid", C.c_int32), ("doc0", C.c_int32)]


INFER_POSTPROCESS, INFER_MOMENTS = 1, 2


FOLD_W, FOLD_V = 8, 16


class GfkFoldClient(C.Structure):
    """One client's pointers for the fold kernels (csrc/gfk_common.h GfkFoldClient)."""
    _fields_ = [("tstart", P), ("indices", P), ("values", P), ("nb", P),
                ("coef", P), ("zn", P), ("thetad", P), ("lse", P), ("s", P), ("rstd", P),
                ("beta", P), ("beta_m", P), ("beta_v", P), ("dthetad", P), ("dz0", P),
                ("w_in", P), ("w_in_m", P), ("w_in_v", P), ("flat", P),
                ("beta_sc", C.c_float), ("win_sc", C.c_float), ("b1", C.c_float), ("b2", C.c_float),
                ("eps", C.c_float), ("wd", C.c_float),
                ("wdz", P * FOLD_W), ("wa", P * FOLD_W), ("wp", P * FOLD_W), ("wm", P * FOLD_W),
                ("wv", P * FOLD_W), ("vsrc", P * FOLD_V), ("vp", P * FOLD_V), ("vm", P * FOLD_V),
                ("vv", P * FOLD_V), ("vg", P * FOLD_V),
                ("wsc", C.c_float * FOLD_W), ("vsc", C.c_float * FOLD_V)]


class GfkFold(C.Structure):
    """The in-epilogue FedAvg of a batched launch (csrc/gfk_common.h GfkFold)."""
    _fields_ = [("models", P), ("upds", P), ("left", P), ("M", C.c_int32), ("mode", C.c_int32),
                ("n_left", C.c_int32), ("nj", C.c_int32), ("cl", P)]


FOLD_ALL, FOLD_FIRST = 0, 1

# optional entry points: name -> (argtypes, restype)
_EXTRA = {
    "gfk_theta_infer": ([C.POINTER(GfkModel), C.POINTER(GfkInfer), C.c_void_p], C.c_int),
    "gfk_theta_infer_smem": ([C.POINTER(GfkModel)], C.c_size_t),
    "gfk_bwd_fold_launch": ([C.POINTER(GfkModel), C.POINTER(GfkFold), C.c_void_p], C.c_int),
    "gfk_win_fold_launch": ([C.POINTER(GfkModel), C.POINTER(GfkUpdate), C.POINTER(GfkFold), C.c_void_p],
                            C.c_int),
}


def declare(lib: C.CDLL) -> None:
    lib.gfk_model_struct_size.restype = C.c_size_t
    lib.gfk_adam_struct_size.restype = C.c_size_t
    if lib.gfk_model_struct_size() != C.sizeof(GfkModel):
        raise RuntimeError(f"GfkModel ABI mismatch: C {lib.gfk_model_struct_size()} vs "
                           f"ctypes {C.sizeof(GfkModel)}")
    if lib.gfk_adam_struct_size() != C.sizeof(GfkAdam):
        raise RuntimeError(f"GfkAdam ABI mismatch: C {lib.gfk_adam_struct_size()} vs "
                           f"ctypes {C.sizeof(GfkAdam)}")
    lib.gfk_update_struct_size.restype = C.c_size_t
    if lib.gfk_update_struct_size() != C.sizeof(GfkUpdate):
        raise RuntimeError("GfkUpdate ABI mismatch")
    lib.gfk_setup.argtypes = [C.POINTER(GfkModel)]
    lib.gfk_setup.restype = C.c_int
    lib.gfk_run.argtypes = [C.POINTER(GfkModel), C.POINTER(GfkAdam), C.c_int, C.POINTER(GfkUpdate),
                            C.c_void_p, C.POINTER(C.c_int32), C.c_int]
    lib.gfk_run.restype = C.c_int
    lib.gfk_smem_required.argtypes = [C.POINTER(GfkModel), C.c_int]
    lib.gfk_smem_required.restype = C.c_size_t
    lib.gfk_scale.argtypes = [C.c_void_p, C.c_int64, C.c_float, C.c_void_p]
    lib.gfk_scale.restype = C.c_int
    lib.gfk_launch_adam.argtypes = [C.POINTER(GfkAdam), C.c_int, C.c_void_p]
    lib.gfk_launch_adam.restype = C.c_int
    lib.gfk_infer_struct_size.restype = C.c_size_t
    if lib.gfk_infer_struct_size() != C.sizeof(GfkInfer):
        raise RuntimeError("GfkInfer ABI mismatch")
    if hasattr(lib, "gfk_fold_struct_size"):
        lib.gfk_fold_struct_size.restype = C.c_size_t
        lib.gfk_fold_client_struct_size.restype = C.c_size_t
        if (lib.gfk_fold_struct_size() != C.sizeof(GfkFold)
                or lib.gfk_fold_client_struct_size() != C.sizeof(GfkFoldClient)):
            raise RuntimeError("GfkFold ABI mismatch")
    for name, args in _EXTRA.items():
        if hasattr(lib, name):
            f = getattr(lib, name)
            f.argtypes, f.restype = args


def phase_array(phases):
    arr = (C.c_int32 * len(phases))(*phases)
    return arr, len(phases)
