// gfedntm_amd -- common device helpers and the C ABI of the fused NTM step.
//
// Target: gfx950 (MI355X, CDNA4), wave64.  Everything here is written for
// 64-lane wavefronts: row reductions use __shfl_xor over 64 lanes, block sizes
// are multiples of 64, and kernels that own one document use one workgroup of
// 4 waves (256 threads).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define GFK_MAX_LAYERS 8
#define GFK_MAX_SEGS 48
// float4 per workgroup of the generic optimizer kernel (one per thread of a 256-thread
// workgroup: ~450 workgroups for the K=50 model, every CU busy)
#define GFK_ADAM_CHUNK 256
#define GFK_WAVE 64

// ---------------------------------------------------------------------------
// C ABI (mirrored by gfedntm_amd/ops/kernel_abi.py -- keep field order in sync)
// ---------------------------------------------------------------------------
extern "C" {

// Activation codes (reference inference_network.py:45-60).
enum GfkAct { GFK_SOFTPLUS = 0, GFK_RELU = 1, GFK_SIGMOID = 2, GFK_TANH = 3,
              GFK_LEAKYRELU = 4, GFK_ELU = 5, GFK_SELU = 6, GFK_RRELU = 7 };

enum GfkModelKind { GFK_PRODLDA = 0, GFK_LDA = 1 };

// Encoder input kinds: BoW only (AVITM), BoW + adapted contextual (CombinedTM),
// contextual only (ZeroShotTM).
enum GfkInput { GFK_IN_BOW = 0, GFK_IN_COMBINED = 1, GFK_IN_CONTEXTUAL = 2 };

typedef struct GfkModel {
  // ---- dimensions ----
  int32_t bmax;          // max rows per minibatch (grid size of per-row kernels)
  int32_t V, K;          // vocabulary, topics
  int32_t n_hidden;      // len(hidden_sizes)
  int32_t H[GFK_MAX_LAYERS];
  int32_t act;           // GfkAct
  int32_t kind;          // GfkModelKind
  int32_t input;         // GfkInput
  int32_t C;             // contextual size (CTM)
  int32_t L;             // label size (CTM)
  int32_t vb;            // decoder vocab-tile width
  int32_t n_tiles;       // ceil(V / vb)
  int32_t dec_grid;      // workgroups of the vocab-tiled decoder kernels
  int32_t learn_priors;
  int32_t stage_flags;   // bit0: encoder weights fit in LDS, bit1: posterior-bwd stash fits in LDS
  int32_t kt;            // row stride of ws_thetad: K padded to 4 x odd (conflict-free MFMA reads)
  int32_t scatter_chunks;   // grid.y of the input-layer scatter (64 non-zeros per chunk)
  int32_t n_dpart;       // partial slabs of d theta_d ([n_dpart, bmax, K]): n_tiles (ProdLDA), 1 (LDA)
  int32_t n_steps;       // length of the batch plan
  float drop_enc, drop_theta;
  float bn_momentum, bn_eps;
  float kl_weight;       // CTM loss_weights["beta"], 1 for AVITM
  int32_t lb_fused;      // the large-batch plan's decoder on the matrix cores: bit 0 forward,
                         //   bit 1 backward (csrc/prodlda.hip prodlda_lb_fwd / _bwd)
  uint64_t seed;

  // ---- parameters (views into the flat fp32 buffer) and their gradients ----
  float *prior_mean, *prior_var, *beta;
  float *w_in;           // input_layer.weight stored TRANSPOSED: [n_in, H0]
  float *b_in;
  float *w_h[GFK_MAX_LAYERS], *b_h[GFK_MAX_LAYERS];   // hidden l: [H[l+1], H[l]]
  float *w_mu, *b_mu, *w_s, *b_s;                      // [K, H_last]
  float *mu_rm, *mu_rv, *s_rm, *s_rv, *beta_rm, *beta_rv;
  int64_t *nbt_mu, *nbt_s, *nbt_beta;                  // num_batches_tracked
  float *g_prior_mean, *g_prior_var, *g_beta, *g_w_in, *g_b_in;
  float *g_w_h[GFK_MAX_LAYERS], *g_b_h[GFK_MAX_LAYERS];
  float *g_w_mu, *g_b_mu, *g_w_s, *g_b_s;

  // ---- data (device-resident CSR shard + batch plan) ----
  const int32_t *indptr, *indices;
  const float *values;
  const float *ctx;      // [D, C] contextual embeddings (CTM) or null
  const int32_t *plan_order, *plan_start, *plan_size;
  int32_t *step;         // device step counter (index into the plan)
  int32_t *adam_t;       // device Adam step count
  float *loss_hist;      // [n_steps]

  // ---- workspace (fp32 unless noted) ----
  int32_t *ws_doc;       // [bmax] doc ids of the current batch
  int32_t *ws_nb;        // [1]    rows of the current batch
  float *ws_z[GFK_MAX_LAYERS];   // pre-activations per layer [bmax, H[l]]
  float *ws_a[GFK_MAX_LAYERS];   // activations act(z) per layer [bmax, H[l]]
  float *ws_hd;          // dropped-out last hidden [bmax, H_last]
  float *ws_mask_h;      // encoder dropout scale   [bmax, H_last]
  float *ws_mu_raw, *ws_ls_raw;  // [bmax, K] pre-BN heads
  float *ws_mu, *ws_ls;          // [bmax, K] post-BN
  float *ws_bn_rstd;             // [2K] rstd of the mu / log-sigma BN
  float *ws_eps;                 // [bmax, K]
  float *ws_theta, *ws_mask_t;   // [bmax, K]
  float *ws_thetad;              // [bmax, kt] dropped-out theta (zero padding columns)
  float *ws_kl, *ws_rl, *ws_lse, *ws_s;      // [bmax]
  float *ws_zn;                  // ProdLDA: BN'ed logits tiled [n_tiles, bmax, 64]; LDA: BN'ed beta^T [V, K]
  float *ws_col_rstd;            // [n_tiles * 64] (ProdLDA: over batch; LDA: over topics)
  float *ws_row_part;            // online (max, sumexp) partials: ProdLDA [n_tiles*4, bmax, 2], LDA [dec_grid, K, 2]
  float *ws_dthetad;             // [n_dpart, bmax, K] d theta_d partials (plain stores, reduced in order)
  float *ws_dz[GFK_MAX_LAYERS];  // d pre-activation of each hidden layer [bmax, H[l]] (l = 0: input layer)
  float *ws_dmr, *ws_dlr;        // [bmax, K] d mu_raw / d log-sigma_raw (BN backward of the heads)
  float *ws_dmu, *ws_dls;        // [bmax, K] dL/d(post-BN mu, log-sigma)
  float *ws_dbsm;                // LDA: per CSR non-zero of the batch, g = -x / (wd + 1e-10) [nnz]
  float *ws_ck;                  // LDA: [K] sum_v beta_sm * d beta_sm
  float *ws_hctx;                // CTM: dense contextual contribution to layer 0 [bmax, H0]
  int32_t *ws_tstart;            // [bmax, n_tiles+1] CSR position of each row's first nz per vocab tile
  int32_t *ws_erange;            // [bmax, 2] CSR extent (e0, e1) of each row of the current batch
  int32_t *ws_next;              // [1 + 3*bmax] next batch, prepared during the previous step:
                                 //   nb, doc[bmax], (e0, e1)[bmax]
  uint64_t *dbg;                 // diagnostic s_memtime stamps (GFK_STAMPS builds only)

  // ---- update (fused Adam epilogues) ----
  float lr, beta1, beta2, adam_eps, weight_decay, fed_scale;
  int32_t update_mode;           // 0: kernels write gradients (generic Adam follows); 1: fused Adam
  int32_t fed_scale_on;          // multiply shared tensors (flat offset < n_shared) by fed_scale
  float *flat_base;              // the parameter flat buffer
  int64_t n_shared;              // floats of the shared (FedAvg) prefix
  int64_t off_m, off_v, off_g;   // exp_avg / exp_avg_sq / grad slot = parameter pointer + off_*
  double *adam_pow;              // [2] beta1^t, beta2^t (advanced on device with t)
  float *adam_coef;              // [2] lr / (1 - beta1^t), 1 / sqrt(1 - beta2^t)
  float *ws_dtheta;              // [bmax, K] reduced d theta_d

  // ---- CombinedTM contextual path on the fused kernels (csrc/ctx.hip) ----
  float *w_a, *b_a;              // adapt_bert.weight [V, C], adapt_bert.bias [V]
  float *ws_actx;                // [n_tiles][bmax][64] adapted rows A (ctx_fwd)
  float *ws_hpart;               // [n_parts][bmax][H0] contextual z0 partials (per tile, or per
                                 // workgroup of the balanced forward: ctx_parts)
  int32_t ctx_fused;             // 1 (CombinedTM): adapt_bert + contextual input layer in
                                 //    ctx_fwd / ctx_bwd / win_update; 2 (ZeroShotTM): the dense
                                 //    [C, H0] input layer in enc_in / win_update (no host GEMMs)
  int32_t ctx_kb, ctx_ckb;       // backward: C split into ctx_kb chunks of ctx_ckb
  int32_t slot_cap;              // non-zero slots per row of ws_sidx / ws_sval (0: not bound)
  // the next batch's CSR rows copied into fixed slots [bmax][slot_cap] by
  // prepare_next_batch, so a row's non-zeros are one round trip away (no CSR extent
  // first); valid entries j < e1 - e0 of the row
  int32_t* ws_sidx;
  float* ws_sval;
  // ---- precision of the decoder GEMMs (theta.beta, theta^T.dlogit, dlogit.beta^T):
  // 0 = fp32 matrix cores (v_mfma_f32_16x16x4_f32, the reference's precision), 1 = bf16
  // operands, fp32 accumulation (v_mfma_f32_16x16x32_bf16); parameters, Adam state and
  // every other op stay fp32.  The large-V pipelined backward (bwd_pre = 3) keeps fp32
  // operands in both modes: it is bound by beta / Adam-state HBM traffic
  int32_t mm_bf16;
  // CombinedTM forward, balanced persistent shape (stage_flags bit 11): ctx_parts
  // workgroups each own a contiguous range of 16-column units and leave ONE partial of the
  // contextual z0 terms in ws_hpart (0: one partial per vocab tile)
  int32_t ctx_parts;

  // ---- CTM label head (reference ctm decoding_network.py:84-85,156-159, ctm.py:292-296,
  // inference_network.py:64,162): the labels widen the encoder input (rows lab_off ..
  // lab_off + L of the transposed input layer) and feed a Linear(K -> L) classifier on
  // theta_d whose mean cross-entropy against argmax(labels) joins the loss ----
  int32_t lab_on;                // label head active (L > 0)
  int32_t lab_off;               // first input-layer row of the label block
  const float* labels;           // [D, L] the bound dataset's labels
  float *w_cls, *b_cls;          // label_classification weight [L, K], bias [L]
  float *ws_lab;                 // [bmax, L] the batch's label rows (enc_in)
  float *ws_dlab;                // [bmax, L] d CE / d logits, mean over the batch (post_fwd)
  float *ws_ce;                  // [bmax] the rows' CE terms / nb (post_fwd)
  float *ws_thd;                 // [bmax, K] compact theta_d (the classifier's weight-gradient input)
  int32_t lab_in_enc;            // enc_in adds the label rows (0: the host hctx carries them)
  // ---- ProdLDA backward, persistent k-range shape (large vocabularies): the logit
  // gradient dlogit = BN_bwd(p S - x p / (p + 1e-10)) is computed ONCE per vocab tile by
  // prodlda_dlogit into ws_dt ([n_tiles][bmax][66], the bwd's LDS tile layout, copied
  // verbatim by LDS-DMA) instead of by each of the tile's 4 k-range workgroups ----
  int32_t bwd_pre;
  float* ws_dt;
  // ---- batched launches: every kernel reads its model from a DEVICE array of n_batch
  // GfkModels (grid z = the model index), so one launch per phase can run the local
  // steps of several federated clients at once (dev: that array, for a single client a
  // device copy of this struct; dev_upd: the matching GfkUpdate array) ----
  const void* dev;
  const void* dev_upd;
  int32_t n_batch;
  // beta's row stride in floats (>= V: the flat layout pads beta's rows to 128-B lines at
  // large V, utils/flat.py); m / v / the gradient share it
  int32_t ldb;
  // CombinedTM backward, persistent pipelined shape (stage_flags bit 12): workgroups
  // (one per CU) of csrc/ctx.hip gfk_ctx_bwd_pp_k (0: the (tile, chunk) grid)
  int32_t ctx_bgrid;
  // ---- the large-batch plan (stage_flags GFK_LB): the posterior's column statistics,
  // computed once per step (csrc/posterior.hip gfk_post_colstats_lb_k): [mean | rstd] of the
  // raw heads, [sum dy | sum dy xhat] of the backward, the priors' sums, 2K floats each ----
  float* ws_colstat;
  // ---- per-step mean KL and reconstruction terms (metrics, reference federated_avitm.py:109,
  // SURVEY 5.5): written next to loss_hist by the batch-level workgroup when non-null ----
  float* kl_hist;
  float* rl_hist;
} GfkModel;

// stage_flags bit 16 (GFK_FWD_POSTFOLD): the ProdLDA strip forward's ring variant computes
// the batch-coupled posterior itself (csrc/prodlda.hip, FP) and post_fwd is not launched --
// where it applies: strip forward (bit 2), K <= 64, B <= 64, no label head
constexpr int GFK_FWD_POSTFOLD = 65536;
// stage_flags bit 19 (GFK_LB): the large-batch plan, 128 < bmax <= GFK_BMAX_LIMIT.  The
// ProdLDA decoder's three products (logits = theta_d beta, dbeta = theta_d^T dlogit,
// d theta_d = dlogit beta^T) are library GEMMs issued by the engine on the step's stream
// between prodlda_lb_colbn (column batch-norm, BN'ed tiles, row sum-exp partials) and
// prodlda_lb_dlogit (the logit gradient as a plain [bmax][ldb] matrix in ws_dt); the
// row-parallel encoder / posterior kernels run as usual with their batch matrices read
// from L2 (bit 1), the weight-gradient jobs stage the batch in row chunks, NeuralLDA's
// beta backward builds its x^T tile per 128-row chunk; gradient mode + the generic
// optimizer kernel
constexpr int GFK_LB = 524288;
// stage_flags bit 20 (GFK_POST_ROWS2, batched launches): post_bwd takes two rows per
// workgroup, and its batch-level workgroup (prior gradients, the loss, the step counter)
// runs as an extra workgroup of row_bwd instead (its inputs -- mu, log sigma^2, KL, RL --
// are final before row_bwd): M clients' post_bwd is M bmax / 2 workgroups, one round
constexpr int GFK_POST_ROWS2 = 1048576;
constexpr int GFK_BMAX_LIMIT = 512;
// H[n_hidden - 1] without a runtime index into the descriptor (a batched kernel's copy of it
// is promoted to registers only when every access has a constant offset)
__host__ __device__ __forceinline__ int gfk_hlast(const GfkModel& m) {
  int h = m.H[0];
#pragma unroll
  for (int l = 1; l < GFK_MAX_LAYERS; ++l) {
#if defined(__HIP_DEVICE_COMPILE__)
    // (readfirstlane: each field's load stays its own -- a select of the loaded values would
    // be folded into one load from a selected offset)
    const int hl = __builtin_amdgcn_readfirstlane(m.H[l]);
#else
    const int hl = m.H[l];
#endif
    if (l < m.n_hidden) h = hl;
  }
  return h;
}
__host__ __device__ inline bool gfk_postfold(const GfkModel& m) {
  return (m.stage_flags & GFK_FWD_POSTFOLD) && (m.stage_flags & 4) &&
         m.K <= 64 && m.bmax <= 64 && !m.lab_on && m.kind == GFK_PRODLDA;
}

// Gradient + update jobs of the small tensors, run by the update kernel next to
// the W_in tiles (csrc/update.hip).  Weight job: G[j][i] = sum_{b < nb} dz[b][j]
// a[b][i] for the 64 x 64 output tile at (j0, i0) of param [rows][cols].  Vector
// job: g[c] = sum_{b < nb} src[b][c] (src [bmax][n]), or the gradient already in
// the grad slot when src is null (priors, written by post_bwd).
typedef struct GfkWJob {
  float* param;
  const float* dz;
  const float* a;
  int32_t rows, cols, j0, i0;
} GfkWJob;

typedef struct GfkVJob {
  float* param;
  const float* src;
  int32_t n, pad;
} GfkVJob;

#define GFK_MAX_WJOBS 40
#define GFK_MAX_VJOBS 16
typedef struct GfkUpdate {
  int32_t n_w, n_v;
  GfkWJob w[GFK_MAX_WJOBS];
  GfkVJob v[GFK_MAX_VJOBS];
} GfkUpdate;

// Update rules of the generic optimizer kernel (gradient mode), torch.optim
// semantics as the reference constructs them (avitm.py:141-153):
//   ADAM      see adam_update (m = exp_avg, v = exp_avg_sq)
//   SGD       buf = b1 buf + g; p -= lr buf                       (m = momentum_buffer)
//   ADAGRAD   sum += g^2; p -= lr g / (sqrt(sum) + eps)           (v = sum)
//   ADADELTA  sq = b2 sq + (1-b2) g^2; d = sqrt(acc + eps) / sqrt(sq + eps) g;
//             acc = b2 acc + (1-b2) d^2; p -= lr d                (v = square_avg, m = acc_delta)
//   RMSPROP   sq = b2 sq + (1-b2) g^2; buf = b1 buf + g / (sqrt(sq) + eps); p -= lr buf
//                                                                 (v = square_avg, m = momentum_buffer)
enum { GFK_SOLVER_ADAM = 0, GFK_SOLVER_SGD = 1, GFK_SOLVER_ADAGRAD = 2, GFK_SOLVER_ADADELTA = 3,
       GFK_SOLVER_RMSPROP = 4 };

typedef struct GfkAdam {
  float *p, *g, *m, *v;
  int32_t n_seg;
  int32_t solver;                    // GFK_SOLVER_*: update rule of the optimizer segments
  int64_t seg_start[GFK_MAX_SEGS];   // in floats, multiples of 4
  int64_t seg_end[GFK_MAX_SEGS];
  int32_t seg_flags[GFK_MAX_SEGS];   // bit0: Adam update, bit1: FedAvg pre-scale,
                                     // bit2: keep the gradient (it is rewritten whole every step)
  float lr, beta1, beta2, eps, weight_decay, scale;
  const int32_t *t;                  // device Adam step count (already incremented)
  const float *coef;                 // [2] step size, 1/sqrt(bias correction 2) (see GfkModel)
  int32_t seg_first_block[GFK_MAX_SEGS];   // first workgroup of each segment (GFK_ADAM_CHUNK float4 each)
  uint64_t* dbg;                     // diagnostic stamps (GFK_STAMPS builds)
} GfkAdam;

// In-epilogue FedAvg of a rank's batched clients (round 6; csrc/prodlda.hip gfk_bwd_fold_k,
// csrc/update.hip gfk_win_fold_k): the kernels that finish the shared tensors take one tile
// for ALL M clients of the launch, in client order, and write the client-order sum of the
// pre-scaled results once -- no per-client post-Adam copies, no fold kernel after the round.
// left: [n_left][2] (first float, floats) pieces of the shared prefix that no update job owns
// (batch-norm running statistics): summed in client order by extra workgroups.
// mode: 0 writes the sum into every client's buffer (one rank: the round's FedAvg is done),
// 1 into client 0's only (the rank's partial sum, all-reduced over the ranks and broadcast).
// One client's pointers for the fold kernels, packed by the host (ops/engine.py
// BatchedSteps.set_fold): a client's turn reads them with a few batched scalar loads from
// one base (the GfkModel / GfkUpdate fields, read one by one between dependent address
// computations, cost ~1.5 us of scalar-load round trips per client turn).  *_m / *_v: the
// Adam moments of the tensor (parameter pointer + off_m / off_v); *_sc: the FedAvg
// pre-scale of the tensor (fed_scale, or 1 where it is not shared -- x * 1 = x exactly).
#define GFK_FOLD_W 8
#define GFK_FOLD_V 16
typedef struct GfkFoldClient {
  const int32_t *tstart, *indices;
  const float* values;
  const int32_t* nb;
  const float *coef, *zn, *thetad, *lse, *s, *rstd;
  float *beta, *beta_m, *beta_v, *dthetad;
  const float* dz0;
  float *w_in, *w_in_m, *w_in_v, *flat;
  float beta_sc, win_sc, b1, b2, eps, wd;
  const float *wdz[GFK_FOLD_W], *wa[GFK_FOLD_W];
  float *wp[GFK_FOLD_W], *wm[GFK_FOLD_W], *wv[GFK_FOLD_W];
  const float* vsrc[GFK_FOLD_V];
  float *vp[GFK_FOLD_V], *vm[GFK_FOLD_V], *vv[GFK_FOLD_V], *vg[GFK_FOLD_V];
  float wsc[GFK_FOLD_W], vsc[GFK_FOLD_V];
} GfkFoldClient;

typedef struct GfkFold {
  const GfkModel* models;        // device array [M] (the batched launch's descriptors)
  const GfkUpdate* upds;         // device array [M]
  const int64_t* left;
  int32_t M, mode, n_left, nj;   // nj: W_in hidden slices of 16 columns (ceil(H0 / 16))
  const GfkFoldClient* cl;       // device array [M]
} GfkFold;

}  // extern "C"

// launch helpers: grid z = the batched models, the kernel argument = the device array
__host__ inline dim3 gfk_grid(dim3 g, const GfkModel* m) {
  g.z = m->n_batch > 1 ? (unsigned)m->n_batch : 1u;
  return g;
}
__host__ inline const GfkModel* gfk_dev(const GfkModel* m) {
  return reinterpret_cast<const GfkModel*>(m->dev);
}

// Kernel argument of every model kernel, in two instantiations: <false> the descriptor BY
// VALUE (one client: kernarg memory, so the pointers in it are known global and the
// kernels keep global_load / global_store), <true> a pointer to the device array of
// gridDim.z descriptors (batched clients: model blockIdx.z; accesses through its pointers
// become FLAT instructions, the price of one launch for many clients).
template <bool B> struct GfkArgT;
template <> struct GfkArgT<false> { GfkModel m; };
template <> struct GfkArgT<true> { const GfkModel* p; };
// Workgroup -> (client, index) of a launch.  One client (gridDim.z = 1): (0, blockIdx.x).
// Batched (gridDim.z = M clients of gridDim.x workgroups each): the dispatcher deals
// workgroups round-robin over the 8 XCDs in linear order L = x + gx z (observed placement,
// MI355X_MICROARCH.md "Workgroup dispatch"; speed only, never correctness), so the
// bijection L -> (client L % M, index L / M) puts ALL of a client's workgroups on the XCD(s)
// L % 8 = client (mod 8) -- at M = 8 one client per XCD: each kernel of the round finds the
// client's previous outputs (heads, theta_d, logit tiles, ...) and parameters in its own
// XCD's L2 instead of another die's.  Indices b and b + 8 of a client still share an XCD
// (their L differ by 8 M), which the pipelined backward's tile grouping relies on.
// (power-of-two client counts only -- shifts and masks on scalar registers; a division here
// would run on the VALU and cost the 64-VGPR kernels spills -- other counts keep the plain
// placement)
__device__ __forceinline__ int gfk_bz() {
  const unsigned M = gridDim.z;
  if (M & (M - 1)) return (int)blockIdx.z;
  return (int)((blockIdx.x + gridDim.x * blockIdx.z) & (M - 1));
}
__device__ __forceinline__ int gfk_bx() {
  const unsigned M = gridDim.z;
  if (M & (M - 1)) return (int)blockIdx.x;
  return (int)((blockIdx.x + gridDim.x * blockIdx.z) >> __builtin_ctz(M));
}
__device__ __forceinline__ const GfkModel& gfk_model(const GfkArgT<false>& a) { return a.m; }
// (the batched models through the constant address space: the field loads stay scalar
// (s_load) after the kernel's own stores, as the by-value kernarg model's do)
#ifndef GFK_BATCHED_COPY
#define GFK_BATCHED_COPY 0
#endif
// Batched kernels: the workgroup's descriptor is COPIED at entry (GFK_BATCHED_COPY, set by
// the sources whose kernels index it with constant offsets only): the copy's field loads
// are issued before any store, so they stay scalar and the pointers in it are known global
// (global_load / global_store with an SGPR base, as the by-value descriptor's) -- through
// the reference every field read after a store is re-loaded, and its pointers are FLAT
// (64-bit VGPR addresses): the batched ProdLDA backward needed 80 VGPRs, 64 with the copy.
// A runtime index into one of its arrays keeps the copy in scratch: those sources keep the
// reference.
// (a kernel whose copy would not fit the scalar registers -- SGPR spills land in VGPR lanes --
// takes gfk_model_ref)
__device__ __forceinline__ const GfkModel& gfk_model_ref(const GfkArgT<false>& a) { return a.m; }
__device__ __forceinline__ const GfkModel& gfk_model_ref(const GfkArgT<true>& a) { return a.p[gfk_bz()]; }
#if GFK_BATCHED_COPY
__device__ __forceinline__ GfkModel gfk_model(const GfkArgT<true>& a) { return a.p[gfk_bz()]; }
#else
__device__ __forceinline__ const GfkModel& gfk_model(const GfkArgT<true>& a) { return a.p[gfk_bz()]; }
#endif
template <bool B> struct GfkUArgT;
template <> struct GfkUArgT<false> { GfkUpdate u; };
template <> struct GfkUArgT<true> { const GfkUpdate* p; };
__device__ __forceinline__ const GfkUpdate& gfk_upd(const GfkUArgT<false>& a) { return a.u; }
__device__ __forceinline__ const GfkUpdate& gfk_upd(const GfkUArgT<true>& a) { return a.p[gfk_bz()]; }

// ---------------------------------------------------------------------------
// Device helpers
// ---------------------------------------------------------------------------
namespace gfk {

// In-kernel phase timestamps for diagnostic builds (-DGFK_STAMPS): lane 0 of
// workgroup 0 writes s_memtime into dbg[slot].  Compiled out otherwise.
#ifdef GFK_STAMPS
#define GFK_STAMP(m, slot)                                                        \
  do {                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                            \
    if (gfk_bx() == 0 && threadIdx.x == 0 && (m).dbg)                           \
      (m).dbg[slot] = __builtin_amdgcn_s_memtime();                               \
    __builtin_amdgcn_sched_barrier(0);                                            \
  } while (0)
#else
#define GFK_STAMP(m, slot) do { } while (0)
#endif

// Philox4x32-10 counter-based RNG: stateless, so every kernel (and every graph
// replay) derives its random numbers from (seed, step, stream, element).
__device__ __forceinline__ uint4 philox(uint32_t k0, uint32_t k1, uint4 c) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1,
                   (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Stream tags keep the draws of different random tensors independent.
enum : uint32_t { RNG_EPS = 1, RNG_DROP_ENC = 2, RNG_DROP_THETA = 3, RNG_INFER = 4,
                  RNG_RRELU = 5 };   // RNG_RRELU | (layer << 8): one stream per hidden layer

__device__ __forceinline__ uint4 rng4(uint64_t seed, uint32_t step, uint32_t tag, uint32_t idx) {
  return philox((uint32_t)seed, (uint32_t)(seed >> 32), make_uint4(idx, step, tag, 0x5eedu));
}

__device__ __forceinline__ float u01(uint32_t x) {        // [0, 1)
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float randn(uint64_t seed, uint32_t step, uint32_t tag, uint32_t idx) {
  const uint4 r = rng4(seed, step, tag, idx);
  const float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);   // (0, 1]
  const float u2 = u01(r.y);
  return sqrtf(-2.0f * logf(u1)) * cospif(2.0f * u2);
}

// Inverted-dropout scale: 0 with probability p, 1/(1-p) otherwise (torch semantics).
__device__ __forceinline__ float drop_scale(uint64_t seed, uint32_t step, uint32_t tag,
                                            uint32_t idx, float p) {
  if (p <= 0.f) return 1.f;
  if (p >= 1.f) return 0.f;
  return u01(rng4(seed, step, tag, idx).x) >= p ? 1.f / (1.f - p) : 0.f;
}

// torch.nn.RReLU defaults (lower 1/8, upper 1/3): training draws the negative-side
// slope per element from U(lower, upper); eval uses their mean.
constexpr float RRELU_LO = 1.f / 8.f, RRELU_HI = 1.f / 3.f;

// Activation in eval mode (inference) -- and every activation but RReLU in training.
__device__ __forceinline__ float act_f(int a, float z) {
  switch (a) {
    case GFK_RRELU: return z >= 0.f ? z : z * (0.5f * (RRELU_LO + RRELU_HI));
    case GFK_SOFTPLUS: return z > 20.f ? z : log1pf(expf(z));
    case GFK_RELU: return z > 0.f ? z : 0.f;
    case GFK_SIGMOID: return 1.f / (1.f + expf(-z));
    case GFK_TANH: return tanhf(z);
    case GFK_LEAKYRELU: return z > 0.f ? z : 0.01f * z;
    case GFK_ELU: return z > 0.f ? z : expm1f(z);
    default: {  // SELU
      const float s = 1.0507009873554804934f, al = 1.6732632423543772848f;
      return z > 0.f ? s * z : s * al * expm1f(z);
    }
  }
}

// Training-mode activation of element idx of hidden layer `layer` (stored as the
// pre-activation z in ws_z for act_d) -- except RReLU, whose slope is a Philox draw:
// its ws_z entry holds d act / d z (1, or the drawn slope) instead, so the backward
// needs neither the step nor the draw (*zs receives what is stored).
__device__ __forceinline__ float act_train(int a, float z, uint64_t seed, uint32_t step, int layer,
                                           uint32_t idx, float* zs) {
  if (a != GFK_RRELU) {
    *zs = z;
    return act_f(a, z);
  }
  const float r = RRELU_LO + (RRELU_HI - RRELU_LO) *
                  u01(rng4(seed, step, RNG_RRELU | ((uint32_t)layer << 8), idx).x);
  *zs = z > 0.f ? 1.f : r;          // torch: the drawn slope applies to z <= 0
  return z > 0.f ? z : z * r;
}

// d act / d z from the ws_z entry written by act_train (the pre-activation z; RReLU:
// the derivative itself).
__device__ __forceinline__ float act_d(int a, float z) {
  switch (a) {
    case GFK_RRELU: return z;
    case GFK_SOFTPLUS: return z > 20.f ? 1.f : 1.f / (1.f + expf(-z));
    case GFK_RELU: return z > 0.f ? 1.f : 0.f;
    case GFK_SIGMOID: { const float s = 1.f / (1.f + expf(-z)); return s * (1.f - s); }
    case GFK_TANH: { const float t = tanhf(z); return 1.f - t * t; }
    case GFK_LEAKYRELU: return z > 0.f ? 1.f : 0.01f;
    case GFK_ELU: return z > 0.f ? 1.f : expf(z);
    default: {
      const float s = 1.0507009873554804934f, al = 1.6732632423543772848f;
      return z > 0.f ? s : s * al * expf(z);
    }
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Combine two online-softmax partials (m, s): s = sum exp(x - m).
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;
  if (m == -INFINITY) { m = m2; s = s2; return; }
  const float mn = fmaxf(m, m2);
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

__device__ __forceinline__ void wave_lse(float& m, float& s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
}

__device__ __forceinline__ int uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }

// Workgroup barrier for LDS-only data exchange.  __syncthreads() is a
// workgroup-scope fence + s_barrier, and on gfx9 the fence waits for EVERY
// outstanding vector-memory operation (vmcnt(0)) -- including global stores,
// whose acknowledgements take a full round trip.  Phases that only hand data
// over through LDS use this instead: LDS ops drained, global stores left in
// flight.  (LDS-DMA staging still needs __syncthreads() / vm_barrier().)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Pin a kernel-argument field in SGPRs at the point of the call: the empty asm
// "modifies" the value, so the compiler can neither sink the scalar load to its
// first use nor re-load it later.  Used in kernel prologues so that all
// argument loads are issued back to back and waited on once, instead of one
// dependent scalar-cache round trip per field in the middle of the kernel.
template <class T>
__device__ __forceinline__ void keep1(T& v) { asm volatile("" : "+s"(v)); }

// torch.optim.Adam element update with the bias corrections precomputed on the
// device (coef = {lr / (1 - b1^t), 1 / sqrt(1 - b2^t)}, from double-precision
// running powers):  m += (1-b1)(g-m);  v = b2 v + (1-b2) g^2;
//                   p -= step * m / (sqrt(v) / sqrt(bc2) + eps)
struct AdamCoef {
  float b1, b2, eps, wd, step, ibc2;
};

__device__ __forceinline__ AdamCoef adam_coef(const GfkModel& m) {
  AdamCoef c;
  c.b1 = m.beta1; c.b2 = m.beta2; c.eps = m.adam_eps; c.wd = m.weight_decay;
  c.step = m.adam_coef[0];
  c.ibc2 = m.adam_coef[1];
  return c;
}

// One optimizer step's advance of the running powers and the bias-correction coefficients
// (post_fwd, the strip forward's folded posterior and the large-batch plan, which must
// produce the same bits: contraction off, every operation explicit).
__device__ __forceinline__ void adam_advance(const GfkModel& m, double pw0, double pw1, double& p1,
                                             double& p2, float& c0, float& c1) {
#pragma clang fp contract(off)
  p1 = pw0 * (double)m.beta1;
  p2 = pw1 * (double)m.beta2;
  c0 = (float)((double)m.lr / (1.0 - p1));
  c1 = (float)(1.0 / sqrt(1.0 - p2));
}

// The square root and the division use the hardware's v_sqrt_f32 / v_rcp_f32 (1 ulp)
// instead of the correctly rounded library sequences (~16 and ~10 VALU instructions
// with their denormal scaling): the optimizer epilogues of the large-vocabulary
// kernels are VALU-heavy, and the step's relative error stays ~1e-7 of an lr-sized term.
// Every fused multiply-add is explicit and contraction is off, so the update rounds the
// same way in every kernel it is inlined into (the in-epilogue FedAvg kernels must agree
// bit for bit with the per-client updates; the compiler's own contraction choices differ
// between kernels).
__device__ __forceinline__ float adam_update(float p, float g, float& mo, float& vo, const AdamCoef& c) {
#pragma clang fp contract(off)
  if (c.wd != 0.f) g = __builtin_fmaf(c.wd, p, g);
  mo = __builtin_fmaf(1.f - c.b1, g - mo, mo);
  vo = __builtin_fmaf(c.b2, vo, (1.f - c.b2) * g * g);
  const float den = __builtin_fmaf(__builtin_amdgcn_sqrtf(vo), c.ibc2, c.eps);
  return __builtin_fmaf(-(c.step * mo), __builtin_amdgcn_rcpf(den), p);
}

// The in-epilogue FedAvg's client-order sum (csrc/prodlda.hip gfk_bwd_fold_k, csrc/update.hip
// gfk_win_fold_k): the client's pre-scaled value w_c p_c rounded on its own, then added --
// contraction off, or acc + p * w would become one fma (one rounding) and differ from the
// per-client epilogue + gfk_local_fedavg in the last bit wherever w_c is not a power of two.
__device__ __forceinline__ float fold_add(float acc, float p, float w, bool first) {
#pragma clang fp contract(off)
  const float x = p * w;
  return first ? x : acc + x;
}

// Final value of a parameter element: fused mode applies Adam (and the FedAvg
// pre-scale for shared tensors) in place; gradient mode stores g into the grad
// slot for the generic Adam kernel.  ptr points into the parameter flat buffer.
__device__ __forceinline__ void param_update(const GfkModel& m, float* ptr, float g, const AdamCoef& c,
                                             bool shared) {
  if (m.update_mode == 0) {
    ptr[m.off_g] = g;
    return;
  }
  float mo = ptr[m.off_m], vo = ptr[m.off_v];
  float p = adam_update(*ptr, g, mo, vo, c);
  if (shared && m.fed_scale_on) p *= m.fed_scale;
  ptr[m.off_m] = mo;
  ptr[m.off_v] = vo;
  *ptr = p;
}

__device__ __forceinline__ bool is_shared(const GfkModel& m, const float* ptr) {
  return (ptr - m.flat_base) < m.n_shared;
}
template <class... T>
__device__ __forceinline__ void keep(T&... v) { (keep1(v), ...); }

// DPP lane permutations inside each 16-lane row (VALU-rate, no LDS round trip):
// quad_perm xor1 / xor2, row_half_mirror, row_mirror.  Applying all four with a
// commutative op reduces over the 16 lanes and leaves the result in every lane.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}

// global -> LDS copy of n floats with U independent loads in flight per thread
// (indices are clamped, never predicated, so hipcc keeps the loads back to back).
template <int U>
__device__ __forceinline__ void stage_lin(float* __restrict__ dst, const float* __restrict__ src,
                                          int n, int tid, int nt) {
  if (n <= 0) return;
  for (int base = tid; base < n; base += U * nt) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[min(base + u * nt, n - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * nt < n) dst[base + u * nt] = v[u];
  }
}

// Asynchronous global -> LDS copy (LDS-DMA, global_load_lds_dwordx4): every lane
// moves one 16-byte chunk straight into LDS, no VGPR round trip, so a whole
// staging phase is issued back to back and drained by ONE barrier.  Copies
// ceil(n/4) chunks: src and dst must be 16-byte aligned and the source must be
// readable up to the next multiple of 4 floats.  The LDS destination of a wave
// instruction is its wave-uniform base + lane*16, so each wave copies 64
// consecutive chunks.
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef const __attribute__((address_space(1))) void* gbl_void_ptr;

__device__ __forceinline__ void glds_copy(float* dst, const float* src, int n, int tid, int nt) {
  const int nchunk = (n + 3) >> 2;
  const int lane = tid & 63, w = tid >> 6, nw = nt >> 6;
  for (int c0 = w * 64; c0 < nchunk; c0 += nw * 64)
    if (c0 + lane < nchunk)
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + 4 * (c0 + lane)),
                                       (lds_void_ptr)(dst + 4 * c0), 16, 0, 0);
}

// glds_copy of a COMPILE-TIME size: straight-line instructions (no loop), so the
// compiler's vmcnt bookkeeping stays exact across it (after a copy loop of unknown trip
// count it can only wait for vmcnt(0)).  N floats, a multiple of 4; NT threads.
template <int N, int NT>
__device__ __forceinline__ void glds_copy_n(float* dst, const float* src, int tid) {
  static_assert(N % 4 == 0 && NT % 64 == 0, "whole chunks, whole waves");
  constexpr int NCH = N / 4, PASS = NT, FULL = NCH / PASS, REM = NCH % PASS;
  const int lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int p = 0; p < FULL; ++p)
    __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + 4 * (p * PASS + w * 64 + lane)),
                                     (lds_void_ptr)(dst + 4 * (p * PASS + w * 64)), 16, 0, 0);
  if constexpr (REM > 0) {
    if (w * 64 + lane < REM)
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + 4 * (FULL * PASS + w * 64 + lane)),
                                       (lds_void_ptr)(dst + 4 * (FULL * PASS + w * 64)), 16, 0, 0);
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x4 fp32 MFMA: lane l supplies A[l&15][l>>4] and B[l>>4][l&15];
// the result holds C[(l>>4)*4 + r][l&15] in element r.
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 MFMA, fp32 accumulation.  gfx950's 16x16x32 (v_mfma_f32_16x16x32_bf16, twice the
// K of the CDNA3-era 16x16x16 per instruction): lane l supplies A[l&15][8(l>>4) + j] and
// B[8(l>>4) + j][l&15] (j < 8) as fp32, rounded to bf16 here (v_cvt_pk_bf16_f32, RNE);
// the 16x16x16 form (j < 4, 4(l>>4) + j) serves a K tail of 16.  The result layout is
// the one of mfma16x16x4.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16x16x32bf(const float (&a)[8], const float (&b)[8], f32x4 c) {
  bf16x8 ab, bb;
#pragma unroll
  for (int j = 0; j < 8; ++j) { ab[j] = (__bf16)a[j]; bb[j] = (__bf16)b[j]; }
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ab, bb, c, 0, 0, 0);
}
// fp32 -> bf16 (round to nearest even) -> fp32: a bf16 operand of an fp32 product (the
// products of bf16 values are exact in fp32, so a bf16 dot / GEMM with fp32 accumulation is
// this rounding followed by fp32 multiply-adds)
__device__ __forceinline__ float bf16_round(float x) { return (float)(__bf16)x; }

// The same with operands converted once by the caller (an operand reused by several MFMAs).
__device__ __forceinline__ bf16x8 to_bf16x8(const f32x4& lo, const f32x4& hi) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) { r[j] = (__bf16)lo[j]; r[4 + j] = (__bf16)hi[j]; }
  return r;
}
__device__ __forceinline__ f32x4 mfma_bf16x8(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16x16x16bf(const float (&a)[4], const float (&b)[4], f32x4 c) {
  bf16x4 ab, bb;
#pragma unroll
  for (int j = 0; j < 4; ++j) { ab[j] = (__bf16)a[j]; bb[j] = (__bf16)b[j]; }
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, ab),
                                                   __builtin_bit_cast(s16x4, bb), c, 0, 0, 0);
}

// A strided, bounds-checked matrix view (LDS or global).  Out-of-range elements
// read as 0 through a clamped address + select, so no load is predicated.
struct MatView {
  const float* p;
  int si, sj, rows, cols;
  __device__ __forceinline__ float at(int i, int j) const {
    const float v = p[(size_t)min(i, rows - 1) * si + (size_t)min(j, cols - 1) * sj];
    return (i < rows && j < cols) ? v : 0.f;
  }
};

// C[M x N] = A[M x R] @ B[R x N] on the fp32 matrix cores; 16x16 output tiles are
// dealt round-robin to the workgroup's waves; store(i, j, value) is called for
// every element with i < M, j < N.
template <class Store>
__device__ __forceinline__ void mfma_gemm(int M, int N, int R, const MatView& A, const MatView& B,
                                          int wave, int nwaves, Store store) {
  const int lane = threadIdx.x & 63;
  const int mt = (M + 15) >> 4, nt = (N + 15) >> 4;
  for (int s = wave; s < mt * nt; s += nwaves) {
    const int i0 = (s / nt) * 16, j0 = (s % nt) * 16;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int ai = i0 + (lane & 15), bj = j0 + (lane & 15), kk = lane >> 4;
    for (int k0 = 0; k0 < R; k0 += 4) acc = mfma16x16x4(A.at(ai, k0 + kk), B.at(k0 + kk, bj), acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = i0 + (lane >> 4) * 4 + r;
      if (i < M && bj < N) store(i, bj, acc[r]);
    }
  }
}

// Prepares the NEXT minibatch (the step counter has already been advanced):
// nb, the doc ids, and each row's CSR extent into ws_next -- a chain of four
// dependent reads (step -> plan -> doc -> indptr) that runs in an extra
// workgroup of win_update, off the critical path, so the next enc_in starts one
// round trip from its data.  Rows past the batch repeat its first doc.
// pnb_e: 2 * bmax ints of LDS, the (e0, e1) of the next batch's rows -- the
// caller's dynamic LDS where it has some, so the win_update kernels carry no static LDS on
// top of their dynamic budget (40 KB + 1 KB would cost the sparse tile its 4th workgroup
// per CU)
__device__ __forceinline__ void prepare_next_batch(const GfkModel& m, int* pnb_e) {
  const int step = *m.step;
  int32_t* nxt = m.ws_next;
  if (step >= m.n_steps) {
    if (threadIdx.x == 0) nxt[0] = 0;
    return;
  }
  const int nb = m.plan_size[step];
  const int base = m.plan_start[step];
  const int bmax = m.bmax;
  for (int b = threadIdx.x; b < bmax; b += blockDim.x) {
    const int doc = m.plan_order[base + (b < nb ? b : 0)];
    const int e0 = m.indptr[doc], e1 = m.indptr[doc + 1];
    nxt[1 + b] = doc;
    nxt[1 + bmax + 2 * b] = e0;
    nxt[2 + bmax + 2 * b] = e1;
    pnb_e[2 * b] = e0;
    pnb_e[2 * b + 1] = e1;
  }
  if (threadIdx.x == 0) nxt[0] = nb;
  const int cap = m.slot_cap;
  if (cap <= 0) return;
  __syncthreads();
  // the rows' non-zeros into their slots: G threads per row, U loads in flight each
  constexpr int U = 8;
  const int G = max(1, (int)blockDim.x / bmax);
  for (int b = threadIdx.x / G; b < bmax; b += blockDim.x / G) {
    const int e0 = pnb_e[2 * b], n = pnb_e[2 * b + 1] - e0;
    int32_t* si = m.ws_sidx + (size_t)b * cap;
    float* sv = m.ws_sval + (size_t)b * cap;
    for (int j0 = (int)threadIdx.x % G; j0 < n; j0 += G * U) {
      int ci[U];
      float xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = min(j0 + G * u, n - 1);
        ci[u] = m.indices[e0 + j];
        xv[u] = m.values[e0 + j];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = j0 + G * u;
        if (j < n) {
          si[j] = ci[u];
          sv[j] = xv[u];
        }
      }
    }
  }
}

__device__ __forceinline__ void prepare_next_batch(const GfkModel& m) {
  __shared__ int pnb_e[2 * GFK_BMAX_LIMIT];
  prepare_next_batch(m, pnb_e);
}


// One workgroup's share of the multi-segment Adam: workgroups are dealt to
// segments in proportion to their size (GFK_ADAM_CHUNK float4 per workgroup, segment s
// starts at workgroup seg_first_block[s]).  A ballot over the segment table
// finds the segment in one round trip.  Used by the generic Adam kernel and by
// the extra workgroups of win_update (small tensors in fused mode).
__device__ __forceinline__ void adam_block(const GfkAdam& a, int blk, int tid, int nthreads) {
  AdamCoef c;                 // bias corrections advanced on the device (enc_head_fwd)
  c.b1 = a.beta1; c.b2 = a.beta2; c.eps = a.eps; c.wd = a.weight_decay;
  c.step = a.coef[0];
  c.ibc2 = a.coef[1];
  const int lane = tid & 63;
  const int nseg = a.n_seg;
  const int fb = lane < nseg ? a.seg_first_block[lane] : 0x7fffffff;
  const uint64_t le = __ballot(fb <= blk);
  const int s = __popcll(le) - 1;
  if (s < 0 || s >= nseg) return;
  const int first = a.seg_first_block[s];
  const int64_t s0 = a.seg_start[s], n4 = (a.seg_end[s] - s0) >> 2;
  const int flags = a.seg_flags[s];
  const bool do_adam = flags & 1, do_scale = flags & 2;
  const int64_t lo = (int64_t)(blk - first) * GFK_ADAM_CHUNK,
                hi = lo + GFK_ADAM_CHUNK < n4 ? lo + GFK_ADAM_CHUNK : n4;
  for (int64_t i = lo + tid; i < hi; i += nthreads) {
    const int64_t o = s0 + 4 * i;
    float4 p = *reinterpret_cast<float4*>(a.p + o);
    if (do_adam) {
      const float4 g = *reinterpret_cast<float4*>(a.g + o);
      float4 m = *reinterpret_cast<float4*>(a.m + o);
      float4 v = *reinterpret_cast<float4*>(a.v + o);
      float* pp = &p.x; const float* gg = &g.x; float* mm = &m.x; float* vv = &v.x;
      switch (a.solver) {
        case GFK_SOLVER_ADAM:
#pragma unroll
          for (int j = 0; j < 4; ++j) pp[j] = adam_update(pp[j], gg[j], mm[j], vv[j], c);
          break;
        case GFK_SOLVER_SGD:
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float g1 = c.wd != 0.f ? gg[j] + c.wd * pp[j] : gg[j];
            mm[j] = c.b1 * mm[j] + g1;
            pp[j] -= a.lr * (c.b1 != 0.f ? mm[j] : g1);
          }
          break;
        case GFK_SOLVER_ADAGRAD:
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float g1 = c.wd != 0.f ? gg[j] + c.wd * pp[j] : gg[j];
            vv[j] += g1 * g1;
            pp[j] -= a.lr * g1 / (sqrtf(vv[j]) + c.eps);
          }
          break;
        case GFK_SOLVER_ADADELTA:
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float g1 = c.wd != 0.f ? gg[j] + c.wd * pp[j] : gg[j];
            vv[j] = c.b2 * vv[j] + (1.f - c.b2) * g1 * g1;
            const float d = sqrtf(mm[j] + c.eps) / sqrtf(vv[j] + c.eps) * g1;
            mm[j] = c.b2 * mm[j] + (1.f - c.b2) * d * d;
            pp[j] -= a.lr * d;
          }
          break;
        default:   // GFK_SOLVER_RMSPROP
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float g1 = c.wd != 0.f ? gg[j] + c.wd * pp[j] : gg[j];
            vv[j] = c.b2 * vv[j] + (1.f - c.b2) * g1 * g1;
            const float q = g1 / (sqrtf(vv[j]) + c.eps);
            mm[j] = c.b1 * mm[j] + q;
            pp[j] -= a.lr * (c.b1 != 0.f ? mm[j] : q);
          }
          break;
      }
      *reinterpret_cast<float4*>(a.m + o) = m;
      *reinterpret_cast<float4*>(a.v + o) = v;
      if (!(flags & 4)) *reinterpret_cast<float4*>(a.g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (do_scale) { p.x *= a.scale; p.y *= a.scale; p.z *= a.scale; p.w *= a.scale; }
    if (do_adam || do_scale) *reinterpret_cast<float4*>(a.p + o) = p;
  }
}

// Sum of one value per thread over the workgroup, computed by wave 0 from the
// per-wave sums in `scratch` (one float per wave).  Result valid in wave 0.
__device__ __forceinline__ float block_sum_wave0(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  if (lane == 0) scratch[wave] = v;
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  float t = lane < nw ? scratch[lane] : 0.f;
  return wave_sum(t);
}

}  // namespace gfk
