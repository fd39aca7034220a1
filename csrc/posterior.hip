// Batch-coupled part of the encoder: batch-norm of the mu / log-sigma^2 heads,
// reparameterised sample, softmax(theta), theta dropout, KL -- forward
// (post_fwd) and backward (row_bwd + post_bwd) -- and the next-batch kernels.
//
// Reference math: inference_network.py:76-85 (mu / log-sigma heads with
// affine-free BatchNorm1d), decoder_network.py:102-118 (reparameterise, softmax,
// theta dropout), avitm.py:207-229 (KL), torch.nn.BatchNorm1d training semantics
// (biased variance normalises, unbiased variance feeds running_var, momentum).
//
// Decomposition (MI355X-first).  One workgroup of 4 waves per batch row, so the
// VALU-heavy per-element work (exp, softmax, BN) of B rows runs on B CUs.  The
// rows couple only through per-column statistics of [B, 2K] matrices (a few
// tens of KB, L2-resident): every workgroup pulls the whole matrix into LDS
// with LDS-DMA and recomputes the statistics it needs -- redundant but a single
// round trip and no cross-workgroup synchronisation.  Weight gradients (sums over
// rows) are left to the update kernel's GEMM tiles, so nothing here needs atomics
// or partial slabs; every result is deterministic.
//
//   post_fwd  : column statistics of the raw heads, own row: normalise,
//               reparameterise, softmax, dropout, KL.  Workgroup 0 updates the
//               running statistics and advances the optimizer step.
//   row_bwd   : own row: fixed-order sum of the decoder's per-tile d theta_d
//               partials, softmax / reparameterisation / KL backward -> dmu, dls.
//   post_bwd  : column sums of dmu, dls (all rows), own row: BN backward ->
//               d mu_raw, d ls_raw, heads and hidden-layer backward -> dz of every
//               layer.  Workgroup 0: prior gradients, the loss, the step counter.
#define GFK_BATCHED_COPY 1   // batched kernels copy their descriptor (gfk_common.h gfk_model)
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int PT = 256;                 // threads per workgroup (row_bwd)
constexpr int FT = 1024;                // threads per workgroup (post_fwd, post_bwd): 16 lanes
                                        // per batch column in the column reductions
__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

// Sum over the 4 lanes of a DPP quad (xor 1, xor 2); result in every lane.
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_f<0xB1>(v);
  return v + dpp_f<0x4E>(v);
}

__host__ __device__ inline int post_hmax(const GfkModel& m) {
  int h = 0;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) h = h > m.H[l] ? h : m.H[l];
  return h;
}

// Floats of the staged backward weights: W_mu, W_s ([K][Hl]), then W_h[l] for
// l = 0 .. nh-2 ([H[l+1]][H[l]]), each padded to 4.
__host__ __device__ inline int post_weight_floats(const GfkModel& m) {
  int n = 2 * pad4(m.K * gfk_hlast(m));
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < m.n_hidden) n += pad4(m.H[l + 1] * m.H[l]);
  return n;
}
}  // namespace

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// stage_flags bit 1 (GFK_STAGE_BATCH_L2): the [B][K] batch matrices are read from
// global memory (L2-resident) instead of being staged in LDS -- large K, where
// four of them would not fit the 160 KiB.
__host__ __device__ inline bool batch_in_lds(const GfkModel& m) { return !(m.stage_flags & 2); }

// Row stride of the LDS-staged [B][K] batch matrices: K (contiguous rows, one LDS-DMA copy).
// A padded 2 x odd stride removed the K = 100 column reductions' bank conflicts (31 % -> 0 %)
// but its per-row dword staging cost more than they did (CombinedTM K = 100 V = 99k: 0.7296 /
// 0.7355 ms contiguous vs 0.7369 / 0.7432 padded, profiles/r5/ab_post_stride.txt; removed in
// round 6).
__host__ __device__ inline int post_lds_ld(int K) { return K; }

// Rows of a row-major [rows][cols] global matrix into LDS rows of stride ld (LDS-DMA, one
// dword per lane: 64 columns of a row per wave instruction; ld == cols: one contiguous copy)
__device__ __forceinline__ void glds_rows(float* dst, const float* src, int rows, int cols, int ld,
                                          int tid, int nt) {
  if (ld == cols) {
    glds_copy(dst, src, rows * cols, tid, nt);
    return;
  }
  const int lane = tid & 63, w = tid >> 6, nw = nt >> 6;
  for (int r = w; r < rows; r += nw)
    for (int c0 = 0; c0 < cols; c0 += 64)
      if (c0 + lane < cols)
        __builtin_amdgcn_global_load_lds((gbl_void_ptr)(src + (size_t)r * cols + c0 + lane),
                                         (lds_void_ptr)(dst + r * ld + c0), 4, 0, 0);
}

extern "C" size_t gfk_post_fwd_smem(const GfkModel* m) {
  const size_t mats = batch_in_lds(*m) ? 2 * (size_t)m->bmax * post_lds_ld(m->K) : 0;
  return sizeof(float) * (mats + 4 * (size_t)pad4(m->K) + 2 * FT);
}

// Column reductions over the batch of [B][K] matrices, lane-per-column: thread t owns
// column c2 = t % 512 of the 2K (mu | log sigma^2) columns and the rows b = t / 512 + 2 i
// (two row groups), so a wave's loads are 64 consecutive floats of a row (coalesced
// from L2, bank-conflict free from LDS) -- the 16-lanes-per-column layout this replaced
// touched 64 cache lines per load instruction.  RPG = rows per group (bmax / 2); the
// two groups' partials meet in `red` [2][512] (LDS).
constexpr int CG = 512;                 // columns per workgroup pass (2K <= 512)
constexpr int NGR = FT / CG;            // row groups

// Column statistics of the raw heads (mean, biased variance -> rstd); workgroup 0
// also advances the running statistics (rm0 / rv0: this thread's column, prefetched).
template <int RPG>
__device__ __forceinline__ void post_colstats(const GfkModel& m, const float* mr, const float* lr,
                                              float* cmean, float* crstd, float* red, float rm0,
                                              float rv0, int nb, float inv_nb, int row, int tid) {
  constexpr int RB = 16;                  // rows per load batch (registers)
  const int K = m.K, c2 = tid % CG, grp = tid / CG;
  const int cc = min(c2, 2 * K - 1);
  const float* x = cc < K ? mr + cc : lr + (cc - K);
  float s = 0.f;
#pragma unroll 1
  for (int i0 = 0; i0 < RPG; i0 += RB) {
    float xv[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) xv[i] = x[min(grp + NGR * (i0 + i), nb - 1) * K];
#pragma unroll
    for (int i = 0; i < RB; ++i) s += grp + NGR * (i0 + i) < nb ? xv[i] : 0.f;
  }
  red[tid] = s;
  lds_barrier();
  const float mean = (red[c2] + red[CG + c2]) * inv_nb;
  float q = 0.f;                          // two-pass variance (re-read, as torch's BN)
#pragma unroll 1
  for (int i0 = 0; i0 < RPG; i0 += RB) {
    float xv[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) xv[i] = x[min(grp + NGR * (i0 + i), nb - 1) * K];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const float d = grp + NGR * (i0 + i) < nb ? xv[i] - mean : 0.f;
      q += d * d;
    }
  }
  red[FT + tid] = q;
  lds_barrier();
  if (grp == 0 && c2 < 2 * K) {
    const float var = (red[FT + c2] + red[FT + CG + c2]) * inv_nb;
    const float rstd = rsqrtf(var + m.bn_eps);
    cmean[c2] = mean;
    crstd[c2] = rstd;
    if (row == 0) {
      const int k = c2 < K ? c2 : c2 - K;
      float* rm = c2 < K ? m.mu_rm + k : m.s_rm + k;
      float* rv = c2 < K ? m.mu_rv + k : m.s_rv + k;
      const float mom = m.bn_momentum;
      const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
      float nm = (1.f - mom) * rm0 + mom * mean, nv = (1.f - mom) * rv0 + mom * unb;
      if (m.fed_scale_on && is_shared(m, rm)) { nm *= m.fed_scale; nv *= m.fed_scale; }
      *rm = nm;
      *rv = nv;
      m.ws_bn_rstd[c2] = rstd;
    }
  }
}

// LDS-resident batch matrices (K small enough): 16 lanes -- one DPP row -- per column,
// RPT rows per lane, 64 columns per pass (rmp / rvp: the running statistics of the
// pass's column, prefetched).
template <int RPT>
__device__ __forceinline__ void post_colstats_dpp(const GfkModel& m, const float* mr, const float* lr,
                                              float* cmean, float* crstd, const float (&rmp)[8],
                                              const float (&rvp)[8], int nb, float inv_nb, int row,
                                              int tid, int ld) {
  constexpr int CP = 8;
  const int K = m.K;
#pragma unroll
  for (int pass = 0; pass < CP; ++pass) {
    const int cb = pass * (FT / 16);
    if (cb >= 2 * K) break;
    const int c2 = cb + (tid >> 4), g = tid & 15;
    const bool valid = c2 < 2 * K;
    const float* x = (c2 < K ? mr + c2 : lr + (c2 - K));
    float xv[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int r = g + 16 * i;
      xv[i] = (valid && r < nb) ? x[r * ld] : 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) s += xv[i];
    const float mean = row16_sum(s) * inv_nb;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const float d = g + 16 * i < nb ? xv[i] - mean : 0.f;
      q += d * d;
    }
    const float var = row16_sum(q) * inv_nb;
    const float rstd = rsqrtf(var + m.bn_eps);
    if (valid && g == 0) {
      cmean[c2] = mean;
      crstd[c2] = rstd;
      if (row == 0) {
        const int k = c2 < K ? c2 : c2 - K;
        float* rm = c2 < K ? m.mu_rm + k : m.s_rm + k;
        float* rv = c2 < K ? m.mu_rv + k : m.s_rv + k;
        const float mom = m.bn_momentum;
        const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
        const float o_m = rmp[pass], o_v = rvp[pass];
        float nm = (1.f - mom) * o_m + mom * mean, nv = (1.f - mom) * o_v + mom * unb;
        if (m.fed_scale_on && is_shared(m, rm)) { nm *= m.fed_scale; nv *= m.fed_scale; }
        *rm = nm;
        *rv = nv;
        m.ws_bn_rstd[c2] = rstd;
      }
    }
  }
}

// CTM label head of the own row (reference ctm decoding_network.py:156-159, ctm.py:292-296):
// est = W_cls theta_d + b_cls, CE(est, argmax(labels)) averaged over the batch.  Writes
// the row's CE / nb (joins the loss in post_bwd), d CE / d est (the classifier's
// weight-gradient jobs in win_update) and d CE / d theta_d = W_cls^T d est as one more
// d theta_d slab (index n_dpart), which row_bwd sums with the decoder's.
// buf: LDS, theta_d of the row in [0, K) (written by wave 0 before the call).
__device__ __forceinline__ void post_label_head(const GfkModel& m, float* buf, int row, int nb,
                                                int tid) {
  const int K = m.K, L = m.L, lane = tid & 63, wave = tid >> 6;
  float* est = buf + 256;
  float* dl = buf + 512;
  lds_barrier();
  // est[l] = b_cls[l] + sum_k theta_d[k] W_cls[l][k]: 16 lanes per output
  for (int l0 = 0; l0 < L; l0 += FT / 16) {
    const int l = l0 + (tid >> 4), s = tid & 15;
    float acc = 0.f;
    if (l < L) {
      const float* w = m.w_cls + (size_t)l * K;
      for (int k = s; k < K; k += 16) acc += buf[k] * w[k];
    }
    acc = row16_sum(acc);
    if (s == 0 && l < L) est[l] = acc + m.b_cls[l];
  }
  lds_barrier();
  if (wave == 0) {
    constexpr int LQ = 4;                    // L <= 256
    const float* lab = m.ws_lab + (size_t)row * L;
    float e[LQ], mx = -INFINITY, best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const int l = lane + 64 * q;
      e[q] = l < L ? est[l] : -INFINITY;
      mx = fmaxf(mx, e[q]);
      const float lv = l < L ? lab[l] : -INFINITY;
      if (lv > best) { best = lv; bi = l; }   // first maximum, like torch.argmax
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float b2 = __shfl_xor(best, o, 64);
      const int i2 = __shfl_xor(bi, o, 64);
      if (b2 > best || (b2 == best && i2 < bi)) { best = b2; bi = i2; }
    }
    mx = wave_max(mx);
    float se = 0.f;
#pragma unroll
    for (int q = 0; q < LQ; ++q) se += lane + 64 * q < L ? __expf(e[q] - mx) : 0.f;
    const float lse = mx + logf(wave_sum(se));
    const float inv_nb = 1.f / (float)nb;
#pragma unroll
    for (int q = 0; q < LQ; ++q) {
      const int l = lane + 64 * q;
      if (l < L) {
        const float d = (expf(e[q] - lse) - (l == bi ? 1.f : 0.f)) * inv_nb;
        dl[l] = d;
        m.ws_dlab[(size_t)row * L + l] = d;
      }
    }
    if (lane == 0) m.ws_ce[row] = (lse - est[bi]) * inv_nb;
  }
  lds_barrier();
  // d theta_d[k] = sum_l dl[l] W_cls[l][k] -> slab n_dpart
  float* slab = m.ws_dthetad + ((size_t)m.n_dpart * m.bmax + row) * K;
  for (int k = tid; k < K; k += FT) {
    float acc = 0.f;
    for (int l = 0; l < L; ++l) acc += dl[l] * m.w_cls[(size_t)l * K + k];
    slab[k] = acc;
  }
}

// grid: bmax workgroups (row = gfk_bx()).  dynamic LDS: mr[B*K] + lr[B*K] (unless
// read from L2) + mean[2K] + rstd[2K]
// InLds: the batch matrices are staged in LDS (compile-time, so every access is a
// ds_read; a runtime select of the pointer would turn them into flat loads).
// PS (the large-batch plan): the column statistics come precomputed from ws_colstat
// (gfk_post_colstats_lb_k), which also did row 0's running-statistic / counter duties.
// KQ: topics per lane of the own row (K <= 64 KQ: 4, or 8 for the plan's K <= 512)
template <bool InLds, bool GB = false, bool PS = false, int KQ = 4>
__global__ void __launch_bounds__(FT) gfk_post_fwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int K = m.K, B = m.bmax;
  const float *mu_raw = m.ws_mu_raw, *ls_raw = m.ws_ls_raw;
  const int32_t* nbp = m.ws_nb;
  keep(K, B, mu_raw, ls_raw, nbp);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int row = gfk_bx();
  constexpr bool in_lds = InLds;
  const int LD = in_lds ? post_lds_ld(K) : K;   // row stride of mr / lr
  const float* mr = in_lds ? smem : mu_raw;
  const float* lr = in_lds ? smem + B * LD : ls_raw;
  float* cmean = smem + (in_lds ? 2 * B * LD : 0);
  float* crstd = cmean + 2 * pad4(K);
  float* red = crstd + 2 * pad4(K);        // [2][FT] column-reduction scratch
  GFK_STAMP(m, 0);

  // ---- one round: the raw heads of every row (LDS-DMA) + the own row + stats ----
  if (in_lds) {
    glds_rows(smem, mu_raw, B, K, LD, tid, FT);
    glds_rows(smem + B * LD, ls_raw, B, K, LD, tid, FT);
  }
  const int nb = *nbp;
  float ep[KQ], mt[KQ], pm[KQ], pv[KQ];
  const int rc = min(row, max(nb - 1, 0));
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = min(lane + 64 * q, K - 1);
    ep[q] = m.ws_eps[rc * K + k];
    mt[q] = m.ws_mask_t[rc * K + k];
    pm[q] = m.prior_mean[k];
    pv[q] = m.prior_var[k];
  }
  // workgroup 0, thread 0: the counters it advances, prefetched
  double pw0 = 0.0, pw1 = 0.0;
  int64_t nbt0 = 0, nbt1 = 0;
  int32_t at0 = 0;
  if (row == 0 && tid == 0) {
    pw0 = m.adam_pow[0];
    pw1 = m.adam_pow[1];
    nbt0 = *m.nbt_mu;
    nbt1 = *m.nbt_s;
    at0 = *m.adam_t;
  }
  // running stats of the columns this thread updates (workgroup 0), prefetched: one
  // per 64-column pass (LDS layout) or its one column (lane-per-column layout)
  constexpr int CP = 8;
  float rmp[CP], rvp[CP];
  float rm0 = 0.f, rv0 = 0.f;
  if constexpr (InLds) {
#pragma unroll
    for (int q = 0; q < CP; ++q) {
      rmp[q] = rvp[q] = 0.f;
      if (row == 0 && q * (FT / 16) < 2 * K) {
        const int c2 = min(q * (FT / 16) + (tid >> 4), 2 * K - 1);
        rmp[q] = c2 < K ? m.mu_rm[c2] : m.s_rm[c2 - K];
        rvp[q] = c2 < K ? m.mu_rv[c2] : m.s_rv[c2 - K];
      }
    }
  } else if (row == 0 && tid < CG) {
    const int c2 = min(tid, 2 * K - 1);
    rm0 = c2 < K ? m.mu_rm[c2] : m.s_rm[c2 - K];
    rv0 = c2 < K ? m.mu_rv[c2] : m.s_rv[c2 - K];
  }
  // NeuralLDA: per-topic log-sum-exp over V from lda_beta_fwd's tile partials
  // (topics dealt to the workgroups' last wave)
  if (m.kind == GFK_LDA && wave == 3) {
    for (int k = row; k < K; k += gridDim.x) {
      float mx = -INFINITY, se = 0.f;
      for (int g = lane; g < m.dec_grid; g += 64) {
        const float* pp = m.ws_row_part + ((size_t)g * K + k) * 2;
        lse_merge(mx, se, pp[0], pp[1]);
      }
      wave_lse(mx, se);
      if (lane == 0) m.ws_lse[k] = mx + logf(se);
    }
  }
  if (row >= nb) {                         // nothing to do for this row: drain the DMA
    vm_barrier();
    return;
  }
  vm_barrier();
  GFK_STAMP(m, 1);

  // ---- column statistics over the batch: 4 threads per column, the column's
  // values held in registers across the mean and variance passes ----
  const float inv_nb = 1.f / (float)nb;
  if constexpr (PS) {
    for (int c = tid; c < 2 * K; c += FT) {
      cmean[c] = m.ws_colstat[c];
      crstd[c] = m.ws_colstat[2 * K + c];
    }
  } else if constexpr (InLds) {
    if (B <= 64) post_colstats_dpp<4>(m, mr, lr, cmean, crstd, rmp, rvp, nb, inv_nb, row, tid, LD);
    else post_colstats_dpp<8>(m, mr, lr, cmean, crstd, rmp, rvp, nb, inv_nb, row, tid, LD);
  } else {
    if (B <= 64) post_colstats<32>(m, mr, lr, cmean, crstd, red, rm0, rv0, nb, inv_nb, row, tid);
    else post_colstats<64>(m, mr, lr, cmean, crstd, red, rm0, rv0, nb, inv_nb, row, tid);
  }
  if (!PS && row == 0 && tid == 0) {
    *m.nbt_mu = nbt0 + 1;
    *m.nbt_s = nbt1 + 1;
    // the optimizer step of this minibatch: t and the bias corrections
    *m.adam_t = at0 + 1;
    double p1, p2;
    float c0, c1;
    adam_advance(m, pw0, pw1, p1, p2, c0, c1);
    m.adam_pow[0] = p1;
    m.adam_pow[1] = p2;
    m.adam_coef[0] = c0;
    m.adam_coef[1] = c1;
  }
  lds_barrier();
  GFK_STAMP(m, 2);

  // ---- own row: normalise, reparameterise, softmax, theta dropout, KL (wave 0) ----
  if (wave == 0) {
    float zq[KQ], muq[KQ], lsq[KQ];
    float zmax = -INFINITY, kl = 0.f, logpv = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      zq[q] = -INFINITY;
      muq[q] = lsq[q] = 0.f;
      if (k < K) {
        const float mu = (mr[row * LD + k] - cmean[k]) * crstd[k];
        const float ls = (lr[row * LD + k] - cmean[K + k]) * crstd[K + k];
        const float sd = expf(0.5f * ls);
        const float z = mu + ep[q] * sd;
        muq[q] = mu;
        lsq[q] = ls;
        zq[q] = z;
        zmax = fmaxf(zmax, z);
        const float dm = pm[q] - mu;
        kl += sd * sd / pv[q] + dm * dm / pv[q] - ls;
        logpv += logf(pv[q]);
      }
    }
    zmax = wave_max(zmax);
    kl = wave_sum(kl);
    logpv = wave_sum(logpv);
    float den = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      zq[q] = (lane + 64 * q < K) ? expf(zq[q] - zmax) : 0.f;
      den += zq[q];
    }
    const float inv = 1.f / wave_sum(den);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      if (k < K) {
        const int ix = row * K + k;
        const float th = zq[q] * inv;
        m.ws_mu[ix] = muq[q];
        m.ws_ls[ix] = lsq[q];
        m.ws_theta[ix] = th;
        m.ws_thetad[row * m.kt + k] = th * mt[q];
        if (m.lab_on) {
          red[k] = th * mt[q];
          m.ws_thd[ix] = th * mt[q];
        }
      }
    }
    if (lane == 0) m.ws_kl[row] = 0.5f * (kl - (float)K + logpv);
  }
  if (m.lab_on) post_label_head(m, red, row, nb, tid);
  GFK_STAMP(m, 3);
}

// ---------------------------------------------------------------------------
// backward, part 1 (own row): d theta_d from the decoder partials, softmax /
// reparameterisation / KL backward
// ---------------------------------------------------------------------------
// grid: bmax workgroups (+ the batch-level one, stage_flags GFK_POST_ROWS2).
// dynamic LDS: part[4][K]
extern "C" size_t gfk_row_bwd_smem(const GfkModel* m) { return sizeof(float) * 4 * (size_t)pad4(m->K); }

// The batch-level work of the step's backward (post_bwd's extra workgroup, here as row_bwd's
// last workgroup of PT threads): the priors' gradients -> their grad slots,
//   d prior_mean = w (nb pm - sum_b mu_b) / pv,
//   d prior_var  = w / 2 (nb / pv - sum_b exp(ls_b) / pv^2 - sum_b (pm - mu_b)^2 / pv^2),
// the loss sum_b (w KL_b + RL_b [+ CE_b]) -> loss_hist[step], and the step counter.  Thread
// (c, g) sums topic column c over rows g, g + NG, ... (CW = 64 / 128 / 256 columns per pass, the
// smallest covering K, NG = PT / CW row groups; 16 rows' loads in flight per thread), the groups'
// partials added in group order through LDS -- at K = 50 four groups of 16 rows where one thread
// per topic walked all 64 rows (the batched round's tail, 9 us).
// metrics (GfkModel kl_hist / rl_hist set): the step's mean KL and reconstruction terms over
// the batch rows, next to loss_hist (two more block sums behind the loss's; off the
// training path: only when a metrics window or the per-minibatch log asks for them)
__device__ __forceinline__ void post_term_hist(const GfkModel& m, int nb, int step0, float* scratch,
                                               int tid, int nt) {
  float k = 0.f, r = 0.f;
  for (int b = tid; b < nb; b += nt) {
    k += m.ws_kl[b];
    r += m.ws_rl[b];
  }
  lds_barrier();                     // every wave read the loss's partials from scratch
  const float ks = block_sum_wave0(k, scratch);
  lds_barrier();
  const float rs = block_sum_wave0(r, scratch);
  if (tid == 0) {
    m.kl_hist[step0] = ks / (float)nb;
    m.rl_hist[step0] = rs / (float)nb;
  }
}

__device__ __forceinline__ void post_batch_level(const GfkModel& m, int nb, float* scratch, int tid) {
  __shared__ float red[3 * PT];
  const int K = m.K;
  const float wk = m.kl_weight;
  const int step0 = *m.step;
  float lterm = 0.f;
  for (int b = tid; b < nb; b += PT)
    lterm += wk * m.ws_kl[b] + m.ws_rl[b] + (m.lab_on ? m.ws_ce[b] : 0.f);
  if (m.learn_priors) {
    constexpr int RB = 16;
    const int cw = K <= 64 ? 64 : K <= 128 ? 128 : PT, ng = PT / cw;
    const int c = tid % cw, g = tid / cw;
    for (int k0 = 0; k0 < K; k0 += cw) {
      const int k = k0 + c, kk = min(k, K - 1);
      const float pm = m.prior_mean[kk];
      float smu = 0.f, svar = 0.f, sdm2 = 0.f;
      for (int r0 = g; r0 < nb; r0 += RB * ng) {
        float mu[RB], ls[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const int r = min(r0 + ng * i, nb - 1);
          mu[i] = m.ws_mu[r * K + kk];
          ls[i] = m.ws_ls[r * K + kk];
        }
#pragma unroll
        for (int i = 0; i < RB; ++i)
          if (r0 + ng * i < nb) {
            smu += mu[i];
            svar += expf(ls[i]);
            const float dm = pm - mu[i];
            sdm2 += dm * dm;
          }
      }
      red[tid] = smu;
      red[PT + tid] = svar;
      red[2 * PT + tid] = sdm2;
      lds_barrier();
      if (g == 0 && k < K) {
        for (int j = 1; j < ng; ++j) {
          smu += red[c + j * cw];
          svar += red[PT + c + j * cw];
          sdm2 += red[2 * PT + c + j * cw];
        }
        const float pv = m.prior_var[k];
        m.prior_mean[k + m.off_g] = wk * ((float)nb * pm - smu) / pv;
        m.prior_var[k + m.off_g] = wk * 0.5f * ((float)nb / pv - svar / (pv * pv) - sdm2 / (pv * pv));
      }
      lds_barrier();
    }
  }
  const float l = block_sum_wave0(lterm, scratch);
  if (tid == 0) {
    m.loss_hist[step0] = l;
    *m.step = step0 + 1;
  }
  if (m.kl_hist) post_term_hist(m, nb, step0, scratch, tid, PT);
}

// KQ = ceil(K / 64) topics per lane: only live topics are loaded (K <= 64 -> one
// load per partial), U partials per wave per round so a row's partials are in
// flight at once.
template <int KQ, bool GB = false>
__global__ void __launch_bounds__(PT) gfk_row_bwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float part[];
  int K = m.K, B = m.bmax, np = m.n_dpart + (m.lab_on ? 1 : 0);   // + the label head's slab
  const float* dpart = m.ws_dthetad;
  const int32_t* nbp = m.ws_nb;
  keep(K, B, np, dpart, nbp);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int row = gfk_bx();
  const int nb = *nbp;
  if ((m.stage_flags & GFK_POST_ROWS2) && row == B) {
    post_batch_level(m, nb, part, tid);    // the batch-level workgroup (grid = bmax + 1)
    return;
  }
  if (row >= nb) return;
  GFK_STAMP(m, 8);
  // ---- wave w sums partials w, w + 4, ... of the row (lane = topic), all loads first ----
  constexpr int U = 32 / KQ;
  float acc[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) acc[q] = 0.f;
  for (int p0 = wave; p0 < np; p0 += 4 * U) {
    float v[U][KQ];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const int p = min(p0 + 4 * u, np - 1), k = min(lane + 64 * q, K - 1);
        v[u][q] = dpart[((size_t)p * B + row) * K + k];
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < KQ; ++q) acc[q] += p0 + 4 * u < np ? v[u][q] : 0.f;
  }
  // the own row's stash (wave 0)
  float th[KQ], mt[KQ], mu[KQ], ls[KQ], ep[KQ], pm[KQ], pv[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = min(lane + 64 * q, K - 1), i = row * K + k;
    th[q] = m.ws_theta[i];
    mt[q] = m.ws_mask_t[i];
    mu[q] = m.ws_mu[i];
    ls[q] = m.ws_ls[i];
    ep[q] = m.ws_eps[i];
    pm[q] = m.prior_mean[k];
    pv[q] = m.prior_var[k];
  }
#pragma unroll
  for (int q = 0; q < KQ; ++q)
    if (lane + 64 * q < pad4(K)) part[wave * pad4(K) + lane + 64 * q] = acc[q];
  lds_barrier();
  if (wave != 0) return;
  const float wk = m.kl_weight;
  float dtd[KQ], c = 0.f;
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = min(lane + 64 * q, pad4(K) - 1), P4 = pad4(K);
    dtd[q] = (part[k] + part[P4 + k]) + (part[2 * P4 + k] + part[3 * P4 + k]);   // d theta_d
    if (lane + 64 * q < K) {
      m.ws_dtheta[row * K + lane + 64 * q] = dtd[q];
      c += mt[q] * dtd[q] * th[q];
    }
  }
  c = wave_sum(c);
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = lane + 64 * q;
    if (k >= K) continue;
    const float dz = th[q] * (mt[q] * dtd[q] - c);
    const float sd = expf(0.5f * ls[q]);
    m.ws_dmu[row * K + k] = dz + wk * (mu[q] - pm[q]) / pv[q];
    m.ws_dls[row * K + k] = dz * ep[q] * 0.5f * sd + wk * 0.5f * (sd * sd / pv[q] - 1.f);
  }
  GFK_STAMP(m, 9);
}

// ---------------------------------------------------------------------------
// backward, part 2
// ---------------------------------------------------------------------------
// LDS plan (floats): dmu, dls, mu, ls [B][K] + s1..s4 [2K] + own-row vectors
// (dmr|dlr [2K], dz ping-pong [2][hmax], z rows, mask) + staged weights.
struct PostLds {
  int dmu, dls, mu, ls, sums, pm, dr, v0, v1, zrow, mask, red, red2, w, total;
};

__host__ __device__ inline PostLds post_lds(const GfkModel& m) {
  PostLds L;
  const int B = m.bmax, K = m.K, hm = pad4(post_hmax(m));
  const int mat = batch_in_lds(m) ? B * post_lds_ld(K) : 0;
  int o = 0;
  L.dmu = o; o += mat;
  L.dls = o; o += mat;
  L.mu = o; o += mat;
  L.ls = o; o += mat;
  L.sums = o; o += 4 * pad4(2 * K);
  L.pm = o; o += pad4(K);
  L.dr = o; o += 2 * pad4(K);
  L.v0 = o; o += hm;
  L.v1 = o; o += hm;
  L.zrow = o;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) o += pad4(m.H[l]);
  L.mask = o; o += pad4(gfk_hlast(m));
  L.red = o; o += FT / 64;                // block_sum_wave0 scratch, one float per wave
  L.red2 = o; o += 2 * FT;                // column-reduction scratch [2][FT]
  L.w = o;
  if (m.stage_flags & 1) o += post_weight_floats(m);
  L.total = o;
  return L;
}

extern "C" size_t gfk_post_bwd_smem(const GfkModel* m) { return sizeof(float) * (size_t)post_lds(*m).total; }

// out[j] = sum_k term(k, j) for j < n_out: LPO lanes per output split k (DPP quad /
// row reduction).  LPO = 4 covers 64 outputs per pass of the 256-thread workgroup,
// so the usual hidden widths take one pass instead of four.
template <int LPO, class Term, class Epi>
__device__ __forceinline__ void gemv_lanes(int n_out, int n_in, int tid, Term term, Epi epi) {
  const int s = tid & (LPO - 1);
  for (int j0 = 0; j0 < n_out; j0 += FT / LPO) {
    const int j = j0 + tid / LPO;
    float acc = 0.f;
    if (j < n_out) {
      float a2 = 0.f;                  // two chains, unrolled: LDS reads of 4 k in flight
      int k = s;
#pragma unroll 2
      for (; k + LPO < n_in; k += 2 * LPO) {
        acc += term(k, j);
        a2 += term(k + LPO, j);
      }
      if (k < n_in) acc += term(k, j);
      acc += a2;
    }
    acc = LPO == 4 ? quad_sum(acc) : row16_sum(acc);
    if (s == 0 && j < n_out) epi(j, acc);
  }
}

template <class Term, class Epi>
__device__ __forceinline__ void gemv_cols(int n_out, int n_in, int tid, Term term, Epi epi) {
  if (n_out * 16 <= FT) gemv_lanes<16>(n_out, n_in, tid, term, epi);
  else gemv_lanes<4>(n_out, n_in, tid, term, epi);
}

// out[j] = sum_k x[k] W[k * ldw + j] for j < n_out (column of a row-major W).
template <class Epi>
__device__ __forceinline__ void colvec_gemv(const float* W, int ldw, const float* x, int n_out, int n_in,
                                            int tid, Epi epi) {
  gemv_cols(n_out, n_in, tid, [&](int k, int j) { return x[k] * W[k * ldw + j]; }, epi);
}

// Column sums over the batch for the BN backward of the heads: s1[c2] = sum_b dy,
// s2[c2] = sum_b dy * xhat over the 2K columns (mu | log sigma^2), lane-per-column
// (see CG / NGR above).  red: [2][FT] LDS scratch.
template <int RPG>
__device__ __forceinline__ void post_bn_sums(int K, int nb, const float* dmu, const float* dls,
                                             const float* mu, const float* ls, float* s1o,
                                             float* s2o, float* red, int tid) {
  constexpr int RB = 16;                  // rows per load batch (registers)
  const int c2 = tid % CG, grp = tid / CG;
  const int cc = min(c2, 2 * K - 1), k = cc < K ? cc : cc - K;
  const float* dy = cc < K ? dmu : dls;
  const float* xh = cc < K ? mu : ls;
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i0 = 0; i0 < RPG; i0 += RB) {
    float dv[RB], xv[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = min(grp + NGR * (i0 + i), nb - 1);
      dv[i] = dy[r * K + k];
      xv[i] = xh[r * K + k];
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
      if (grp + NGR * (i0 + i) < nb) {
        s1 += dv[i];
        s2 += dv[i] * xv[i];
      }
  }
  red[tid] = s1;
  red[FT + tid] = s2;
  lds_barrier();
  if (grp == 0 && c2 < 2 * K) {
    s1o[c2] = red[c2] + red[CG + c2];
    s2o[c2] = red[FT + c2] + red[FT + CG + c2];
  }
}

// The extra workgroup's sums for the prior gradients: s3[c2] = sum_b mu (c2 < K) |
// sum_b exp(ls) (c2 >= K), s4[k] = sum_b (prior_mean - mu)^2 -- same layout.
template <int RPG>
__device__ __forceinline__ void post_prior_sums(int K, int nb, const float* mu, const float* ls,
                                                const float* pmean, float* s3o, float* s4o,
                                                float* red, int tid) {
  constexpr int RB = 16;
  const int c2 = tid % CG, grp = tid / CG;
  const int cc = min(c2, 2 * K - 1), k = cc < K ? cc : cc - K;
  const float* xh = cc < K ? mu : ls;
  const float pm = pmean[k];
  float s3 = 0.f, s4 = 0.f;
#pragma unroll
  for (int i0 = 0; i0 < RPG; i0 += RB) {
    float xv[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) xv[i] = xh[min(grp + NGR * (i0 + i), nb - 1) * K + k];
#pragma unroll
    for (int i = 0; i < RB; ++i)
      if (grp + NGR * (i0 + i) < nb) {
        const float x = xv[i];
        s3 += cc < K ? x : expf(x);
        const float dm = pm - x;
        s4 += cc < K ? dm * dm : 0.f;
      }
  }
  red[tid] = s3;
  red[FT + tid] = s4;
  lds_barrier();
  if (grp == 0 && c2 < 2 * K) {
    s3o[c2] = red[c2] + red[CG + c2];
    s4o[c2] = red[FT + c2] + red[FT + CG + c2];
  }
}

// grid: bmax + 1 workgroups: row = gfk_bx() < bmax, plus one extra workgroup
// (the last) for the batch-level work -- prior gradients, the loss, the step
// counter -- so no row workgroup carries it on the critical path.
// PS (the large-batch plan): the column sums come precomputed from ws_colstat.
// R rows per workgroup (stage_flags GFK_POST_ROWS2, batched launches: R = 2): the batch
// matrices, weights and column sums are staged / computed once for both rows, whose own-row
// sections run one after the other -- M clients' bmax / 2 workgroups fill one round of the
// CUs (one 16-wave workgroup per CU) where bmax + 1 ran in three
template <bool InLds, bool Staged, bool GB = false, bool PS = false, int R = 1>
__global__ void __launch_bounds__(FT) gfk_post_bwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model_ref(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int K = m.K, B = m.bmax, nh = m.n_hidden, sflags = m.stage_flags;
  const float *dmu_g = m.ws_dmu, *dls_g = m.ws_dls, *mu_g = m.ws_mu, *ls_g = m.ws_ls;
  const int32_t* nbp = m.ws_nb;
  keep(K, B, nh, sflags, dmu_g, dls_g, mu_g, ls_g, nbp);
  const int tid = threadIdx.x, lane = tid & 63;
  const int r0 = gfk_bx() * R;          // this workgroup's first row
  int row = r0;
  const bool extra = !(sflags & GFK_POST_ROWS2) && gfk_bx() == (int)gridDim.x - 1;
  const PostLds L = post_lds(m);
  const int Hl = gfk_hlast(m);
  constexpr bool staged = Staged;
  GFK_STAMP(m, 10);

  constexpr bool in_lds = InLds;
  const int LD = in_lds ? post_lds_ld(K) : K;   // row stride of the batch matrices
  // ---- one round: the four [B][K] matrices, the own row, the weights, stats ----
  if (in_lds) {
    glds_rows(smem + L.dmu, dmu_g, B, K, LD, tid, FT);
    glds_rows(smem + L.dls, dls_g, B, K, LD, tid, FT);
    glds_rows(smem + L.mu, mu_g, B, K, LD, tid, FT);
    glds_rows(smem + L.ls, ls_g, B, K, LD, tid, FT);
  }
  if (!extra) {                         // own row (the extra workgroup has none)
    int o = L.zrow;
#pragma unroll
    for (int l = 0; l < GFK_MAX_LAYERS; ++l) {
      if (l < nh) {
        glds_copy(smem + o, m.ws_z[l] + (size_t)row * m.H[l], m.H[l], tid, FT);
        o += pad4(m.H[l]);
      }
    }
    glds_copy(smem + L.mask, m.ws_mask_h + (size_t)row * Hl, Hl, tid, FT);
  }
  glds_copy(smem + L.pm, m.prior_mean, K, tid, FT);
  if (staged && !extra) {
    float* p = smem + L.w;
    glds_copy(p, m.w_mu, K * Hl, tid, FT); p += pad4(K * Hl);
    glds_copy(p, m.w_s, K * Hl, tid, FT); p += pad4(K * Hl);
#pragma unroll
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
      if (l + 1 < nh) { glds_copy(p, m.w_h[l], m.H[l + 1] * m.H[l], tid, FT); p += pad4(m.H[l + 1] * m.H[l]); }
  }
  const int nb = *nbp;
  constexpr int CQ = (512 + FT - 1) / FT;   // columns tid, tid + FT, ... of the 2K (K <= 256)
  float rs[CQ];                         // rstd of those columns
#pragma unroll
  for (int q = 0; q < CQ; ++q) rs[q] = m.ws_bn_rstd[min(tid + q * FT, 2 * K - 1)];
  // extra workgroup: the loss terms, priors, step
  float lterm = 0.f, pmk = 0.f, pvk = 1.f;
  int step0 = 0;
  if (extra) {
    if (tid < nb) lterm = m.kl_weight * m.ws_kl[tid] + m.ws_rl[tid] + (m.lab_on ? m.ws_ce[tid] : 0.f);
    if (tid < K) { pmk = m.prior_mean[tid]; pvk = m.prior_var[tid]; }
    if (tid == 0) step0 = *m.step;
  }
  if (row >= nb && !extra) {
    vm_barrier();
    return;
  }
  vm_barrier();
  GFK_STAMP(m, 11);

  // ---- column sums over the batch (DPP rows in LDS, lane-per-column from L2) ----
  const float* dmu = in_lds ? smem + L.dmu : dmu_g;
  const float* dls = in_lds ? smem + L.dls : dls_g;
  const float* mu = in_lds ? smem + L.mu : mu_g;
  const float* ls = in_lds ? smem + L.ls : ls_g;
  float* S = smem + L.sums;             // [4][pad4(2K)]: sum dy, sum dy * xh | (extra:) priors
  const int P2 = pad4(2 * K);
  const float inv_nb = 1.f / (float)nb;
  if (extra) {
    // ---- extra workgroup: prior gradients (-> grad slots), loss, step ----
    const float* pmean = smem + L.pm;   // prior mean, staged
    if constexpr (in_lds) {             // LDS: 16 lanes per column, DPP reductions
      for (int cb = 0; cb < 2 * K; cb += FT / 16) {
        const int c2 = cb + (tid >> 4), g = tid & 15;
        const bool valid = c2 < 2 * K;
        const int k = c2 < K ? c2 : c2 - K;
        const float* xh = c2 < K ? mu : ls;
        const float pm = pmean[k];
        float s3 = 0.f, s4 = 0.f;         // sum mu | sum exp(ls), sum (pm - mu)^2
        if (valid)
#pragma unroll 4
          for (int r = g; r < nb; r += 16) {
            const float x = xh[r * LD + k];
            s3 += c2 < K ? x : expf(x);
            const float dm = pm - x;
            s4 += c2 < K ? dm * dm : 0.f;
          }
        s3 = row16_sum(s3);
        s4 = row16_sum(s4);
        if (valid && g == 0) {
          S[2 * P2 + c2] = s3;
          S[3 * P2 + c2] = s4;
        }
      }
    } else if constexpr (PS) {          // precomputed (gfk_post_colstats_lb_k)
      for (int c = tid; c < 2 * K; c += FT) {
        S[2 * P2 + c] = m.ws_colstat[8 * K + c];
        S[3 * P2 + c] = m.ws_colstat[10 * K + c];
      }
    } else {                            // L2: lane-per-column (coalesced)
      if (B <= 64) post_prior_sums<32>(K, nb, mu, ls, pmean, S + 2 * P2, S + 3 * P2, smem + L.red2, tid);
      else post_prior_sums<64>(K, nb, mu, ls, pmean, S + 2 * P2, S + 3 * P2, smem + L.red2, tid);
    }
    lds_barrier();
    const float wk = m.kl_weight;
    if (tid < K && m.learn_priors) {
      const float sdm2 = S[3 * P2 + tid];                 // sum_b (pm - mu_b)^2
      const float smu = S[2 * P2 + tid], svar = S[2 * P2 + K + tid];
      m.prior_mean[tid + m.off_g] = wk * ((float)nb * pmk - smu) / pvk;
      m.prior_var[tid + m.off_g] =
          wk * 0.5f * ((float)nb / pvk - svar / (pvk * pvk) - sdm2 / (pvk * pvk));
    }
    const float l = block_sum_wave0(lterm, smem + L.red);
    if (tid == 0) {
      m.loss_hist[step0] = l;
      *m.step = step0 + 1;
    }
    if (m.kl_hist) post_term_hist(m, nb, step0, smem + L.red, tid, FT);
    return;
  }
  if constexpr (in_lds) {               // LDS: 16 lanes per column, DPP reductions
    for (int cb = 0; cb < 2 * K; cb += FT / 16) {
      const int c2 = cb + (tid >> 4), g = tid & 15;
      const bool valid = c2 < 2 * K;
      const int k = c2 < K ? c2 : c2 - K;
      const float* dy = c2 < K ? dmu : dls;
      const float* xh = c2 < K ? mu : ls;
      float s1 = 0.f, s2 = 0.f;
      if (valid)
#pragma unroll 4
        for (int r = g; r < nb; r += 16) {
          const float d = dy[r * LD + k], x = xh[r * LD + k];
          s1 += d;
          s2 += d * x;
        }
      s1 = row16_sum(s1);
      s2 = row16_sum(s2);
      if (valid && g == 0) {
        S[c2] = s1;
        S[P2 + c2] = s2;
      }
    }
  } else if constexpr (PS) {            // precomputed (gfk_post_colstats_lb_k)
    for (int c = tid; c < 2 * K; c += FT) {
      S[c] = m.ws_colstat[4 * K + c];
      S[P2 + c] = m.ws_colstat[6 * K + c];
    }
  } else {                              // L2: lane-per-column (coalesced)
    if (B <= 64) post_bn_sums<32>(K, nb, dmu, dls, mu, ls, S, S + P2, smem + L.red2, tid);
    else post_bn_sums<64>(K, nb, dmu, dls, mu, ls, S, S + P2, smem + L.red2, tid);
  }
  lds_barrier();
  GFK_STAMP(m, 12);
  GFK_STAMP(m, 14);

#pragma unroll 1
  for (int rr = 0; rr < R; ++rr) {
  row = r0 + rr;
  if (row >= nb) break;                 // (uniform)
  if (rr > 0) {                         // the next row's z / mask (the previous row's reads done)
    lds_barrier();
    int o = L.zrow;
#pragma unroll
    for (int l = 0; l < GFK_MAX_LAYERS; ++l) {
      if (l < nh) {
        glds_copy(smem + o, m.ws_z[l] + (size_t)row * m.H[l], m.H[l], tid, FT);
        o += pad4(m.H[l]);
      }
    }
    glds_copy(smem + L.mask, m.ws_mask_h + (size_t)row * Hl, Hl, tid, FT);
    vm_barrier();
  }
  // ---- own row: BN backward -> d mu_raw | d ls_raw ----
  float* dr = smem + L.dr;              // [2K]: dmr then dlr
#pragma unroll
  for (int q = 0; q < CQ; ++q) {
    const int c2 = tid + q * FT;
    if (c2 < 2 * K) {
      const int k = c2 < K ? c2 : c2 - K;
      const float* dy = c2 < K ? dmu : dls;
      const float* xh = c2 < K ? mu : ls;
      const float v =
          rs[q] * (dy[row * LD + k] - S[c2] * inv_nb - xh[row * LD + k] * S[P2 + c2] * inv_nb);
      dr[c2] = v;
      (c2 < K ? m.ws_dmr : m.ws_dlr)[row * K + k] = v;
    }
  }
  lds_barrier();
  GFK_STAMP(m, 15);

  // ---- heads backward: d hd[j] = sum_k dmr[k] W_mu[k][j] + dlr[k] W_s[k][j] ----
  const float* wst = smem + L.w;
  const float* Wmu = staged ? wst : m.w_mu;
  const float* Ws = staged ? wst + pad4(K * Hl) : m.w_s;
  float* v0 = smem + L.v0;
  float* v1 = smem + L.v1;
  const float* zrow = smem + L.zrow;
  int zoff_last = 0;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < nh) zoff_last += pad4(m.H[l]);
  {
    const float* mask = smem + L.mask;
    const float* zl = zrow + zoff_last;
    float* dzo = m.ws_dz[nh - 1] + (size_t)row * Hl;
    gemv_cols(Hl, K, tid,
              [&](int k, int j) { return dr[k] * Wmu[k * Hl + j] + dr[K + k] * Ws[k * Hl + j]; },
              [&](int j, float acc) {
                const float g = acc * mask[j] * act_d(m.act, zl[j]);
                v0[j] = g;
                dzo[j] = g;
              });
  }
  lds_barrier();
  GFK_STAMP(m, 29);

  // ---- hidden layers, last to first: dz_{l} = (dz_{l+1} W_l) * act'(z_l) ----
  float* din = v0;
  float* dout = v1;
  const float* wl_base = wst + 2 * pad4(K * Hl);
#pragma unroll
  for (int l = GFK_MAX_LAYERS - 2; l >= 0; --l) {
    if (l + 1 >= nh) continue;
    const int Hi = m.H[l], Ho = m.H[l + 1];
    int woff = 0, zoff = 0;
#pragma unroll
    for (int ll = 0; ll + 1 < GFK_MAX_LAYERS; ++ll)
      if (ll < l) { woff += pad4(m.H[ll + 1] * m.H[ll]); zoff += pad4(m.H[ll]); }
    const float* W = staged ? wl_base + woff : m.w_h[l];
    const float* zl = zrow + zoff;
    float* dzo = m.ws_dz[l] + (size_t)row * Hi;
    colvec_gemv(W, Hi, din, Hi, Ho, tid, [&](int i, float acc) {
      const float g = acc * act_d(m.act, zl[i]);
      dout[i] = g;
      dzo[i] = g;
    });
    lds_barrier();
    float* t = din; din = dout; dout = t;
  }
  }                                     // (rows of the workgroup)
  GFK_STAMP(m, 13);
}

// ---------------------------------------------------------------------------
// next batch
// ---------------------------------------------------------------------------
template <bool GB>
__global__ void gfk_batch_prep(GfkArgT<GB> ga) { prepare_next_batch(gfk_model(ga)); }

// Publishes the prepared batch (doc ids of every row < bmax, nb) before the dense
// contextual GEMMs of the CTM encoders, which run on all bmax rows.
template <bool GB = false>
__global__ void gfk_batch_docs(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  const int32_t* nxt = m.ws_next;
  for (int b = threadIdx.x; b < m.bmax; b += blockDim.x) m.ws_doc[b] = nxt[1 + b];
  if (threadIdx.x == 0) *m.ws_nb = nxt[0];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Large batches (stage_flags GFK_LB): the column statistics of the [B][2K] batch matrices,
// computed ONCE per step by ceil(2K / 64) workgroups -- the row workgroups' own recomputation
// (one round trip, no grid sync: the right trade at B <= 128) reads the whole matrices per
// row, B^2 K floats from L2 per kernel (post_fwd 36 us, post_bwd 62 us at B = 256, K = 50:
// profiles/r5/lb256_k50_kernels.md).  Lane = column c2 = 64 blockIdx + lane of the 2K
// (mu | log sigma^2) columns, wave w = rows w + 16 i (coalesced 256-B row segments), the 16
// waves' partials met in LDS.  BWD = false: mean / rstd of the raw heads (two-pass variance,
// as torch's batch norm) -> ws_colstat[0, 2K) / [2K, 4K) and ws_bn_rstd, the running
// statistics, and (workgroup 0) the counters and the optimizer step -- post_fwd's row-0
// duties.  BWD = true: S1 = sum_b dy, S2 = sum_b dy xhat -> ws_colstat[4K, 6K) / [6K, 8K), and
// the prior gradients' sums -> [8K, 10K) / [10K, 12K) (post_bwd's batch-level workgroup:
// alone over all rows it was the kernel's tail, 39 us at B = 256).
template <bool BWD>
__global__ void __launch_bounds__(FT) gfk_post_colstats_lb_k(GfkArgT<false> ga) {
  const GfkModel& m = ga.m;
  __shared__ float red[2][16][64];
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c2 = 64 * (int)blockIdx.x + lane, cc = min(c2, 2 * K - 1);
  const int k = cc < K ? cc : cc - K;
  const int nb = *m.ws_nb;
  const float inv_nb = 1.f / (float)nb;
  float* cs = m.ws_colstat;
  if constexpr (!BWD) {
    const float* x = (cc < K ? m.ws_mu_raw : m.ws_ls_raw) + k;
    float rm0 = 0.f, rv0 = 0.f;
    if (w == 0) {
      rm0 = cc < K ? m.mu_rm[k] : m.s_rm[k];
      rv0 = cc < K ? m.mu_rv[k] : m.s_rv[k];
    }
    float sm = 0.f;
#pragma unroll 4
    for (int r = w; r < nb; r += 16) sm += x[r * K];
    red[0][w][lane] = sm;
    __syncthreads();
    float mean = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) mean += red[0][j][lane];
    mean *= inv_nb;
    float q = 0.f;
#pragma unroll 4
    for (int r = w; r < nb; r += 16) {
      const float d = x[r * K] - mean;
      q += d * d;
    }
    red[1][w][lane] = q;
    __syncthreads();
    float var = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) var += red[1][j][lane];
    var *= inv_nb;
    const float rstd = rsqrtf(var + m.bn_eps);
    if (w == 0 && c2 < 2 * K) {
      cs[c2] = mean;
      cs[2 * K + c2] = rstd;
      m.ws_bn_rstd[c2] = rstd;
      float* rm = c2 < K ? m.mu_rm + k : m.s_rm + k;
      float* rv = c2 < K ? m.mu_rv + k : m.s_rv + k;
      const float mom = m.bn_momentum;
      const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
      float nm = (1.f - mom) * rm0 + mom * mean, nv = (1.f - mom) * rv0 + mom * unb;
      if (m.fed_scale_on && is_shared(m, rm)) { nm *= m.fed_scale; nv *= m.fed_scale; }
      *rm = nm;
      *rv = nv;
    }
    if (blockIdx.x == 0 && tid == 0) {
      const double pw0 = m.adam_pow[0], pw1 = m.adam_pow[1];
      *m.nbt_mu += 1;
      *m.nbt_s += 1;
      *m.adam_t += 1;
      double p1, p2;
      float c0, c1;
      adam_advance(m, pw0, pw1, p1, p2, c0, c1);
      m.adam_pow[0] = p1;
      m.adam_pow[1] = p2;
      m.adam_coef[0] = c0;
      m.adam_coef[1] = c1;
    }
  } else {
    // + the prior gradients' sums (post_bwd's batch-level workgroup): S3 = sum_b mu
    // (c2 < K) | sum_b exp(ls) (c2 >= K), S4 = sum_b (prior_mean - mu)^2 (c2 < K)
    const float* dy = (cc < K ? m.ws_dmu : m.ws_dls) + k;
    const float* xh = (cc < K ? m.ws_mu : m.ws_ls) + k;
    const float pm = m.prior_mean[k];
    float s1 = 0.f, s2 = 0.f, s3 = 0.f, s4 = 0.f;
#pragma unroll 4
    for (int r = w; r < nb; r += 16) {
      const float d = dy[r * K], x = xh[r * K];
      s1 += d;
      s2 += d * x;
      s3 += cc < K ? x : expf(x);
      const float dm = pm - x;
      s4 += cc < K ? dm * dm : 0.f;
    }
    __shared__ float red2[2][16][64];
    red[0][w][lane] = s1;
    red[1][w][lane] = s2;
    red2[0][w][lane] = s3;
    red2[1][w][lane] = s4;
    __syncthreads();
    if (w == 0 && c2 < 2 * K) {
      float a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        a1 += red[0][j][lane];
        a2 += red[1][j][lane];
        a3 += red2[0][j][lane];
        a4 += red2[1][j][lane];
      }
      cs[4 * K + c2] = a1;
      cs[6 * K + c2] = a2;
      cs[8 * K + c2] = a3;
      cs[10 * K + c2] = a4;
    }
  }
}

static int launch_colstats_lb(const GfkModel* m, hipStream_t s, bool bwd) {
  if (m->n_batch > 1 || !m->ws_colstat) return -1;
  const dim3 g((2 * m->K + 63) / 64);
  if (bwd) hipLaunchKernelGGL((gfk_post_colstats_lb_k<true>), g, dim3(FT), 0, s, GfkArgT<false>{*m});
  else hipLaunchKernelGGL((gfk_post_colstats_lb_k<false>), g, dim3(FT), 0, s, GfkArgT<false>{*m});
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_post_fwd(const GfkModel* m, hipStream_t s) {
  if (m->stage_flags & GFK_LB) {        // large batches: statistics once, then the rows
    if (batch_in_lds(*m)) return -1;
    const int e = launch_colstats_lb(m, s, false);
    if (e) return e;
    if (m->K <= 256)
      hipLaunchKernelGGL((gfk_post_fwd_k<false, false, true>), dim3(m->bmax), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<false>{*m});
    else if (m->K <= 512)
      hipLaunchKernelGGL((gfk_post_fwd_k<false, false, true, 8>), dim3(m->bmax), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<false>{*m});
    else
      return -1;
    return (int)hipGetLastError();
  }
  if (batch_in_lds(*m))
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_fwd_k<true, true>), gfk_grid(dim3(m->bmax), m), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_fwd_k<true, false>), dim3(m->bmax), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<false>{*m}); } while (0);
  else
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_fwd_k<false, true>), gfk_grid(dim3(m->bmax), m), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_fwd_k<false, false>), dim3(m->bmax), dim3(FT), gfk_post_fwd_smem(m), s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_post_bwd(const GfkModel* m, hipStream_t s) {
  const int kq = (m->K + 63) / 64;
  // GFK_POST_ROWS2 (batched launches only): the batch-level workgroup runs in row_bwd
  const bool moved = m->stage_flags & GFK_POST_ROWS2;
  if (moved && (m->n_batch < 2 || (m->stage_flags & GFK_LB))) return -1;
  const dim3 g(m->bmax + (moved ? 1 : 0)), t(PT);
  const size_t sm = gfk_row_bwd_smem(m);
  if (kq <= 1) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_row_bwd_k<1, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_row_bwd_k<1, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else if (kq == 2) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_row_bwd_k<2, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_row_bwd_k<2, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else if (kq == 3) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_row_bwd_k<3, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_row_bwd_k<3, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else if (kq > 4) {                   // K <= 512 (the large-batch plan; one client)
    if (kq > 8 || m->n_batch > 1) return -1;
    hipLaunchKernelGGL((gfk_row_bwd_k<8, false>), g, t, sm, s, GfkArgT<false>{*m});
  }
  else do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_row_bwd_k<4, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_row_bwd_k<4, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const dim3 gb(m->bmax + (moved ? 0 : 1)), tb(FT);   // + the prior / loss / step workgroup
  const size_t sb = gfk_post_bwd_smem(m);
  const bool st = m->stage_flags & 1;
  if (moved) {
    // two rows per workgroup (batched launches)
    const dim3 g2((m->bmax + 1) / 2 + (moved ? 0 : 1));
    const GfkArgT<true> a{gfk_dev(m)};
    if (batch_in_lds(*m)) {
      if (st) hipLaunchKernelGGL((gfk_post_bwd_k<true, true, true, false, 2>), gfk_grid(g2, m), tb, sb, s, a);
      else hipLaunchKernelGGL((gfk_post_bwd_k<true, false, true, false, 2>), gfk_grid(g2, m), tb, sb, s, a);
    } else {
      if (st) hipLaunchKernelGGL((gfk_post_bwd_k<false, true, true, false, 2>), gfk_grid(g2, m), tb, sb, s, a);
      else hipLaunchKernelGGL((gfk_post_bwd_k<false, false, true, false, 2>), gfk_grid(g2, m), tb, sb, s, a);
    }
    return (int)hipGetLastError();
  }
  if (m->stage_flags & GFK_LB) {        // large batches: the column sums once, then the rows
    if (batch_in_lds(*m)) return -1;
    const int e2 = launch_colstats_lb(m, s, true);
    if (e2) return e2;
    if (st) hipLaunchKernelGGL((gfk_post_bwd_k<false, true, false, true>), gb, tb, sb, s, GfkArgT<false>{*m});
    else hipLaunchKernelGGL((gfk_post_bwd_k<false, false, false, true>), gb, tb, sb, s, GfkArgT<false>{*m});
    return (int)hipGetLastError();
  }
  if (batch_in_lds(*m)) {
    if (st) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_bwd_k<true, true, true>), gfk_grid(gb, m), tb, sb, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_bwd_k<true, true, false>), gb, tb, sb, s, GfkArgT<false>{*m}); } while (0);
    else do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_bwd_k<true, false, true>), gfk_grid(gb, m), tb, sb, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_bwd_k<true, false, false>), gb, tb, sb, s, GfkArgT<false>{*m}); } while (0);
  } else {
    if (st) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_bwd_k<false, true, true>), gfk_grid(gb, m), tb, sb, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_bwd_k<false, true, false>), gb, tb, sb, s, GfkArgT<false>{*m}); } while (0);
    else do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_post_bwd_k<false, false, true>), gfk_grid(gb, m), tb, sb, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_post_bwd_k<false, false, false>), gb, tb, sb, s, GfkArgT<false>{*m}); } while (0);
  }
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_batch_prep(const GfkModel* m, hipStream_t s) {
  do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_batch_prep<true>), gfk_grid(dim3(1), m), dim3(256), 0, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_batch_prep<false>), dim3(1), dim3(256), 0, s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_batch_docs(const GfkModel* m, hipStream_t s) {
  do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_batch_docs<true>), gfk_grid(dim3(1), m), dim3(256), 0, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_batch_docs<false>), dim3(1), dim3(256), 0, s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_post_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)gfk_post_fwd_k<true>, (const void*)gfk_post_fwd_k<true, true>, (const void*)gfk_post_fwd_k<false>, (const void*)gfk_post_fwd_k<false, true>,
                      (const void*)gfk_row_bwd_k<1>, (const void*)gfk_row_bwd_k<1, true>, (const void*)gfk_row_bwd_k<2>, (const void*)gfk_row_bwd_k<2, true>,
                      (const void*)gfk_row_bwd_k<3>, (const void*)gfk_row_bwd_k<3, true>, (const void*)gfk_row_bwd_k<4>, (const void*)gfk_row_bwd_k<4, true>,
                      (const void*)gfk_post_bwd_k<true, true>, (const void*)gfk_post_bwd_k<true, true, true>, (const void*)gfk_post_bwd_k<true, false>, (const void*)gfk_post_bwd_k<true, false, true>,
                      (const void*)gfk_post_bwd_k<false, true>, (const void*)gfk_post_bwd_k<false, true, true>, (const void*)gfk_post_bwd_k<false, false>, (const void*)gfk_post_bwd_k<false, false, true>,
                      (const void*)gfk_post_fwd_k<false, false, true>, (const void*)gfk_post_fwd_k<false, false, true, 8>,
                      (const void*)gfk_row_bwd_k<8>, (const void*)gfk_post_bwd_k<false, true, false, true>,
                      (const void*)gfk_post_bwd_k<false, false, false, true>,
                      (const void*)gfk_post_bwd_k<true, true, true, false, 2>, (const void*)gfk_post_bwd_k<true, false, true, false, 2>,
                      (const void*)gfk_post_bwd_k<false, true, true, false, 2>, (const void*)gfk_post_bwd_k<false, false, true, false, 2>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" size_t gfk_post_smem(const GfkModel* m) {
  size_t a = gfk_post_fwd_smem(m), b = gfk_post_bwd_smem(m), c = gfk_row_bwd_smem(m);
  a = a > b ? a : b;
  return a > c ? a : c;
}

extern "C" size_t gfk_post_weight_bytes(const GfkModel* m) {
  return sizeof(float) * (size_t)post_weight_floats(*m);
}
