// ProdLDA decoder: word_dist = softmax_V(BN_batch(theta_d @ beta)), its
// reconstruction loss -sum x log(word_dist + 1e-10), and the backward.
//
// Reference math: decoder_network.py:121-126, avitm.py:225.
//
// Tiling (MI355X-first): one workgroup (4 waves) owns one vocabulary tile of
// VB=64 columns x ALL batch rows (B <= 128), so the per-column batch-norm
// statistics (a reduction over B) never leave the workgroup, and the softmax
// over V is an online (max, sum-exp) per row whose partials are merged by
// row_loss.  The three GEMM-shaped products run on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32, exact fp32 -- the reference is fp32):
//     logits[B, VB]  = theta_d[B, K] @ beta[K, VB]           (forward)
//     dbeta[K, VB]   = theta_d^T[K, B] @ dlogit[B, VB]       (backward, per tile)
//     dtheta_d[B, K] = sum_tiles dlogit[B, VB] @ beta^T[VB, K] (per-tile partials)
//
// Latency discipline (the kernels are tiny, so round trips dominate):
//  * every global read of a kernel is issued in ONE staging round before the
//    first barrier: theta_d and the BN'ed logit tile go through LDS-DMA
//    (global_load_lds_dwordx4), the beta tile through registers;
//  * forward: wave w owns columns [16w, 16w+16) for all rows, so the column
//    batch-norm statistics, the normalisation, the running-stat update and the
//    per-row (max, sum-exp) partials are computed straight from the MFMA
//    accumulators (cross-lane shuffles, no LDS pass, no second barrier);
//  * backward: the x tile is never materialised -- the sparse -x p/(p+1e-10)
//    terms are written into a pre-zeroed dlogit tile, then one register pass
//    adds p*S and applies the BN backward.
//
// The loss never needs the dense [B, V] word distribution: only the CSR
// non-zeros are gathered (row_loss), and the backward needs per row
//   dL/dz_bj = p_bj * S_b - x_bj * p_bj / (p_bj + 1e-10),
//   S_b = sum_{v in nz(b)} x_bv p_bv / (p_bv + 1e-10),
// with p recomputed from the stored BN'ed logits.  row_loss also records where
// each row's non-zeros of every vocab tile start (ws_tstart).
//
// Layouts: ws_thetad is [bmax, kt] (kt = K padded to 4 x odd, zero padding, so
// the MFMA A-operand reads are bank-conflict free); ws_zn is tiled
// [n_tiles][bmax][VB] so a tile is one contiguous LDS-DMA copy; ws_row_part is
// [dec_grid * 4][bmax][2] (one partial per forward wave column strip).
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int DEC_THREADS = 1024;
constexpr int VB = 64;
constexpr int LDB_F = 80;   // fwd beta tile stride: B-role reads (lane -> column) conflict free
// bwd strides, 2 mod 32: the transposed B-role reads of the beta tile (lane -> k row) and
// the A-role reads of dlogit (lane -> row) put 16 rows x 2 columns of a half-wave on 32
// distinct ds_read_b32 banks; so do the dense pass's 16 rows x 2 columns of dlogit
constexpr int LDB_B = 66;
constexpr int LDD = 66;
// BN'ed logit tiles (ws_zn) are stored XOR-swizzled: element (row, col) of a tile at
// row * VB + (col ^ zswz(row)).  The bwd dense pass reads 16 rows x 2 columns per
// half-wave; unswizzled (stride VB = 64) those 16 rows hit ONE bank (16-way conflict),
// swizzled they cover 32 distinct banks.  The tile is LDS-DMA'd verbatim, so the
// swizzle is applied by the writer (prodlda_fwd) and every reader.
__host__ __device__ __forceinline__ int zswz(int row) { return (row & 15) << 1; }
constexpr float RL_EPS = 1e-10f;

__host__ __device__ __forceinline__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

// beta[0:KP, c0:c0+VB] -> bt[KP x ld] (zero for k >= K or column >= V); one
// round of independent loads per 16 elements per thread.
__device__ __forceinline__ void stage_beta_tile(float* bt, int ld, const float* __restrict__ beta,
                                                int K, int KP, int V, int c0, int tid) {
  constexpr int U = 16;
  const int n = KP * VB;
  for (int base = tid; base < n; base += U * DEC_THREADS) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(base + u * DEC_THREADS, n - 1);
      const int k = min(i / VB, K - 1), c = min(c0 + i % VB, V - 1);
      v[u] = beta[(size_t)k * V + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * DEC_THREADS;
      const int k = i / VB, c = i % VB;
      if (i < n) bt[k * ld + c] = (k < K && c0 + c < V) ? v[u] : 0.f;
    }
  }
}

// sum over the 4 lane groups (lanes l, l^16, l^32, l^48): a column reduction
__device__ __forceinline__ float sum_groups(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
}  // namespace

// grid: dec_grid workgroups of 16 waves (persistent: workgroup g owns vocab tiles
// g, g + dec_grid, ...; the usual case is one tile each).  theta_d is staged once per
// workgroup, so large vocabularies do not re-read it per tile, and the per-row
// (max, sum-exp) partials are merged across the workgroup's tiles in registers
// (ws_row_part holds dec_grid * 4 partials per row).  Wave w owns column strip
// cs = w & 3 (16 columns) and row tiles rt = (w >> 2) + 4 i.
// dynamic LDS: th[BM*kt] + bt[KP*LDB_F] + colp[4][64] + colq[4][64] + stat[2][64]
template <int BM>
__global__ void __launch_bounds__(DEC_THREADS) prodlda_fwd_kernel(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, KT = m.kt, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  const int KP = round_up(K, 4);
  float* th = smem;
  float* bt = th + BM * KT;
  float* colp = bt + KP * LDB_F;
  float* colq = colp + 4 * VB;
  constexpr int RT = BM / 16;                 // row tiles
  constexpr int NRT = (RT + 3) / 4;           // row tiles per wave
  const int cs = wave & 3, rt0 = wave >> 2;
  const int col = 16 * cs + (lane & 15);      // this lane's column within a tile
  float rm_[NRT][4], rs_[NRT][4];             // running (max, sum-exp) of this lane's rows
#pragma unroll
  for (int i = 0; i < NRT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) { rm_[i][e] = -INFINITY; rs_[i][e] = 0.f; }

  GFK_STAMP(m, 16);
  glds_copy(th, m.ws_thetad, BM * KT, tid, DEC_THREADS);
  const int nb = *m.ws_nb;
  if (blockIdx.x == 0 && tid == 0) *m.nbt_beta += 1;
#pragma unroll 1
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
  const int c0 = tile * VB;
  // ---- one staging round: beta tile, running stats (theta_d: first iteration) ----
  const int v = c0 + col;
  const bool valid = v < V;
  const float rm0 = m.beta_rm[min(v, V - 1)], rv0 = m.beta_rv[min(v, V - 1)];
  if (tile != (int)blockIdx.x) __syncthreads();     // previous tile's bt / colp reads done
  stage_beta_tile(bt, LDB_F, m.beta, K, KP, V, c0, tid);
  __syncthreads();
  GFK_STAMP(m, 17);
  // ---- logits for this wave's row tiles x 16 columns ----
  f32x4 acc[NRT];
#pragma unroll
  for (int i = 0; i < NRT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const float* bp = bt + (lane >> 4) * LDB_F + col;
    const float* ap = th + (rt0 * 16 + (lane & 15)) * KT + (lane >> 4);
    if (rt0 < RT) {
      for (int k0 = 0; k0 < KP; k0 += 4) {
        const float b = bp[k0 * LDB_F];
#pragma unroll
        for (int i = 0; i < NRT; ++i)
          if (rt0 + 4 * i < RT) acc[i] = mfma16x16x4(ap[i * 64 * KT + k0], b, acc[i]);
      }
    }
  }
  GFK_STAMP(m, 18);

  // ---- column batch-norm: wave partials over its rows, combined through LDS ----
  const float inv_nb = 1.f / (float)nb;
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NRT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = (rt0 + 4 * i) * 16 + (lane >> 4) * 4 + e;
      s += (row < nb && rt0 + 4 * i < RT) ? acc[i][e] : 0.f;
    }
  s = sum_groups(s);
  if (lane < 16) colp[rt0 * VB + col] = s;
  __syncthreads();
  const float mean = (colp[col] + colp[VB + col] + colp[2 * VB + col] + colp[3 * VB + col]) * inv_nb;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NRT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = (rt0 + 4 * i) * 16 + (lane >> 4) * 4 + e;
      const float d = acc[i][e] - mean;
      q += (row < nb && rt0 + 4 * i < RT) ? d * d : 0.f;
    }
  q = sum_groups(q);
  if (lane < 16) colq[rt0 * VB + col] = q;
  __syncthreads();
  const float var = (colq[col] + colq[VB + col] + colq[2 * VB + col] + colq[3 * VB + col]) * inv_nb;
  const float rstd = rsqrtf(var + m.bn_eps);
  if (rt0 == 0 && lane < 16 && valid) {
    const float mom = m.bn_momentum;
    const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
    float nm = (1.f - mom) * rm0 + mom * mean, nv = (1.f - mom) * rv0 + mom * unb;
    if (m.fed_scale_on && is_shared(m, m.beta_rm)) { nm *= m.fed_scale; nv *= m.fed_scale; }
    m.beta_rm[v] = nm;
    m.beta_rv[v] = nv;
    m.ws_col_rstd[v] = rstd;
  }
  GFK_STAMP(m, 19);

  // ---- normalise, store the BN'ed tile, merge the per-row (max, sum-exp) ----
  float* zt = m.ws_zn + (size_t)tile * BM * VB;
#pragma unroll
  for (int i = 0; i < NRT; ++i) {
    if (rt0 + 4 * i >= RT) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = (rt0 + 4 * i) * 16 + (lane >> 4) * 4 + e;
      const float z = (acc[i][e] - mean) * rstd;
      if (row < nb) zt[row * VB + (col ^ zswz(row))] = z;
      const float zv = valid ? z : -INFINITY;
      const float mx = row16_max(zv);
      const float se = row16_sum(valid ? __expf(zv - mx) : 0.f);
      lse_merge(rm_[i][e], rs_[i][e], mx, se);
    }
  }
  GFK_STAMP(m, 20);
  }
  // ---- this workgroup's per-row partials (one per wave column strip) ----
  float* part = m.ws_row_part + (size_t)(blockIdx.x * 4 + cs) * m.bmax * 2;
#pragma unroll
  for (int i = 0; i < NRT; ++i) {
    if (rt0 + 4 * i >= RT) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = (rt0 + 4 * i) * 16 + (lane >> 4) * 4 + e;
      if ((lane & 15) == 0 && row < nb) {
        part[2 * row] = rm_[i][e];
        part[2 * row + 1] = rs_[i][e];
      }
    }
  }
}

// One wave per batch row: log-sum-exp from the per-wave partials, the sparse
// reconstruction loss and S_b over the row's non-zeros (read from the row slots
// prepared with the batch, so the logit gathers are the second round trip).
extern "C" __global__ void __launch_bounds__(64) gfk_prodlda_row_loss(GfkModel m) {
  int n_tiles = m.n_tiles, bmax = m.bmax;
  const int32_t *nbp = m.ws_nb, *erange = m.ws_erange;
  const float *row_part = m.ws_row_part, *zn = m.ws_zn;
  keep(n_tiles, bmax, nbp, erange, row_part, zn);
  const int b = blockIdx.x, lane = threadIdx.x;
  // ---- round 1: batch size, the row's extent, LSE partials, its non-zeros (slots) ----
  const int nb = *nbp;
  const int np = m.dec_grid * 4;                 // per-workgroup partials of prodlda_fwd
  const int e0 = erange[2 * b], e1 = erange[2 * b + 1];
  constexpr int PU = 8, SU = 4;
  float pm[PU], ps[PU];
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int g = min(lane + 64 * u, np - 1);
    const float2 p = *reinterpret_cast<const float2*>(row_part + ((size_t)g * bmax + b) * 2);
    pm[u] = p.x;
    ps[u] = p.y;
  }
  const int cap = m.slot_cap;
  const int32_t* sidx = m.ws_sidx + (size_t)b * cap;
  const float* sval = m.ws_sval + (size_t)b * cap;
  int ci[SU];
  float xv[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int j = min(lane + 64 * u, cap - 1);
    ci[u] = sidx[j];
    xv[u] = sval[j];
  }
  if (b >= nb) return;
  const int n = e1 - e0;
  // ---- round 2: the BN'ed logits at the non-zeros ----
  const size_t tstride = (size_t)bmax * VB;
  const float* zr = zn + (size_t)b * VB;
  float zv[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int c = ci[u];
    zv[u] = lane + 64 * u < n ? zr[(size_t)(c / VB) * tstride + ((c % VB) ^ zswz(b))] : 0.f;
  }
  float mx = -INFINITY, se = 0.f;
#pragma unroll
  for (int u = 0; u < PU; ++u)
    if (lane + 64 * u < np) lse_merge(mx, se, pm[u], ps[u]);
  for (int g = lane + 64 * PU; g < np; g += 64) {
    const float2 p = *reinterpret_cast<const float2*>(row_part + ((size_t)g * bmax + b) * 2);
    lse_merge(mx, se, p.x, p.y);
  }
  wave_lse(mx, se);
  const float lse = mx + logf(se);
  float rl = 0.f, S = 0.f;
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    if (lane + 64 * u >= n) continue;
    const float p = expf(zv[u] - lse);
    rl += xv[u] * logf(p + RL_EPS);
    S += xv[u] * p / (p + RL_EPS);
  }
  for (int j = lane + 64 * SU; j < n; j += 64) {    // rows of more than 256 non-zeros
    const int c = sidx[j];
    const float x = sval[j];
    const float p = expf(zr[(size_t)(c / VB) * tstride + ((c % VB) ^ zswz(b))] - lse);
    rl += x * logf(p + RL_EPS);
    S += x * p / (p + RL_EPS);
  }
  rl = wave_sum(rl);
  S = wave_sum(S);
  if (lane == 0) {
    m.ws_lse[b] = lse;
    m.ws_rl[b] = -rl;
    m.ws_s[b] = S;
  }
}

// Backward.  grid: n_tiles workgroups of 16 waves.
// dynamic LDS: th[BM*kt] + bt[KP16*LDB_B] + zt[BM*VB] + dt[BM*LDD] + lse[BM] + S[BM] + rstd[VB]
// MAXU: dbeta 16x16 output tiles per wave = ceil(K / 64) (Adam state prefetched for
// each; a compile-time count keeps the prefetch in registers)
template <int BM, int MAXU>
__global__ void __launch_bounds__(DEC_THREADS) prodlda_bwd_kernel(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, KT = m.kt, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  const int KP16 = round_up(K, 16);
  const int tile = blockIdx.x, c0 = tile * VB;
  float* th = smem;
  float* bt = th + BM * KT;
  float* zt = bt + KP16 * LDB_B;
  float* dt = zt + BM * VB;
  float* lse = dt + BM * LDD;
  float* Sb = lse + BM;
  float* rs = Sb + BM;
  constexpr int TPR = DEC_THREADS / BM < 16 ? DEC_THREADS / BM : 16;   // threads per row (sparse x)

  GFK_STAMP(m, 24);
  // ---- one staging round ----
  glds_copy(th, m.ws_thetad, BM * KT, tid, DEC_THREADS);
  glds_copy(zt, m.ws_zn + (size_t)tile * BM * VB, BM * VB, tid, DEC_THREADS);
  glds_copy(lse, m.ws_lse, BM, tid, DEC_THREADS);
  glds_copy(Sb, m.ws_s, BM, tid, DEC_THREADS);
  glds_copy(rs, m.ws_col_rstd + c0, VB, tid, DEC_THREADS);
  const int nb = *m.ws_nb;
  // sparse x of this tile: TPR threads per row, the first non-zero prefetched
  const int xrow = tid / TPR, xsub = tid % TPR;
  int xe0 = 0, xe1 = 0;
  if (xrow < BM) {
    const int32_t* ts = m.ws_tstart + (size_t)xrow * (m.n_tiles + 1) + tile;
    xe0 = ts[0];
    xe1 = ts[1];
  }
  const int xe = min(xe0 + xsub, max(xe1 - 1, 0));
  const int xc0 = m.indices[xe];
  const float xv0 = m.values[xe];
  // optimizer state of this lane's dbeta outputs (fused mode): wave -> (k tile, column strip)
  const int ksub = KP16 / 16;
  const int NB_T = ksub * 4;
  const bool fused = m.update_mode == 1;
  float bp_[MAXU][4], bm_[MAXU][4], bv_[MAXU][4];
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int t = wave + 16 * u;
    const int ks = t >> 2, cst = t & 3;
    const int c = min(c0 + cst * 16 + (lane & 15), V - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = min(ks * 16 + (lane >> 4) * 4 + r, K - 1);
      bp_[u][r] = bm_[u][r] = bv_[u][r] = 0.f;
      if (fused && t < NB_T) {
        const float* p = m.beta + (size_t)k * V + c;
        bp_[u][r] = *p;
        bm_[u][r] = p[m.off_m];
        bv_[u][r] = p[m.off_v];
      }
    }
  }
  stage_beta_tile(bt, LDB_B, m.beta, K, KP16, V, c0, tid);
  // zero the dlogit tile (dense-pass layout: column tid>>4, rows (tid&15) + 16 i)
  const int dcol = tid >> 4, dg = tid & 15;
  for (int row = dg; row < BM; row += 16) dt[row * LDD + dcol] = 0.f;
  __syncthreads();
  GFK_STAMP(m, 25);

  // ---- sparse term: dt[b, c] = -x p / (p + 1e-10) at this tile's non-zeros ----
  if (xrow < nb && xrow < BM) {
    const float l = lse[xrow];
    for (int i = 0, e = xe0 + xsub; e < xe1; ++i, e += TPR) {
      const int c = (i == 0 ? xc0 : m.indices[e]) - c0;
      const float x = i == 0 ? xv0 : m.values[e];
      const float p = __expf(zt[xrow * VB + (c ^ zswz(xrow))] - l);
      dt[xrow * LDD + c] = -x * p / (p + RL_EPS);
    }
  }
  __syncthreads();
  GFK_STAMP(m, 26);

  // ---- dense term p*S and the column BN backward: 16 lanes per column ----
  {
    const bool valid = c0 + dcol < V;
    constexpr int NR = BM / 16;
    float d[NR], z[NR];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = dg + 16 * i;
      z[i] = zt[row * VB + (dcol ^ zswz(row))];
      const float p = __expf(z[i] - lse[row]);
      d[i] = (row < nb && valid) ? p * Sb[row] + dt[row * LDD + dcol] : 0.f;
      s1 += d[i];
      s2 += d[i] * z[i];
    }
    s1 = row16_sum(s1) / (float)nb;
    s2 = row16_sum(s2) / (float)nb;
    const float r = valid ? rs[dcol] : 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = dg + 16 * i;
      dt[row * LDD + dcol] = row < nb ? r * (d[i] - s1 - z[i] * s2) : 0.f;
    }
  }
  __syncthreads();
  GFK_STAMP(m, 27);

  // ---- dbeta[k, c] = sum_b th[b, k] dlogit[b, c]  -> update (fused) or gradient ----
  {
    const AdamCoef ac = adam_coef(m);
    const bool sh = is_shared(m, m.beta);
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
      const int t = wave + 16 * u;
      if (t >= NB_T) break;
      const int ks = t >> 2, cst = t & 3;
      const float* ap = th + (lane >> 4) * KT + ks * 16 + (lane & 15);
      const float* bp = dt + (lane >> 4) * LDD + cst * 16 + (lane & 15);
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b0 = 0; b0 < BM; b0 += 8) {
        a0 = mfma16x16x4(ap[b0 * KT], bp[b0 * LDD], a0);
        a1 = mfma16x16x4(ap[(b0 + 4) * KT], bp[(b0 + 4) * LDD], a1);
      }
      const int c = c0 + cst * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = ks * 16 + (lane >> 4) * 4 + e;
        if (k >= K || c >= V) continue;
        float* p = m.beta + (size_t)k * V + c;
        const float g = a0[e] + a1[e];
        if (!fused) {
          p[m.off_g] = g;
        } else {
          float mo = bm_[u][e], vo = bv_[u][e];
          float np = adam_update(bp_[u][e], g, mo, vo, ac);
          if (sh && m.fed_scale_on) np *= m.fed_scale;
          p[m.off_m] = mo;
          p[m.off_v] = vo;
          *p = np;
        }
      }
    }
  }
  // ---- this tile's partial dtheta_d[b, k] = sum_c dlogit[b, c] beta[k, c] (plain stores;
  //      dtheta_reduce sums the n_tiles partials in a fixed order) ----
  {
    float* dpart = m.ws_dthetad + (size_t)tile * m.bmax * K;
    for (int t = wave; t < (BM / 16) * ksub; t += 16) {
      const int rt = t / ksub, ks = t % ksub;
      const float* ap = dt + (rt * 16 + (lane & 15)) * LDD + (lane >> 4);
      const float* bp = bt + (ks * 16 + (lane & 15)) * LDB_B + (lane >> 4);
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < VB; c += 8) {
        a0 = mfma16x16x4(ap[c], bp[c], a0);
        a1 = mfma16x16x4(ap[c + 4], bp[c + 4], a1);
      }
      const int k = ks * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rt * 16 + (lane >> 4) * 4 + e;
        if (row < nb && k < K) dpart[(size_t)row * K + k] = a0[e] + a1[e];
      }
    }
  }
  GFK_STAMP(m, 28);
}

// Backward, persistent variant for large vocabularies (n_tiles > dec_grid): the same
// per-tile work; theta_d, lse and S staged once per workgroup, and the workgroup's
// dtheta_d partial sums its tiles (first tile stores, later tiles add to the same slab,
// each element owned by one lane -- deterministic), so row_bwd reduces dec_grid
// partials instead of n_tiles.
// dynamic LDS: th[BM*kt] + bt[KP16*LDB_B] + zt[BM*VB] + dt[BM*LDD] + lse[BM] + S[BM] + rstd[VB]
// MAXU: dbeta 16x16 output tiles per wave = ceil(K / 64) (Adam state prefetched for
// each; a compile-time count keeps the prefetch in registers)
template <int BM, int MAXU>
__global__ void __launch_bounds__(DEC_THREADS) prodlda_bwd_persist_kernel(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, KT = m.kt, tid0 = threadIdx.x;
  const int KP16 = round_up(K, 16);
  float* th = smem;
  float* bt = th + BM * KT;
  float* zt = bt + KP16 * LDB_B;
  float* dt = zt + BM * VB;
  float* lse = dt + BM * LDD;
  float* Sb = lse + BM;
  float* rs = Sb + BM;
  constexpr int TPR = DEC_THREADS / BM < 16 ? DEC_THREADS / BM : 16;   // threads per row (sparse x)

  glds_copy(th, m.ws_thetad, BM * KT, tid0, DEC_THREADS);
  glds_copy(lse, m.ws_lse, BM, tid0, DEC_THREADS);
  glds_copy(Sb, m.ws_s, BM, tid0, DEC_THREADS);
#pragma unroll 1
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
  // the thread index is made opaque per iteration so the compiler rebuilds the
  // lane-dependent LDS / global addresses inside the loop instead of hoisting them
  // all out of it (which costs ~60 VGPRs and spills)
  int tid = tid0;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = uniform(tid >> 6);
  const int c0 = tile * VB;
  if (tile != (int)blockIdx.x) vm_barrier();   // previous tile: LDS reads and slab stores done
  glds_copy(zt, m.ws_zn + (size_t)tile * BM * VB, BM * VB, tid, DEC_THREADS);
  glds_copy(rs, m.ws_col_rstd + c0, VB, tid, DEC_THREADS);
  const int nb = *m.ws_nb;
  // sparse x of this tile: TPR threads per row, the first non-zero prefetched
  const int xrow = tid / TPR, xsub = tid % TPR;
  int xe0 = 0, xe1 = 0;
  if (xrow < BM) {
    const int32_t* ts = m.ws_tstart + (size_t)xrow * (m.n_tiles + 1) + tile;
    xe0 = ts[0];
    xe1 = ts[1];
  }
  const int xe = min(xe0 + xsub, max(xe1 - 1, 0));
  const int xc0 = m.indices[xe];
  const float xv0 = m.values[xe];
  // optimizer state of this lane's dbeta outputs (fused mode): wave -> (k tile, column strip)
  const int ksub = KP16 / 16;
  const int NB_T = ksub * 4;
  const bool fused = m.update_mode == 1;
  float bp_[MAXU][4], bm_[MAXU][4], bv_[MAXU][4];
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int t = wave + 16 * u;
    const int ks = t >> 2, cst = t & 3;
    const int c = min(c0 + cst * 16 + (lane & 15), V - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = min(ks * 16 + (lane >> 4) * 4 + r, K - 1);
      bp_[u][r] = bm_[u][r] = bv_[u][r] = 0.f;
      if (fused && t < NB_T) {
        const float* p = m.beta + (size_t)k * V + c;
        bp_[u][r] = *p;
        bm_[u][r] = p[m.off_m];
        bv_[u][r] = p[m.off_v];
      }
    }
  }
  stage_beta_tile(bt, LDB_B, m.beta, K, KP16, V, c0, tid);
  // zero the dlogit tile (dense-pass layout: column tid>>4, rows (tid&15) + 16 i)
  const int dcol = tid >> 4, dg = tid & 15;
  for (int row = dg; row < BM; row += 16) dt[row * LDD + dcol] = 0.f;
  __syncthreads();
  GFK_STAMP(m, 25);

  // ---- sparse term: dt[b, c] = -x p / (p + 1e-10) at this tile's non-zeros ----
  if (xrow < nb && xrow < BM) {
    const float l = lse[xrow];
    for (int i = 0, e = xe0 + xsub; e < xe1; ++i, e += TPR) {
      const int c = (i == 0 ? xc0 : m.indices[e]) - c0;
      const float x = i == 0 ? xv0 : m.values[e];
      const float p = __expf(zt[xrow * VB + (c ^ zswz(xrow))] - l);
      dt[xrow * LDD + c] = -x * p / (p + RL_EPS);
    }
  }
  __syncthreads();
  GFK_STAMP(m, 26);

  // ---- dense term p*S and the column BN backward: 16 lanes per column ----
  {
    const bool valid = c0 + dcol < V;
    constexpr int NR = BM / 16;
    float d[NR], z[NR];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = dg + 16 * i;
      z[i] = zt[row * VB + (dcol ^ zswz(row))];
      const float p = __expf(z[i] - lse[row]);
      d[i] = (row < nb && valid) ? p * Sb[row] + dt[row * LDD + dcol] : 0.f;
      s1 += d[i];
      s2 += d[i] * z[i];
    }
    s1 = row16_sum(s1) / (float)nb;
    s2 = row16_sum(s2) / (float)nb;
    const float r = valid ? rs[dcol] : 0.f;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = dg + 16 * i;
      dt[row * LDD + dcol] = row < nb ? r * (d[i] - s1 - z[i] * s2) : 0.f;
    }
  }
  __syncthreads();
  GFK_STAMP(m, 27);

  // ---- dbeta[k, c] = sum_b th[b, k] dlogit[b, c]  -> update (fused) or gradient ----
  {
    const AdamCoef ac = adam_coef(m);
    const bool sh = is_shared(m, m.beta);
#pragma unroll
    for (int u = 0; u < MAXU; ++u) {
      const int t = wave + 16 * u;
      if (t >= NB_T) break;
      const int ks = t >> 2, cst = t & 3;
      const float* ap = th + (lane >> 4) * KT + ks * 16 + (lane & 15);
      const float* bp = dt + (lane >> 4) * LDD + cst * 16 + (lane & 15);
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b0 = 0; b0 < BM; b0 += 8) {
        a0 = mfma16x16x4(ap[b0 * KT], bp[b0 * LDD], a0);
        a1 = mfma16x16x4(ap[(b0 + 4) * KT], bp[(b0 + 4) * LDD], a1);
      }
      const int c = c0 + cst * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = ks * 16 + (lane >> 4) * 4 + e;
        if (k >= K || c >= V) continue;
        float* p = m.beta + (size_t)k * V + c;
        const float g = a0[e] + a1[e];
        if (!fused) {
          p[m.off_g] = g;
        } else {
          float mo = bm_[u][e], vo = bv_[u][e];
          float np = adam_update(bp_[u][e], g, mo, vo, ac);
          if (sh && m.fed_scale_on) np *= m.fed_scale;
          p[m.off_m] = mo;
          p[m.off_v] = vo;
          *p = np;
        }
      }
    }
  }
  // ---- this tile's partial dtheta_d[b, k] = sum_c dlogit[b, c] beta[k, c] (plain stores;
  //      dtheta_reduce sums the n_tiles partials in a fixed order) ----
  {
    const bool first = tile == (int)blockIdx.x;
    float* dpart = m.ws_dthetad + (size_t)blockIdx.x * m.bmax * K;
    for (int t = wave; t < (BM / 16) * ksub; t += 16) {
      const int rt = t / ksub, ks = t % ksub;
      const float* ap = dt + (rt * 16 + (lane & 15)) * LDD + (lane >> 4);
      const float* bp = bt + (ks * 16 + (lane & 15)) * LDB_B + (lane >> 4);
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < VB; c += 8) {
        a0 = mfma16x16x4(ap[c], bp[c], a0);
        a1 = mfma16x16x4(ap[c + 4], bp[c + 4], a1);
      }
      const int k = ks * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rt * 16 + (lane >> 4) * 4 + e;
        if (row < nb && k < K) {
          float* q = dpart + (size_t)row * K + k;
          *q = first ? a0[e] + a1[e] : *q + (a0[e] + a1[e]);
        }
      }
    }
  }
  }
}

extern "C" size_t gfk_prodlda_fwd_smem(const GfkModel* m) {
  const size_t KP = round_up(m->K, 4);
  return sizeof(float) * ((size_t)m->bmax * m->kt + KP * LDB_F + 8 * VB);
}

extern "C" size_t gfk_prodlda_bwd_smem(const GfkModel* m) {
  const size_t KP16 = round_up(m->K, 16), B = m->bmax;
  return sizeof(float) * (B * m->kt + KP16 * LDB_B + B * VB + B * LDD + 2 * B + VB);
}

extern "C" int gfk_launch_prodlda_fwd(const GfkModel* m, hipStream_t s) {
  const size_t sm = gfk_prodlda_fwd_smem(m);
  dim3 g(m->dec_grid), blk(DEC_THREADS);
  switch (m->bmax) {
    case 16: hipLaunchKernelGGL(prodlda_fwd_kernel<16>, g, blk, sm, s, *m); break;
    case 32: hipLaunchKernelGGL(prodlda_fwd_kernel<32>, g, blk, sm, s, *m); break;
    case 64: hipLaunchKernelGGL(prodlda_fwd_kernel<64>, g, blk, sm, s, *m); break;
    case 128: hipLaunchKernelGGL(prodlda_fwd_kernel<128>, g, blk, sm, s, *m); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

template <int MAXU>
static void launch_bwd(const GfkModel* m, dim3 g, dim3 blk, size_t sm, hipStream_t s) {
  if (m->n_dpart < m->n_tiles) {         // persistent: dec_grid workgroups, dec_grid partials
    g = dim3(m->n_dpart);
    switch (m->bmax) {
      case 16: hipLaunchKernelGGL((prodlda_bwd_persist_kernel<16, MAXU>), g, blk, sm, s, *m); break;
      case 32: hipLaunchKernelGGL((prodlda_bwd_persist_kernel<32, MAXU>), g, blk, sm, s, *m); break;
      case 64: hipLaunchKernelGGL((prodlda_bwd_persist_kernel<64, MAXU>), g, blk, sm, s, *m); break;
      default: hipLaunchKernelGGL((prodlda_bwd_persist_kernel<128, MAXU>), g, blk, sm, s, *m); break;
    }
    return;
  }
  switch (m->bmax) {
    case 16: hipLaunchKernelGGL((prodlda_bwd_kernel<16, MAXU>), g, blk, sm, s, *m); break;
    case 32: hipLaunchKernelGGL((prodlda_bwd_kernel<32, MAXU>), g, blk, sm, s, *m); break;
    case 64: hipLaunchKernelGGL((prodlda_bwd_kernel<64, MAXU>), g, blk, sm, s, *m); break;
    default: hipLaunchKernelGGL((prodlda_bwd_kernel<128, MAXU>), g, blk, sm, s, *m); break;
  }
}

extern "C" int gfk_launch_prodlda_bwd(const GfkModel* m, hipStream_t s) {
  const size_t sm = gfk_prodlda_bwd_smem(m);
  dim3 g(m->n_tiles), blk(DEC_THREADS);          // one vocab tile per workgroup
  if (m->bmax != 16 && m->bmax != 32 && m->bmax != 64 && m->bmax != 128) return -1;
  switch ((m->K + 63) / 64) {
    case 1: launch_bwd<1>(m, g, blk, sm, s); break;
    case 2: launch_bwd<2>(m, g, blk, sm, s); break;
    case 3: launch_bwd<3>(m, g, blk, sm, s); break;
    default: launch_bwd<4>(m, g, blk, sm, s); break;
  }
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_prodlda_row_loss(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_prodlda_row_loss, dim3(m->bmax), dim3(64), 0, s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_prodlda_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)prodlda_fwd_kernel<16>, (const void*)prodlda_fwd_kernel<32>,
                      (const void*)prodlda_fwd_kernel<64>, (const void*)prodlda_fwd_kernel<128>,
#define GFK_BWD_PTRS(U) (const void*)prodlda_bwd_kernel<16, U>, (const void*)prodlda_bwd_kernel<32, U>, \
    (const void*)prodlda_bwd_kernel<64, U>, (const void*)prodlda_bwd_kernel<128, U>, \
    (const void*)prodlda_bwd_persist_kernel<16, U>, (const void*)prodlda_bwd_persist_kernel<32, U>, \
    (const void*)prodlda_bwd_persist_kernel<64, U>, (const void*)prodlda_bwd_persist_kernel<128, U>
                      GFK_BWD_PTRS(1), GFK_BWD_PTRS(2), GFK_BWD_PTRS(3), GFK_BWD_PTRS(4)};
#undef GFK_BWD_PTRS
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
