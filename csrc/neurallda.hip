// NeuralLDA decoder: beta_sm = softmax_V(BN_K(beta)), word_dist = theta_d @ beta_sm,
// loss -sum x log(word_dist + 1e-10), and the backward.
//
// Reference math: decoder_network.py:127-132 (BatchNorm1d(V) applied to beta
// [K, V]: the "batch" axis is the K topics), avitm.py:225.
//
// MI355X design: the dense [K, V] part (BN over topics, softmax over V and
// their backward) is vocab-tiled across workgroups; the [B, V] word
// distribution is never materialised -- the loss only needs it at the CSR
// non-zeros, so each document gathers the K-vectors beta_sm[:, v] of its own
// tokens (stored transposed, [V, K], one contiguous 4K-byte row per token).
// The softmax-over-V backward needs c_k = sum_v beta_sm[k,v] dbeta_sm[k,v],
// which equals sum_b theta_d[b,k] dtheta_d[b,k] and is computed from the tiny
// [B, K] tensors in lda_beta_bwd's prologue instead of a V-wide reduction.
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int VB = 64;
constexpr int LD = VB + 1;
constexpr float RL_EPS = 1e-10f;
}  // namespace

// grid: dec_grid workgroups over the vocab tiles, 16 waves each.  Per tile: ONE round
// of independent loads (the beta tile into registers, this lane's column running
// statistics), then BN over the topics (16 lanes per column), the transposed store
// beta_bn^T [V, K], and the per-topic online (max, sum-exp) over the tile's columns.
// dynamic LDS: bn[K*LD] + rowm[K] + rows[K]
constexpr int LBT = 1024;
constexpr int LBW = LBT / 64;

// KM: the largest K compiled in (the beta tile's registers); the K <= 64 instance fits 64
// VGPRs, so two workgroups share a CU (a batched launch of M clients' tiles in fewer rounds)
template <bool GB = false, int KM = 256>
__global__ void __launch_bounds__(LBT) __attribute__((amdgpu_waves_per_eu(KM <= 64 ? 8 : 1)))
gfk_lda_beta_fwd(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, tid = threadIdx.x;
  float* bn = smem;
  float* rowm = bn + K * LD;
  float* rows = rowm + K;
  for (int k = tid; k < K; k += LBT) { rowm[k] = -INFINITY; rows[k] = 0.f; }
  if (gfk_bx() == 0 && tid == 0) *m.nbt_beta += 1;
  constexpr int BU = (KM * VB + LBT - 1) / LBT;       // K <= KM
  const int c = tid >> 4, sub = tid & 15;             // BN: 16 lanes per column
  for (int tile = gfk_bx(); tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB, nv = min(VB, V - c0);
    const bool valid = c < nv;
    __syncthreads();
    float bv[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
      const int i = tid + LBT * u, k = i / VB, cc = i % VB;
      bv[u] = (i < K * VB && cc < nv) ? m.beta[(size_t)k * m.ldb + c0 + cc] : 0.f;
    }
    float rm0 = 0.f, rv0 = 0.f;
    if (sub == 0 && valid) { rm0 = m.beta_rm[c0 + c]; rv0 = m.beta_rv[c0 + c]; }
#pragma unroll
    for (int u = 0; u < BU; ++u) {
      const int i = tid + LBT * u;
      if (i < K * VB) bn[(i / VB) * LD + i % VB] = bv[u];
    }
    lds_barrier();
    {  // BN over the K topics of each column
      float s = 0.f;
      for (int k = sub; k < K; k += 16) s += bn[k * LD + c];
      const float mean = row16_sum(s) / (float)K;
      float q = 0.f;
      for (int k = sub; k < K; k += 16) { const float d = bn[k * LD + c] - mean; q += d * d; }
      const float var = row16_sum(q) / (float)K;
      const float rstd = rsqrtf(var + m.bn_eps);
      for (int k = sub; k < K; k += 16) {
        const int i = k * LD + c;
        bn[i] = valid ? (bn[i] - mean) * rstd : -INFINITY;
      }
      if (sub == 0 && valid) {
        const int v = c0 + c;
        const float mom = m.bn_momentum;
        const float unb = K > 1 ? var * (float)K / (float)(K - 1) : var;
        float nm = (1.f - mom) * rm0 + mom * mean, nv2 = (1.f - mom) * rv0 + mom * unb;
        if (m.fed_scale_on && is_shared(m, m.beta_rm)) { nm *= m.fed_scale; nv2 *= m.fed_scale; }
        m.beta_rm[v] = nm;
        m.beta_rv[v] = nv2;
        m.ws_col_rstd[v] = rstd;
      }
    }
    lds_barrier();
    // transposed store bn^T [V, K] (contiguous K-vector per token)
    for (int i = tid; i < K * VB; i += LBT) {
      const int cc = i / K, k = i % K;
      if (cc < nv) m.ws_zn[(size_t)(c0 + cc) * K + k] = bn[k * LD + cc];
    }
    // online (max, sum exp) over this tile for every topic row: 16 lanes per row
    for (int k = tid >> 4; k < K; k += LBT / 16) {
      const float* row = bn + k * LD + 4 * sub;
      float mx = fmaxf(fmaxf(row[0], row[1]), fmaxf(row[2], row[3]));
      mx = row16_max(mx);
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) se += __expf(row[j] - mx);
      se = row16_sum(se);
      if (sub == 0) {
        float rm = rowm[k], rs = rows[k];
        lse_merge(rm, rs, mx, se);
        rowm[k] = rm;
        rows[k] = rs;
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < K; k += LBT) {
    float* p = m.ws_row_part + ((size_t)gfk_bx() * K + k) * 2;
    p[0] = rowm[k];
    p[1] = rows[k];
  }
}

// One workgroup (16 waves) per document: the sparse loss, d theta_d, and the
// coefficient g = -x / (wd + 1e-10) of every non-zero (ws_dbsm, indexed by CSR
// position).  d beta_sm^T[v, k] = sum_b theta_d[b, k] g[b, v] is formed later by
// lda_beta_bwd as an MFMA product per vocab tile -- deterministic, no atomics.
// Each wave takes U non-zeros per round so their gathers are in flight together.
// dynamic LDS: dth[16*K] + rls[16]
constexpr int LDA_ROW_THREADS = 1024;
constexpr int LDA_ROW_WAVES = LDA_ROW_THREADS / 64;

template <int KQ, bool GB = false>
__global__ void __launch_bounds__(LDA_ROW_THREADS) gfk_lda_row_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = gfk_bx(), nb = *m.ws_nb;
  if (b >= nb) return;
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  // matmul_dtype = "bf16": theta_d and beta_sm are bf16 operands of word_dist = theta_d
  // beta_sm and of d theta_d = g beta_sm^T (fp32 accumulation)
  const bool bfo = m.mm_bf16;
  float* dth = smem;
  float* rls = dth + LDA_ROW_WAVES * K;
  float th[KQ], ls[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = lane + 64 * q;
    th[q] = k < K ? m.ws_thetad[(size_t)b * m.kt + k] : 0.f;
    if (bfo) th[q] = bf16_round(th[q]);
    ls[q] = k < K ? m.ws_lse[k] : 0.f;
  }
  const int e0 = m.ws_erange[2 * b], e1 = m.ws_erange[2 * b + 1];
  constexpr int U = 4;
  float acc[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) acc[q] = 0.f;
  float rl = 0.f;
  for (int e = e0 + wave; e < e1; e += LDA_ROW_WAVES * U) {
    int v[U];
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ee = min(e + LDA_ROW_WAVES * u, e1 - 1);
      v[u] = m.indices[ee];
      x[u] = e + LDA_ROW_WAVES * u < e1 ? m.values[ee] : 0.f;
    }
    float z[U][KQ];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        z[u][q] = m.ws_zn[(size_t)v[u] * K + min(lane + 64 * q, K - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ee = e + LDA_ROW_WAVES * u;
      float bs[KQ], wd = 0.f;
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        bs[q] = lane + 64 * q < K ? __expf(z[u][q] - ls[q]) : 0.f;
        if (bfo) bs[q] = bf16_round(bs[q]);
        wd += th[q] * bs[q];
      }
      wd = wave_sum(wd);
      if (ee < e1) {                       // wave-uniform
        const float g = -x[u] / (wd + RL_EPS);
        rl += x[u] * logf(wd + RL_EPS);
#pragma unroll
        for (int q = 0; q < KQ; ++q) acc[q] += g * bs[q];
        if (lane == 0) m.ws_dbsm[ee] = g;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = lane + 64 * q;
    if (k < K) dth[wave * K + k] = acc[q];
  }
  if (lane == 0) rls[wave] = rl;
  __syncthreads();
  for (int k = tid; k < K; k += LDA_ROW_THREADS) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < LDA_ROW_WAVES; ++w) s += dth[w * K + k];
    m.ws_dthetad[(size_t)b * K + k] = s;
  }
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < LDA_ROW_WAVES; ++w) s += rls[w];
    m.ws_rl[b] = -s;
  }
}

// grid: dec_grid workgroups over vocab tiles.  Per tile: d beta_sm^T = G^T theta_d
// on the matrix cores (G = the tile's [64 x B] non-zero coefficients, built in LDS
// from the per-row CSR tile table), then the softmax-over-V backward and the
// BN-over-K backward.  ThLds: theta_d staged in LDS (K up to ~128), else read from L2.
// dynamic LDS: bn[K*LD] + d[K*LD] + xt[64*XS] (+ thd[B*kt + 64]) + ck[pad4(K)] (+ dth[B*K])
// x^T tile stride: 2 x odd, so the A-role MFMA reads (16 rows x 2 k per half-wave)
// hit 32 distinct ds_read_b32 banks
constexpr int LDA_XB = 128;            // rows of the x^T tile (larger batches: chunks)
__host__ __device__ inline int lda_xs(int B) {
  int s = (B + 1) & ~1;
  if ((s / 2) % 2 == 0) s += 2;
  return s;
}

// 16 waves; one vocab tile per workgroup per iteration.  Every global read of the
// iteration is issued in ONE round before the first barrier: theta_d, d theta_d and
// the tile's BN'ed beta^T rows [64][K] (LDS-DMA; the tile lands in d's storage and is
// transposed LDS -> LDS), the rows' CSR extents in the tile, and the Adam state of the
// outputs this thread updates (fused mode).  Second round: the tile's per-non-zero
// coefficients (ws_dbsm).  Then c_k, the x^T theta_d MFMA, the BN backward over the
// topics and the update, all out of LDS.
// CH (the large-batch plan, bmax > 128): the x^T tile built and multiplied in row chunks
template <bool ThLds, bool GB = false, bool CH = false>
__global__ void __launch_bounds__(LBT) gfk_lda_beta_bwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  // the x^T tile holds XB = min(bmax, 128) rows: larger batches take it in row chunks,
  // the G accumulators carrying over (one chunk, and the same summation order, up to 128)
  const int B = m.bmax, kt = m.kt, XB = B < LDA_XB ? B : LDA_XB, XS = lda_xs(XB), nb = *m.ws_nb;
  const int nch = (B + XB - 1) / XB;
  float* bn = smem;
  float* d = bn + ((K * LD + 3) & ~3);
  float* xt = d + ((K * LD + 3) & ~3);      // 16-B aligned: thd / dtl are LDS-DMA destinations
  float* thd = xt + VB * XS;
  float* ckl = thd + (ThLds ? B * kt + 64 : 0);
  float* dtl = ckl + ((K + 3) & ~3);                 // staged d theta_d [B][K] (ThLds)
  float* lsl = dtl + (ThLds ? ((B * K + 3) & ~3) : 0);   // per-topic log-sum-exp [K]
  if (ThLds) {                                        // LDS-DMA: theta_d and d theta_d
    glds_copy(thd, m.ws_thetad, B * kt, tid, LBT);
    glds_copy(dtl, m.ws_dtheta, B * K, tid, LBT);
    for (int i = tid; i < 64; i += LBT) thd[B * kt + i] = 0.f;
  }
  glds_copy(lsl, m.ws_lse, K, tid, LBT);
  const float* thv = ThLds ? thd : m.ws_thetad;
  const float* dtv = ThLds ? dtl : m.ws_dtheta;
  const int NT = (K + 15) / 16;
  const bool fused = m.update_mode == 1;
  constexpr int PU = 4;                               // prefetched updates per thread (K <= 64)
  const int n_upd = (K * VB + LBT - 1) / LBT;
  for (int tile = gfk_bx(); tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB, nv = min(VB, V - c0);
    __syncthreads();
    // ---- round 1 ----
    glds_copy(d, m.ws_zn + (size_t)c0 * K, nv * K, tid, LBT);
    // 16 threads per batch row: rows tid/16 and, at bmax >= 128, tid/16 + 64 (of the chunk)
    const int xrow = tid >> 4, xsub = tid & 15, xrow2 = xrow + LBT / 16;
    int es = 0, ee = 0, fs = 0, fe = 0;
    if (xrow < nb && xrow < XB) {
      const int32_t* ts = m.ws_tstart + (size_t)xrow * (m.n_tiles + 1) + tile;
      es = ts[0];
      ee = ts[1];
    }
    if (xrow2 < nb && xrow2 < XB) {
      const int32_t* ts = m.ws_tstart + (size_t)xrow2 * (m.n_tiles + 1) + tile;
      fs = ts[0];
      fe = ts[1];
    }
    float pp[PU], pm[PU], pv[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      pp[u] = pm[u] = pv[u] = 0.f;
      const int i = tid + LBT * u, k = i / VB, c = i % VB;
      if (fused && u < n_upd && k < K && c < nv) {
        const float* p = m.beta + (size_t)k * m.ldb + c0 + c;
        pp[u] = *p;
        pm[u] = p[m.off_m];
        pv[u] = p[m.off_v];
      }
    }
    for (int i = tid; i < VB * XS; i += LBT) xt[i] = 0.f;
    vm_barrier();
    // ---- round 2: the tile's non-zero coefficients g = -x / (wd + eps) -> x^T tile ----
    for (int e = es + xsub; e < ee; e += 16) xt[(m.indices[e] - c0) * XS + xrow] = m.ws_dbsm[e];
    for (int e = fs + xsub; e < fe; e += 16) xt[(m.indices[e] - c0) * XS + xrow2] = m.ws_dbsm[e];
    // c_k = sum_b theta_d[b, k] d theta_d[b, k] (softmax-over-V backward), 16 lanes per topic
    if (tile == (int)gfk_bx()) {
      for (int k0 = 0; k0 < K; k0 += LBT / 16) {
        const int k = k0 + (tid >> 4), sub = tid & 15;
        float s = 0.f;
        if (k < K)
          for (int r = sub; r < nb; r += 16) s += thv[r * kt + k] * dtv[r * K + k];
        s = row16_sum(s);
        if (sub == 0 && k < K) ckl[k] = s;
      }
    }
    // the BN'ed beta^T rows (in d's storage) -> bn [K][LD]
    float zr[(VB * 256 + LBT - 1) / LBT];             // K <= 256
    {
      int u = 0;
      for (int i = tid; i < K * VB; i += LBT, ++u) {
        const int c = i / K, k = i % K;
        zr[u] = c < nv ? d[c * K + k] : 0.f;
      }
    }
    lds_barrier();
    {
      int u = 0;
      for (int i = tid; i < K * VB; i += LBT, ++u) {
        const int c = i / K, k = i % K;
        bn[k * LD + c] = zr[u];
        d[k * LD + c] = c < nv ? __expf(zr[u] - lsl[k]) : 0.f;   // beta_sm
      }
    }
    lds_barrier();
    if constexpr (!CH) {
    // G[c][k] = sum_b xt[c][b] theta_d[b][k]; then d <- beta_sm * (G - c_k)
    for (int t = wave; t < 4 * NT; t += LBW) {
      const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
      const float* ap = xt + (i0 + (lane & 15)) * XS + (lane >> 4);
      const float* bp = thv + (lane >> 4) * kt + j0 + (lane & 15);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (m.mm_bf16)        // bf16 operands (the coefficients and theta_d), fp32 accumulation
        for (int kb = 0; kb < B; kb += 4) acc = mfma16x16x4(bf16_round(ap[kb]), bf16_round(bp[kb * kt]), acc);
      else
        for (int kb = 0; kb < B; kb += 4) acc = mfma16x16x4(ap[kb], bp[kb * kt], acc);
      const int k = j0 + (lane & 15);
      if (k < K) {
        const float ck = ckl[k];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = i0 + (lane >> 4) * 4 + r;
          d[k * LD + c] = d[k * LD + c] * (acc[r] - ck);
        }
      }
    }
    } else {
    // G[c][k] = sum_b xt[c][b] theta_d[b][k] (x^T chunk by chunk); then d <- beta_sm (G - c_k)
    constexpr int TW = (4 * 16 + LBW - 1) / LBW;       // subtiles per wave (K <= 256)
    f32x4 acc[TW];
#pragma unroll
    for (int u = 0; u < TW; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
      const int b0 = ch * XB, cb = min(XB, B - b0);
      if (ch > 0) {                     // the next chunk's coefficients into the x^T tile
        lds_barrier();                  // (the previous chunk's MFMA reads are done)
        for (int i = tid; i < VB * XS; i += LBT) xt[i] = 0.f;
        int s0 = 0, s1 = 0, t0 = 0, t1 = 0;
        if (b0 + xrow < nb && xrow < cb) {
          const int32_t* ts = m.ws_tstart + (size_t)(b0 + xrow) * (m.n_tiles + 1) + tile;
          s0 = ts[0];
          s1 = ts[1];
        }
        if (b0 + xrow2 < nb && xrow2 < cb) {
          const int32_t* ts = m.ws_tstart + (size_t)(b0 + xrow2) * (m.n_tiles + 1) + tile;
          t0 = ts[0];
          t1 = ts[1];
        }
        lds_barrier();
        for (int e = s0 + xsub; e < s1; e += 16) xt[(m.indices[e] - c0) * XS + xrow] = m.ws_dbsm[e];
        for (int e = t0 + xsub; e < t1; e += 16) xt[(m.indices[e] - c0) * XS + xrow2] = m.ws_dbsm[e];
        lds_barrier();
      }
#pragma unroll
      for (int u = 0; u < TW; ++u) {
        const int t = wave + LBW * u;
        if (t >= 4 * NT) break;
        const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
        const float* ap = xt + (i0 + (lane & 15)) * XS + (lane >> 4);
        const float* bp = thv + (size_t)(b0 + (lane >> 4)) * kt + j0 + (lane & 15);
        if (m.mm_bf16)      // bf16 operands (the coefficients and theta_d), fp32 accumulation
          for (int kb = 0; kb < cb; kb += 4) acc[u] = mfma16x16x4(bf16_round(ap[kb]), bf16_round(bp[kb * kt]), acc[u]);
        else
          for (int kb = 0; kb < cb; kb += 4) acc[u] = mfma16x16x4(ap[kb], bp[kb * kt], acc[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      const int t = wave + LBW * u;
      if (t >= 4 * NT) break;
      const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
      const int k = j0 + (lane & 15);
      if (k < K) {
        const float ck = ckl[k];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = i0 + (lane >> 4) * 4 + r;
          d[k * LD + c] = d[k * LD + c] * (acc[u][r] - ck);
        }
      }
    }
    }
    lds_barrier();
    {  // BN backward over the K topics of each column: 16 lanes per column
      const int c = tid >> 4, sub = tid & 15;
      float s1 = 0.f, s2 = 0.f;
      for (int k = sub; k < K; k += 16) {
        const float g = d[k * LD + c];
        s1 += g;
        s2 += g * bn[k * LD + c];
      }
      s1 = row16_sum(s1);
      s2 = row16_sum(s2);
      const float inv = 1.f / (float)K;
      if (c < nv) {
        const float rstd = m.ws_col_rstd[c0 + c];
        for (int k = sub; k < K; k += 16) {
          const int i = k * LD + c;
          d[i] = rstd * (d[i] - s1 * inv - bn[i] * s2 * inv);
        }
      }
    }
    lds_barrier();
    // gradient (gradient mode) or Adam + FedAvg pre-scale in place (fused mode)
    const AdamCoef ac = adam_coef(m);
    const bool sh = is_shared(m, m.beta);
    {
      int u = 0;
      for (int i = tid; i < K * VB; i += LBT, ++u) {
        const int k = i / VB, c = i % VB;
        if (c >= nv) continue;
        float* p = m.beta + (size_t)k * m.ldb + c0 + c;
        const float g = d[k * LD + c];
        if (!fused) {
          p[m.off_g] = g;
        } else if (u < PU) {
          float mo = pm[u], vo = pv[u];
          float np = adam_update(pp[u], g, mo, vo, ac);
          if (sh && m.fed_scale_on) np *= m.fed_scale;
          p[m.off_m] = mo;
          p[m.off_v] = vo;
          *p = np;
        } else {
          param_update(m, p, g, ac, sh);
        }
      }
    }
  }
}

extern "C" size_t gfk_lda_fwd_smem(int K) { return sizeof(float) * ((size_t)K * LD + 2 * K); }
extern "C" size_t gfk_lda_row_smem(int K) {
  return sizeof(float) * ((size_t)K * LDA_ROW_WAVES + LDA_ROW_WAVES);
}
static size_t lda_bwd_floats(const GfkModel* m, bool th_lds) {
  const int xb = m->bmax < LDA_XB ? m->bmax : LDA_XB;
  size_t n = ((((size_t)m->K * LD) + 3) & ~(size_t)3) * 2 + (size_t)VB * lda_xs(xb) +
             (((size_t)m->K + 3) & ~(size_t)3);
  if (th_lds) n += (size_t)m->bmax * m->kt + 64 + (((size_t)m->bmax * m->K + 3) & ~(size_t)3);
  return n + (((size_t)m->K + 3) & ~(size_t)3);     // per-topic log-sum-exp
}
static bool lda_bwd_th_lds(const GfkModel* m) {
  return m->bmax <= LDA_XB && sizeof(float) * lda_bwd_floats(m, true) <= 160 * 1024;
}
extern "C" size_t gfk_lda_bwd_smem(const GfkModel* m) {
  return sizeof(float) * lda_bwd_floats(m, lda_bwd_th_lds(m));
}

extern "C" int gfk_launch_lda_beta_fwd(const GfkModel* m, hipStream_t s) {
  if (m->K <= 64)
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_beta_fwd<true, 64>), gfk_grid(dim3(m->dec_grid), m), dim3(LBT), gfk_lda_fwd_smem(m->K), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_beta_fwd<false, 64>), dim3(m->dec_grid), dim3(LBT), gfk_lda_fwd_smem(m->K), s, GfkArgT<false>{*m}); } while (0);
  else
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_beta_fwd<true>), gfk_grid(dim3(m->dec_grid), m), dim3(LBT), gfk_lda_fwd_smem(m->K), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_beta_fwd<false>), dim3(m->dec_grid), dim3(LBT), gfk_lda_fwd_smem(m->K), s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_lda_row(const GfkModel* m, hipStream_t s) {
  const dim3 g(m->bmax), t(LDA_ROW_THREADS);
  const size_t sm = gfk_lda_row_smem(m->K);
  const int kq = (m->K + 63) / 64;
  if (kq <= 1) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_row_k<1, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_row_k<1, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else if (kq == 2) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_row_k<2, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_row_k<2, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else if (kq == 3) do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_row_k<3, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_row_k<3, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  else do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_row_k<4, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_row_k<4, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_lda_beta_bwd(const GfkModel* m, hipStream_t s) {
  const dim3 g(m->dec_grid), t(LBT);
  if (m->bmax > LDA_XB)
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_beta_bwd_k<false, true, true>), gfk_grid(g, m), t, gfk_lda_bwd_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_beta_bwd_k<false, false, true>), g, t, gfk_lda_bwd_smem(m), s, GfkArgT<false>{*m}); } while (0);
  else if (lda_bwd_th_lds(m))
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_beta_bwd_k<true, true>), gfk_grid(g, m), t, gfk_lda_bwd_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_beta_bwd_k<true, false>), g, t, gfk_lda_bwd_smem(m), s, GfkArgT<false>{*m}); } while (0);
  else
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_lda_beta_bwd_k<false, true>), gfk_grid(g, m), t, gfk_lda_bwd_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_lda_beta_bwd_k<false, false>), g, t, gfk_lda_bwd_smem(m), s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_lda_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)gfk_lda_beta_fwd<false>, (const void*)gfk_lda_beta_fwd<true>,
                      (const void*)gfk_lda_beta_fwd<false, 64>, (const void*)gfk_lda_beta_fwd<true, 64>, (const void*)gfk_lda_beta_bwd_k<true>, (const void*)gfk_lda_beta_bwd_k<true, true>,
                      (const void*)gfk_lda_beta_bwd_k<false>, (const void*)gfk_lda_beta_bwd_k<false, true>,
                      (const void*)gfk_lda_beta_bwd_k<false, false, true>, (const void*)gfk_lda_beta_bwd_k<false, true, true>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
