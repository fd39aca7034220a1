// ProdLDA decoder: word_dist = softmax_V(BN_batch(theta_d @ beta)), its
// reconstruction loss -sum x log(word_dist + 1e-10), and the backward.
//
// Reference math: decoder_network.py:121-126, avitm.py:225.
//
// Tiling (MI355X-first): a workgroup (4 waves) owns a vocabulary tile of VB=64
// columns x ALL batch rows (B <= 128), so the per-column batch-norm statistics
// (a reduction over B) stay inside the tile; the softmax over V is an online
// (max, sum-exp) per row across tiles.  The three GEMM-shaped products run on
// the fp32 matrix cores (v_mfma_f32_16x16x4_f32, exact fp32 -- the reference is
// fp32, so no bf16 here):
//     logits[B, VB]  = theta_d[B, K] @ beta[K, VB]           (forward)
//     dbeta[K, VB]   = theta_d^T[K, B] @ dlogit[B, VB]       (backward, per tile)
//     dtheta_d[B, K] += dlogit[B, VB] @ beta^T[VB, K]        (backward, across tiles)
// with 16x16 output sub-tiles distributed over the 4 waves.  LDS row strides are
// padded by one word so the MFMA operand reads are bank-conflict free.
//
// The loss never needs the dense [B, V] word distribution: only the CSR
// non-zeros are gathered (row_loss), and the backward needs per row
//   dL/dz_bj = p_bj * S_b - x_bj * p_bj / (p_bj + 1e-10),
//   S_b = sum_{v in nz(b)} x_bv p_bv / (p_bv + 1e-10),
// with p recomputed from the stored BN'ed logits.  row_loss also records where
// each row's non-zeros of every vocab tile start (ws_tstart), so the backward
// fills its x tile with two loads per row instead of a binary search.
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int DEC_THREADS = 256;
constexpr int VB = 64;
constexpr int LDB = VB + 1;        // padded row stride of the beta / dlogit / logit tiles
constexpr float RL_EPS = 1e-10f;

__host__ __device__ __forceinline__ int round_up(int x, int m) { return (x + m - 1) / m * m; }

// Stage beta[:, c0:c0+VB] (rows < K, columns < V; zero elsewhere) into bt[KP x LDB].
__device__ __forceinline__ void stage_beta_tile(float* bt, const float* __restrict__ beta, int K,
                                                int KP, int V, int c0, int tid) {
  constexpr int U = 8;
  const int n = KP * VB;
  for (int base = tid; base < n; base += U * DEC_THREADS) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * DEC_THREADS;
      const int k = min(i / VB, K - 1), c = min(c0 + i % VB, V - 1);
      v[u] = beta[(size_t)k * V + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * DEC_THREADS;
      const int k = i / VB, c = i % VB;
      if (i < n) bt[k * LDB + c] = (k < K && c0 + c < V) ? v[u] : 0.f;
    }
  }
}

// Stage theta_d[nb, K] into th[BM x LDT] (zero rows >= nb, zero columns >= K).
__device__ __forceinline__ void stage_theta(float* th, const float* __restrict__ thetad, int nb,
                                            int K, int BM, int KP, int LDT, int tid) {
  constexpr int U = 8;
  const int n = BM * KP;
  for (int base = tid; base < n; base += U * DEC_THREADS) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * DEC_THREADS;
      const int b = min(i / KP, max(nb - 1, 0)), k = min(i % KP, K - 1);
      v[u] = thetad[(size_t)b * K + k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = base + u * DEC_THREADS;
      const int b = i / KP, k = i % KP;
      if (i < n) th[b * LDT + k] = (b < nb && k < K) ? v[u] : 0.f;
    }
  }
}
}  // namespace

// grid: dec_grid workgroups, grid-stride over the n_tiles vocab tiles.
// dynamic LDS: th[BM*LDT] + bt[KP*LDB] + lt[BM*LDB] + rowm[BM] + rows[BM]
template <int BM>
__global__ void __launch_bounds__(DEC_THREADS) prodlda_fwd_kernel(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, nb = *m.ws_nb, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  const int KP = round_up(K, 4), LDT = KP + 1;
  float* th = smem;
  float* bt = th + BM * LDT;
  float* lt = bt + KP * LDB;
  float* rowm = lt + BM * LDB;
  float* rows = rowm + BM;

  GFK_STAMP(m, 16);
  stage_theta(th, m.ws_thetad, nb, K, BM, KP, LDT, tid);
  for (int b = tid; b < BM; b += DEC_THREADS) { rowm[b] = -INFINITY; rows[b] = 0.f; }
  if (blockIdx.x == 0 && tid == 0) *m.nbt_beta += 1;

  constexpr int NSUB = (BM / 16) * (VB / 16);   // 16x16 output sub-tiles per vocab tile
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB;
    __syncthreads();
    GFK_STAMP(m, 17);
    stage_beta_tile(bt, m.beta, K, KP, V, c0, tid);
    __syncthreads();
    GFK_STAMP(m, 18);
    // ---- logits = theta_d @ beta_tile on the matrix cores ----
    for (int s = wave; s < NSUB; s += 4) {
      const int rs = s / (VB / 16), cs = s % (VB / 16);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* ap = th + (rs * 16 + (lane & 15)) * LDT + (lane >> 4);
      const float* bp = bt + (lane >> 4) * LDB + cs * 16 + (lane & 15);
      for (int k0 = 0; k0 < KP; k0 += 4) acc = mfma16x16x4(ap[k0], bp[k0 * LDB], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        lt[(rs * 16 + (lane >> 4) * 4 + r) * LDB + cs * 16 + (lane & 15)] = acc[r];
    }
    __syncthreads();
    GFK_STAMP(m, 19);
    // ---- column batch-norm: 4 threads per column ----
    {
      const int c = tid >> 2, sub = tid & 3;
      const bool valid = c0 + c < V;
      float s = 0.f;
      for (int b = sub; b < nb; b += 4) s += lt[b * LDB + c];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      const float mean = s / (float)nb;
      float q = 0.f;
      for (int b = sub; b < nb; b += 4) {
        const float d = lt[b * LDB + c] - mean;
        q += d * d;
      }
      q += __shfl_xor(q, 1, 64);
      q += __shfl_xor(q, 2, 64);
      const float var = q / (float)nb;
      const float rstd = rsqrtf(var + m.bn_eps);
      for (int b = sub; b < nb; b += 4) {
        const int i = b * LDB + c;
        lt[i] = valid ? (lt[i] - mean) * rstd : -INFINITY;
      }
      if (sub == 0 && valid) {
        const int v = c0 + c;
        const float mom = m.bn_momentum;
        const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
        m.beta_rm[v] = (1.f - mom) * m.beta_rm[v] + mom * mean;
        m.beta_rv[v] = (1.f - mom) * m.beta_rv[v] + mom * unb;
        m.ws_col_rstd[v] = rstd;
      }
    }
    __syncthreads();
    GFK_STAMP(m, 20);
    // ---- coalesced store of the BN'ed logits ----
    for (int i = tid; i < nb * VB; i += DEC_THREADS) {
      const int b = i / VB, c = i % VB;
      if (c0 + c < V) m.ws_zn[(size_t)b * V + c0 + c] = lt[b * LDB + c];
    }
    // ---- online (max, sum exp) per row: 4 threads per row, 16 columns each ----
    for (int b = tid >> 2; b < nb; b += DEC_THREADS / 4) {
      const int sub = tid & 3;
      const float* row = lt + b * LDB + 16 * sub;
      float mx = -INFINITY;
#pragma unroll
      for (int c = 0; c < 16; ++c) mx = fmaxf(mx, row[c]);
      mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
      float se = 0.f;
#pragma unroll
      for (int c = 0; c < 16; ++c) se += __expf(row[c] - mx);
      se += __shfl_xor(se, 1, 64);
      se += __shfl_xor(se, 2, 64);
      if (sub == 0) {
        float rm = rowm[b], rs_ = rows[b];
        lse_merge(rm, rs_, mx, se);
        rowm[b] = rm;
        rows[b] = rs_;
      }
    }
  }
  __syncthreads();
  GFK_STAMP(m, 21);
  for (int b = tid; b < nb; b += DEC_THREADS) {
    float* p = m.ws_row_part + ((size_t)blockIdx.x * m.bmax + b) * 2;
    p[0] = rowm[b];
    p[1] = rows[b];
  }
  GFK_STAMP(m, 22);
}

// One wave per batch row: log-sum-exp from the per-workgroup partials, the
// sparse reconstruction loss, S_b, and the per-tile CSR start table.
extern "C" __global__ void __launch_bounds__(64) gfk_prodlda_row_loss(GfkModel m) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int nb = *m.ws_nb;
  if (b >= nb) return;
  float mx = -INFINITY, se = 0.f;
  for (int g = lane; g < m.dec_grid; g += 64) {
    const float2 p = *reinterpret_cast<const float2*>(m.ws_row_part + ((size_t)g * m.bmax + b) * 2);
    lse_merge(mx, se, p.x, p.y);
  }
  wave_lse(mx, se);
  const float lse = mx + logf(se);
  const int doc = m.ws_doc[b];
  const int e0 = m.indptr[doc], e1 = m.indptr[doc + 1];
  const float* zn = m.ws_zn + (size_t)b * m.V;
  int32_t* ts = m.ws_tstart + (size_t)b * (m.n_tiles + 1);
  float rl = 0.f, S = 0.f;
  for (int e = e0 + lane; e < e1; e += 64) {
    const int col = m.indices[e];
    const int prev = e > e0 ? m.indices[e - 1] / VB : -1;
    const float x = m.values[e];
    const float p = expf(zn[col] - lse);
    rl += x * logf(p + RL_EPS);
    S += x * p / (p + RL_EPS);
    for (int t = prev + 1; t <= col / VB; ++t) ts[t] = e;
  }
  {  // tiles after the last non-zero start at e1
    const int last = e1 > e0 ? m.indices[e1 - 1] / VB : -1;
    for (int t = last + 1 + lane; t <= m.n_tiles; t += 64) ts[t] = e1;
  }
  rl = wave_sum(rl);
  S = wave_sum(S);
  if (lane == 0) {
    m.ws_lse[b] = lse;
    m.ws_rl[b] = -rl;
    m.ws_s[b] = S;
  }
}

// Backward.  dynamic LDS: th[BM*LDT] + bt[KP*LDB] + dt[BM*LDB] + zt[BM*LDB] + xt[BM*VB]
//                         + dacc[BM*LDT]   (KP = K rounded up to 16, LDT = KP + 1)
template <int BM>
__global__ void __launch_bounds__(DEC_THREADS) prodlda_bwd_kernel(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, nb = *m.ws_nb, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  const int KP = round_up(K, 16), LDT = KP + 1;
  float* th = smem;
  float* bt = th + BM * LDT;
  float* dt = bt + KP * LDB;
  float* zt = dt + BM * LDB;
  float* xt = zt + BM * LDB;
  float* dacc = xt + BM * VB;

  GFK_STAMP(m, 24);
  stage_theta(th, m.ws_thetad, nb, K, BM, KP, LDT, tid);
  for (int i = tid; i < BM * LDT; i += DEC_THREADS) dacc[i] = 0.f;
  const int ksub = KP / 16;
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB;
    __syncthreads();
    stage_beta_tile(bt, m.beta, K, KP, V, c0, tid);
    for (int i = tid; i < BM * VB; i += DEC_THREADS) xt[i] = 0.f;
    // zn tile (rows >= nb and columns >= V are zero so they drop out of every product)
    {
      constexpr int U = 8;
      for (int base = tid; base < BM * VB; base += U * DEC_THREADS) {
        float z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = base + u * DEC_THREADS;
          const int b = min(i / VB, max(nb - 1, 0)), c = min(c0 + i % VB, V - 1);
          z[u] = m.ws_zn[(size_t)b * V + c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = base + u * DEC_THREADS;
          const int b = i / VB, c = i % VB;
          if (i < BM * VB) zt[b * LDB + c] = (b < nb && c0 + c < V) ? z[u] : 0.f;
        }
      }
    }
    __syncthreads();
    GFK_STAMP(m, 25);
    // x tile from the per-tile CSR start table
    for (int b = tid; b < nb; b += DEC_THREADS) {
      const int32_t* ts = m.ws_tstart + (size_t)b * (m.n_tiles + 1) + tile;
      const int e0 = ts[0], e1 = ts[1];
      for (int e = e0; e < e1; ++e) xt[b * VB + m.indices[e] - c0] = m.values[e];
    }
    __syncthreads();
    GFK_STAMP(m, 26);
    // dL/dzn
    for (int i = tid; i < BM * VB; i += DEC_THREADS) {
      const int b = i / VB, c = i % VB;
      float d = 0.f;
      if (b < nb && c0 + c < V) {
        const float p = __expf(zt[b * LDB + c] - m.ws_lse[b]);
        d = p * m.ws_s[b] - xt[b * VB + c] * p / (p + RL_EPS);
      }
      dt[b * LDB + c] = d;
    }
    __syncthreads();
    GFK_STAMP(m, 27);
    // column BN backward (batch statistics)
    {
      const int c = tid >> 2, sub = tid & 3;
      float s1 = 0.f, s2 = 0.f;
      for (int b = sub; b < nb; b += 4) {
        const float g = dt[b * LDB + c];
        s1 += g;
        s2 += g * zt[b * LDB + c];
      }
      s1 += __shfl_xor(s1, 1, 64); s1 += __shfl_xor(s1, 2, 64);
      s2 += __shfl_xor(s2, 1, 64); s2 += __shfl_xor(s2, 2, 64);
      const float inv = 1.f / (float)nb;
      const float rstd = (c0 + c < V) ? m.ws_col_rstd[c0 + c] : 0.f;
      for (int b = sub; b < nb; b += 4) {
        const int i = b * LDB + c;
        dt[i] = rstd * (dt[i] - s1 * inv - zt[i] * s2 * inv);
      }
    }
    __syncthreads();
    GFK_STAMP(m, 28);
    // dbeta[k, c] = sum_b th[b, k] dlogit[b, c]: sub-tiles (KP/16) x (VB/16)
    for (int s = wave; s < ksub * (VB / 16); s += 4) {
      const int ks = s / (VB / 16), cs = s % (VB / 16);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* ap = th + (lane >> 4) * LDT + ks * 16 + (lane & 15);
      const float* bp = dt + (lane >> 4) * LDB + cs * 16 + (lane & 15);
      for (int b0 = 0; b0 < BM; b0 += 4) acc = mfma16x16x4(ap[b0 * LDT], bp[b0 * LDB], acc);
      const int c = c0 + cs * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = ks * 16 + (lane >> 4) * 4 + r;
        if (k < K && c < V) m.g_beta[(size_t)k * V + c] = acc[r];
      }
    }
    // dtheta_d[b, k] += sum_c dlogit[b, c] beta[k, c]: sub-tiles (BM/16) x (KP/16)
    for (int s = wave; s < (BM / 16) * ksub; s += 4) {
      const int rs = s / ksub, ks = s % ksub;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* ap = dt + (rs * 16 + (lane & 15)) * LDB + (lane >> 4);
      const float* bp = bt + (ks * 16 + (lane & 15)) * LDB + (lane >> 4);
      for (int c = 0; c < VB; c += 4) acc = mfma16x16x4(ap[c], bp[c], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dacc[(rs * 16 + (lane >> 4) * 4 + r) * LDT + ks * 16 + (lane & 15)] += acc[r];
    }
  }
  __syncthreads();
  GFK_STAMP(m, 29);
  for (int i = tid; i < nb * K; i += DEC_THREADS) {
    const int b = i / K, k = i % K;
    atomicAdd(m.ws_dthetad + i, dacc[b * LDT + k]);
  }
  GFK_STAMP(m, 30);
}

extern "C" size_t gfk_prodlda_fwd_smem(int bmax, int K) {
  const int KP = round_up(K, 4), LDT = KP + 1;
  return sizeof(float) * ((size_t)bmax * LDT + (size_t)KP * LDB + (size_t)bmax * LDB + 2 * bmax);
}

extern "C" size_t gfk_prodlda_bwd_smem(int bmax, int K) {
  const int KP = round_up(K, 16), LDT = KP + 1;
  return sizeof(float) * ((size_t)bmax * LDT * 2 + (size_t)KP * LDB + 2 * (size_t)bmax * LDB +
                          (size_t)bmax * VB);
}

extern "C" int gfk_launch_prodlda_fwd(const GfkModel* m, hipStream_t s) {
  const size_t sm = gfk_prodlda_fwd_smem(m->bmax, m->K);
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

extern "C" int gfk_launch_prodlda_bwd(const GfkModel* m, hipStream_t s) {
  const size_t sm = gfk_prodlda_bwd_smem(m->bmax, m->K);
  dim3 g(m->dec_grid), blk(DEC_THREADS);
  switch (m->bmax) {
    case 16: hipLaunchKernelGGL(prodlda_bwd_kernel<16>, g, blk, sm, s, *m); break;
    case 32: hipLaunchKernelGGL(prodlda_bwd_kernel<32>, g, blk, sm, s, *m); break;
    case 64: hipLaunchKernelGGL(prodlda_bwd_kernel<64>, g, blk, sm, s, *m); break;
    case 128: hipLaunchKernelGGL(prodlda_bwd_kernel<128>, g, blk, sm, s, *m); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_prodlda_row_loss(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_prodlda_row_loss, dim3(m->bmax), dim3(64), 0, s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_prodlda_set_smem(size_t bytes) {
  const void* ks[] = {(const void*)prodlda_fwd_kernel<16>, (const void*)prodlda_fwd_kernel<32>,
                      (const void*)prodlda_fwd_kernel<64>, (const void*)prodlda_fwd_kernel<128>,
                      (const void*)prodlda_bwd_kernel<16>, (const void*)prodlda_bwd_kernel<32>,
                      (const void*)prodlda_bwd_kernel<64>, (const void*)prodlda_bwd_kernel<128>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
