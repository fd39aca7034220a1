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
// [B, K] tensors in the posterior backward instead of a V-wide reduction.
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int LDA_THREADS = 256;
constexpr int VB = 64;
constexpr int LD = VB + 1;
constexpr float RL_EPS = 1e-10f;
}  // namespace

// grid: dec_grid workgroups over the vocab tiles.
// dynamic LDS: bn[K*LD] + rowm[K] + rows[K]
extern "C" __global__ void __launch_bounds__(LDA_THREADS) gfk_lda_beta_fwd(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, tid = threadIdx.x;
  float* bn = smem;
  float* rowm = bn + K * LD;
  float* rows = rowm + K;
  for (int k = tid; k < K; k += LDA_THREADS) { rowm[k] = -INFINITY; rows[k] = 0.f; }
  if (blockIdx.x == 0 && tid == 0) *m.nbt_beta += 1;
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB;
    __syncthreads();
    for (int i = tid; i < K * VB; i += LDA_THREADS) {
      const int k = i / VB, c = i % VB;
      bn[k * LD + c] = (c0 + c < V) ? m.beta[(size_t)k * V + c0 + c] : 0.f;
    }
    __syncthreads();
    {  // BN over the K topics of each column: 4 threads per column
      const int c = tid >> 2, sub = tid & 3;
      const bool valid = c0 + c < V;
      float s = 0.f;
      for (int k = sub; k < K; k += 4) s += bn[k * LD + c];
      s += __shfl_xor(s, 1, 64); s += __shfl_xor(s, 2, 64);
      const float mean = s / (float)K;
      float q = 0.f;
      for (int k = sub; k < K; k += 4) { const float d = bn[k * LD + c] - mean; q += d * d; }
      q += __shfl_xor(q, 1, 64); q += __shfl_xor(q, 2, 64);
      const float var = q / (float)K;
      const float rstd = rsqrtf(var + m.bn_eps);
      for (int k = sub; k < K; k += 4) {
        const int i = k * LD + c;
        bn[i] = valid ? (bn[i] - mean) * rstd : -INFINITY;
      }
      if (sub == 0 && valid) {
        const int v = c0 + c;
        const float mom = m.bn_momentum;
        const float unb = K > 1 ? var * (float)K / (float)(K - 1) : var;
        m.beta_rm[v] = (1.f - mom) * m.beta_rm[v] + mom * mean;
        m.beta_rv[v] = (1.f - mom) * m.beta_rv[v] + mom * unb;
        m.ws_col_rstd[v] = rstd;
      }
    }
    __syncthreads();
    // transposed store bn^T [V, K] (contiguous K-vector per token)
    for (int i = tid; i < K * VB; i += LDA_THREADS) {
      const int c = i / K, k = i % K;
      if (c0 + c < V) m.ws_zn[(size_t)(c0 + c) * K + k] = bn[k * LD + c];
    }
    // online (max, sum exp) over this tile for every topic row: 4 threads per row
    for (int k = tid >> 2; k < K; k += LDA_THREADS / 4) {
      const int sub = tid & 3;
      const float* row = bn + k * LD + 16 * sub;
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
        float rm = rowm[k], rs = rows[k];
        lse_merge(rm, rs, mx, se);
        rowm[k] = rm;
        rows[k] = rs;
      }
    }
  }
  __syncthreads();
  for (int k = tid; k < K; k += LDA_THREADS) {
    float* p = m.ws_row_part + ((size_t)blockIdx.x * K + k) * 2;
    p[0] = rowm[k];
    p[1] = rows[k];
  }
}

// One workgroup per document: sparse loss + d theta_d + scatter of d beta_sm^T.
// dynamic LDS: dth[4*K] + th[K] + rls[4]
extern "C" __global__ void __launch_bounds__(LDA_THREADS) gfk_lda_row_loss_bwd(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, nb = *m.ws_nb;
  if (b >= nb) return;
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  float* dth = smem;
  float* th = dth + 4 * K;
  float* rls = th + K;
  for (int k = tid; k < K; k += LDA_THREADS) th[k] = m.ws_thetad[(size_t)b * m.kt + k];
  __syncthreads();
  const int e0 = m.ws_erange[2 * b], e1 = m.ws_erange[2 * b + 1];
  constexpr int KQ = 4;   // K <= 256
  float acc[KQ] = {0.f, 0.f, 0.f, 0.f};
  float rl = 0.f;
  for (int e = e0 + wave; e < e1; e += 4) {
    const int v = m.indices[e];
    const float x = m.values[e];
    const float* bnr = m.ws_zn + (size_t)v * K;
    float bs[KQ];
    float wd = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      bs[q] = k < K ? __expf(bnr[k] - m.ws_lse[k]) : 0.f;
      wd += (k < K ? th[k] : 0.f) * bs[q];
    }
    wd = wave_sum(wd);
    const float g = -x / (wd + RL_EPS);
    rl += x * logf(wd + RL_EPS);
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      if (k < K) {
        acc[q] += g * bs[q];
        atomicAdd(m.ws_dbsm + (size_t)v * K + k, th[k] * g);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = lane + 64 * q;
    if (k < K) dth[wave * K + k] = acc[q];
  }
  // x and wd are wave-uniform, so every lane of a wave holds the wave's loss partial
  if (lane == 0) rls[wave] = rl;
  __syncthreads();
  for (int k = tid; k < K; k += LDA_THREADS)
    m.ws_dthetad[(size_t)b * K + k] = dth[k] + dth[K + k] + dth[2 * K + k] + dth[3 * K + k];
  if (tid == 0) m.ws_rl[b] = -(rls[0] + rls[1] + rls[2] + rls[3]);
}

// grid: dec_grid workgroups over vocab tiles.  softmax-over-V backward and
// BN-over-K backward; clears the consumed d beta_sm accumulator.
// dynamic LDS: bn[K*LD] + d[K*LD]
extern "C" __global__ void __launch_bounds__(LDA_THREADS) gfk_lda_beta_bwd(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, V = m.V, tid = threadIdx.x;
  float* bn = smem;
  float* d = bn + K * LD;
  for (int tile = blockIdx.x; tile < m.n_tiles; tile += gridDim.x) {
    const int c0 = tile * VB;
    __syncthreads();
    for (int i = tid; i < K * VB; i += LDA_THREADS) {
      const int c = i / K, k = i % K;
      float z = 0.f, g = 0.f;
      if (c0 + c < V) {
        const size_t o = (size_t)(c0 + c) * K + k;
        z = m.ws_zn[o];
        const float bs = __expf(z - m.ws_lse[k]);
        g = bs * (m.ws_dbsm[o] - m.ws_ck[k]);
        m.ws_dbsm[o] = 0.f;
      }
      bn[k * LD + c] = z;
      d[k * LD + c] = g;
    }
    __syncthreads();
    {
      const int c = tid >> 2, sub = tid & 3;
      float s1 = 0.f, s2 = 0.f;
      for (int k = sub; k < K; k += 4) {
        const float g = d[k * LD + c];
        s1 += g;
        s2 += g * bn[k * LD + c];
      }
      s1 += __shfl_xor(s1, 1, 64); s1 += __shfl_xor(s1, 2, 64);
      s2 += __shfl_xor(s2, 1, 64); s2 += __shfl_xor(s2, 2, 64);
      const float inv = 1.f / (float)K;
      if (c0 + c < V) {
        const float rstd = m.ws_col_rstd[c0 + c];
        for (int k = sub; k < K; k += 4) {
          const int i = k * LD + c;
          d[i] = rstd * (d[i] - s1 * inv - bn[i] * s2 * inv);
        }
      }
    }
    __syncthreads();
    for (int i = tid; i < K * VB; i += LDA_THREADS) {
      const int k = i / VB, c = i % VB;
      if (c0 + c < V) m.g_beta[(size_t)k * V + c0 + c] = d[k * LD + c];
    }
  }
}

extern "C" size_t gfk_lda_fwd_smem(int K) { return sizeof(float) * ((size_t)K * LD + 2 * K); }
extern "C" size_t gfk_lda_row_smem(int K) { return sizeof(float) * ((size_t)K * 5 + 4); }
extern "C" size_t gfk_lda_bwd_smem(int K) { return sizeof(float) * ((size_t)K * LD * 2); }

extern "C" int gfk_launch_lda_beta_fwd(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_lda_beta_fwd, dim3(m->dec_grid), dim3(LDA_THREADS), gfk_lda_fwd_smem(m->K),
                     s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_lda_row(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_lda_row_loss_bwd, dim3(m->bmax), dim3(LDA_THREADS), gfk_lda_row_smem(m->K),
                     s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_lda_beta_bwd(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_lda_beta_bwd, dim3(m->dec_grid), dim3(LDA_THREADS), gfk_lda_bwd_smem(m->K),
                     s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_lda_set_smem(size_t bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)gfk_lda_beta_fwd,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)gfk_lda_beta_bwd,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  return (int)e;
}
