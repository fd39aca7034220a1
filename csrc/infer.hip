// theta inference: the document-topic distribution of a whole corpus in one
// launch (reference avitm.py:470-523 get_doc_topic_distribution,
// decoder_network.py:137-147 get_theta, federated_model.py:170-173 the theta
// post-processing).
//
// The reference runs S = 20 full passes over the dataset, each one re-running
// the encoder on dense [B, V] rows, and averages softmax(mu + eps * sigma).  In
// eval mode mu and sigma are deterministic (batch-norm uses running statistics,
// no dropout), so here the encoder runs ONCE per document and the S samples are
// drawn in registers:
//
//   z0 = x W_in^T + b_in (+ contextual part)   sparse gather over the CSR row
//   h  = act(...) through the hidden MLP        weights staged in LDS (transposed)
//   mu, log s^2 = heads, BN with running stats
//   theta = mean_s softmax(mu + eps_s * exp(log s^2 / 2))
//   optional: theta[theta < thr] = 0, rows L1-normalised
//
// Mapping (throughput, not latency): one wave64 per document, 8 waves per
// workgroup sharing one LDS copy of the MLP weights, the grid sized to fill the
// 256 CUs with documents dealt round-robin over all waves (a persistent loop
// every wave leaves after its last document).  The input-layer gather keeps
// CH row loads in flight per lane; the hidden layers and heads read weights
// out of LDS with lane j on output j (transposed layout: conflict-free, the
// activation operand is an LDS broadcast); the sampling draws four normals per
// Philox call (Box-Muller, both branches) and reduces each sample's softmax
// with wave shuffles.  Draws are keyed by (seed, global document index, topic),
// so the result does not depend on the grid or on how the corpus is chunked.
#define GFK_BATCHED_COPY 1   // batched kernels copy their descriptor (gfk_common.h gfk_model)
#include "gfk_common.h"

using namespace gfk;

extern "C" {
typedef struct GfkInfer {
  const int32_t *indptr, *indices;  // indptr: this chunk's row pointers (n_docs + 1)
  const float *values;
  const float *hctx;     // [n_docs, H0] dense contextual contribution (CTM) or null
  float *out;            // [n_docs, K]; flags bit1: [n_docs, 2, K] (mu | log-sigma^2)
  int32_t n_docs, n_samples;
  int32_t flags;         // bit0: threshold + L1 normalise; bit1: posterior moments only
  float thr;
  uint64_t seed;
  int32_t grid, doc0;    // doc0: global index of the chunk's first document (RNG key)
} GfkInfer;
}

namespace {

constexpr int INF_THREADS = 512;
constexpr int INF_WAVES = INF_THREADS / 64;

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline int inf_hmax(const GfkModel& m) {
  int h = m.K;
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) h = h > m.H[l] ? h : m.H[l];
  return h;
}

// Staged floats: per hidden layer W^T [Hi][Ho] + b [Ho]; heads W_mu^T, W_s^T
// [Hl][K]; b_mu, b_s, mu running mean, mu rstd, s running mean, s rstd [K] each.
__host__ __device__ inline int inf_weight_floats(const GfkModel& m) {
  int n = 0;
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < m.n_hidden) n += pad4(m.H[l] * m.H[l + 1]) + pad4(m.H[l + 1]);
  const int Hl = gfk_hlast(m);
  return n + 2 * pad4(Hl * m.K) + 6 * pad4(m.K);
}

__host__ __device__ inline size_t inf_act_floats(const GfkModel& m) {
  return (size_t)INF_WAVES * 2 * pad4(inf_hmax(m));
}

__device__ __forceinline__ void wave_lds_sync() {
  // LDS hand-off between the lanes of ONE wave: LDS executes a wave's
  // instructions in order, so draining lgkmcnt is enough; the clobber keeps the
  // compiler from moving LDS accesses across.
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// acc[q] (output j = lane + 64 q) = sum over the row's non-zeros of x * W_in^T[v][j].
template <int NQ>
__device__ __forceinline__ void gather_doc(const int32_t* __restrict__ idx, const float* __restrict__ val,
                                           int e0, int e1, const float* __restrict__ w, int H, int lane,
                                           float* acc) {
  constexpr int CH = NQ == 1 ? 16 : (NQ == 2 ? 8 : 4);
  for (int base = e0; base < e1; base += 64) {
    const int le = base + lane;
    const int e = min(le, e1 - 1);
    const int my_v = idx[e];
    const float my_x = le < e1 ? val[e] : 0.f;
    const int cnt = min(64, e1 - base);
    for (int g = 0; g < cnt; g += CH) {
      float wv[CH][NQ];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int v = __builtin_amdgcn_readlane(my_v, min(g + i, 63));
        const float* wr = w + (size_t)v * H;
#pragma unroll
        for (int q = 0; q < NQ; ++q) wv[i][q] = wr[min(lane + 64 * q, H - 1)];
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_x), min(g + i, 63)));
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += (g + i < cnt ? x : 0.f) * wv[i][q];
      }
    }
  }
}

// Box-Muller on both halves of one Philox draw: four N(0, 1) values.
__device__ __forceinline__ void randn4(uint64_t seed, uint32_t ctr, uint32_t idx, float* n) {
  const uint4 r = rng4(seed, ctr, RNG_INFER, idx);
  const float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u2 = u01(r.y);
  const float u3 = ((float)(r.z >> 8) + 1.0f) * (1.0f / 16777216.0f);
  const float u4 = u01(r.w);
  const float ra = sqrtf(-2.0f * logf(u1)), rb = sqrtf(-2.0f * logf(u3));
  float s2, c2, s4, c4;
  sincospif(2.0f * u2, &s2, &c2);
  sincospif(2.0f * u4, &s4, &c4);
  n[0] = ra * c2; n[1] = ra * s2; n[2] = rb * c4; n[3] = rb * s4;
}

// NQ: input-layer outputs per lane (H0 <= 64 NQ); KQ: topics per lane (K <= 64 KQ).
template <bool Staged, int NQ, int KQ, bool GB = false>
__global__ void __launch_bounds__(INF_THREADS) gfk_theta_infer_k(GfkArgT<GB> ga, GfkInfer p) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int H0 = m.H[0], K = m.K, nh = m.n_hidden, act = m.act, input = m.input;
  const int Hl = gfk_hlast(m), hm = pad4(inf_hmax(m));
  const float bn_eps = m.bn_eps;
  float* wst = smem;
  float* abuf = smem + (Staged ? inf_weight_floats(m) : 0) + wave * 2 * hm;

  // ---- stage the MLP (transposed), head biases and BN running statistics ----
  if (Staged) {
    float* q = wst;
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
      if (l + 1 >= nh) break;
      const int Hi = m.H[l], Ho = m.H[l + 1];
      const float* W = m.w_h[l];
      for (int t = tid; t < Hi * Ho; t += INF_THREADS) {
        const int j = t / Hi, i = t - j * Hi;       // coalesced read of W[j][i]
        q[i * Ho + j] = W[t];
      }
      q += pad4(Hi * Ho);
      for (int t = tid; t < Ho; t += INF_THREADS) q[t] = m.b_h[l][t];
      q += pad4(Ho);
    }
    for (int t = tid; t < K * Hl; t += INF_THREADS) {
      const int k = t / Hl, i = t - k * Hl;
      q[i * K + k] = m.w_mu[t];
      q[pad4(Hl * K) + i * K + k] = m.w_s[t];
    }
    q += 2 * pad4(Hl * K);
    for (int t = tid; t < K; t += INF_THREADS) {
      q[t] = m.b_mu[t];
      q[pad4(K) + t] = m.b_s[t];
      q[2 * pad4(K) + t] = m.mu_rm[t];
      q[3 * pad4(K) + t] = rsqrtf(m.mu_rv[t] + bn_eps);
      q[4 * pad4(K) + t] = m.s_rm[t];
      q[5 * pad4(K) + t] = rsqrtf(m.s_rv[t] + bn_eps);
    }
    __syncthreads();
  }

  const int n_docs = p.n_docs, S = p.n_samples, flags = p.flags;
  const int nwaves_total = gridDim.x * INF_WAVES;
  const size_t ostride = (flags & 2) ? 2 * (size_t)K : (size_t)K;
  float bias_in[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) bias_in[q] = m.b_in[min(lane + 64 * q, H0 - 1)];

  for (int d = blockIdx.x * INF_WAVES + wave; d < n_docs; d += nwaves_total) {
    // ---- input layer ----
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
    if (input != GFK_IN_CONTEXTUAL) {
      const int e0 = p.indptr[d], e1 = p.indptr[d + 1];
      gather_doc<NQ>(p.indices, p.values, e0, e1, m.w_in, H0, lane, acc);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int j = lane + 64 * q;
      if (j < H0) {
        float z = acc[q] + bias_in[q];
        if (input != GFK_IN_BOW) z += p.hctx[(size_t)d * H0 + j];
        abuf[j] = act_f(act, z);
      }
    }
    wave_lds_sync();

    // ---- hidden layers (lane j -> outputs j, j + 64, ...) ----
    float* ain = abuf;
    float* aout = abuf + hm;
    const float* wq = wst;
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
      if (l + 1 >= nh) break;
      const int Hi = m.H[l], Ho = m.H[l + 1];
      for (int j = lane; j < Ho; j += 64) {
        float z;
        if (Staged) {
          z = wq[pad4(Hi * Ho) + j];
          for (int i = 0; i < Hi; ++i) z += wq[i * Ho + j] * ain[i];
        } else {
          const float* W = m.w_h[l] + (size_t)j * Hi;
          z = m.b_h[l][j];
          for (int i = 0; i < Hi; ++i) z += W[i] * ain[i];
        }
        aout[j] = act_f(act, z);
      }
      if (Staged) wq += pad4(Hi * Ho) + pad4(Ho);
      wave_lds_sync();
      float* t = ain; ain = aout; aout = t;
    }

    // ---- heads + batch-norm with running statistics ----
    float mu[KQ], ls[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = min(lane + 64 * q, K - 1);
      float a, b;
      if (Staged) {
        const float* Wm = wq;
        const float* Ws = wq + pad4(Hl * K);
        const float* v = wq + 2 * pad4(Hl * K);
        a = v[k];
        b = v[pad4(K) + k];
        for (int i = 0; i < Hl; ++i) {
          const float h = ain[i];
          a += Wm[i * K + k] * h;
          b += Ws[i * K + k] * h;
        }
        mu[q] = (a - v[2 * pad4(K) + k]) * v[3 * pad4(K) + k];
        ls[q] = (b - v[4 * pad4(K) + k]) * v[5 * pad4(K) + k];
      } else {
        const float* Wm = m.w_mu + (size_t)k * Hl;
        const float* Ws = m.w_s + (size_t)k * Hl;
        a = m.b_mu[k];
        b = m.b_s[k];
        for (int i = 0; i < Hl; ++i) {
          const float h = ain[i];
          a += Wm[i] * h;
          b += Ws[i] * h;
        }
        mu[q] = (a - m.mu_rm[k]) * rsqrtf(m.mu_rv[k] + bn_eps);
        ls[q] = (b - m.s_rm[k]) * rsqrtf(m.s_rv[k] + bn_eps);
      }
    }
    float* orow = p.out + (size_t)d * ostride;
    if (flags & 2) {                 // posterior moments only (tests, custom samplers)
#pragma unroll
      for (int q = 0; q < KQ; ++q) {
        const int k = lane + 64 * q;
        if (k < K) { orow[k] = mu[q]; orow[K + k] = ls[q]; }
      }
      continue;
    }

    // ---- S reparameterised samples of softmax(theta), averaged ----
    const uint32_t key0 = (uint32_t)((size_t)(p.doc0 + d) * K);
    float sd[KQ], th[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      sd[q] = __expf(0.5f * ls[q]);
      th[q] = 0.f;
    }
    for (int s0 = 0; s0 < S; s0 += 4) {
      float nz[KQ][4];
#pragma unroll
      for (int q = 0; q < KQ; ++q) randn4(p.seed, (uint32_t)(s0 >> 2), key0 + lane + 64 * q, nz[q]);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (s0 + r >= S) break;
        float z[KQ], mx = -INFINITY;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          z[q] = lane + 64 * q < K ? mu[q] + nz[q][r] * sd[q] : -INFINITY;
          mx = fmaxf(mx, z[q]);
        }
        mx = wave_max(mx);
        float e[KQ], sum = 0.f;
#pragma unroll
        for (int q = 0; q < KQ; ++q) {
          e[q] = lane + 64 * q < K ? __expf(z[q] - mx) : 0.f;
          sum += e[q];
        }
        const float inv = 1.f / wave_sum(sum);
#pragma unroll
        for (int q = 0; q < KQ; ++q) th[q] += e[q] * inv;
      }
    }
    const float invS = 1.f / (float)S;
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      th[q] *= invS;
      if (flags & 1) {
        if (th[q] < p.thr) th[q] = 0.f;
        tot += lane + 64 * q < K ? th[q] : 0.f;
      }
    }
    if (flags & 1) {
      tot = wave_sum(tot);
      const float inv = tot > 0.f ? 1.f / tot : 1.f;
#pragma unroll
      for (int q = 0; q < KQ; ++q) th[q] *= inv;
    }
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      if (k < K) orow[k] = th[q];
    }
  }
}

template <bool Staged, int NQ>
int launch_kq(const GfkModel* m, const GfkInfer* p, size_t smem, hipStream_t s) {
  const int KQ = (m->K + 63) / 64;
  void (*k)(GfkArgT<false>, GfkInfer) = nullptr;
  switch (KQ) {
    case 1: k = gfk_theta_infer_k<Staged, NQ, 1>; break;
    case 2: k = gfk_theta_infer_k<Staged, NQ, 2>; break;
    case 3: k = gfk_theta_infer_k<Staged, NQ, 3>; break;
    case 4: k = gfk_theta_infer_k<Staged, NQ, 4>; break;
    case 5: case 6: case 7: case 8: k = gfk_theta_infer_k<Staged, NQ, 8>; break;   // (K <= 512)
    default: return -3;
  }
  hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(k, dim3(p->grid), dim3(INF_THREADS), smem, s, GfkArgT<false>{*m}, *p);
  return (int)hipGetLastError();
}

template <bool Staged>
int launch_nq(const GfkModel* m, const GfkInfer* p, size_t smem, hipStream_t s) {
  const int H0 = m->H[0];
  if (H0 <= 64) return launch_kq<Staged, 1>(m, p, smem, s);
  if (H0 <= 128) return launch_kq<Staged, 2>(m, p, smem, s);
  if (H0 <= 256) return launch_kq<Staged, 4>(m, p, smem, s);
  if (H0 <= 512) return launch_kq<Staged, 8>(m, p, smem, s);
  return -4;
}

}  // namespace

extern "C" size_t gfk_infer_struct_size() { return sizeof(GfkInfer); }

// LDS bytes of the staged variant (the launcher falls back to the unstaged one
// above 160 KiB).
extern "C" size_t gfk_theta_infer_smem(const GfkModel* m) {
  return sizeof(float) * ((size_t)inf_weight_floats(*m) + inf_act_floats(*m));
}

// Host checks mirror the kernel's assumptions: K <= 512, H0 <= 512, a CSR with
// n_docs + 1 row pointers (or, for contextual-only input, hctx), grid >= 1.
extern "C" int gfk_theta_infer(const GfkModel* m, const GfkInfer* p, hipStream_t s) {
  if (p->n_docs <= 0) return 0;
  if (m->K <= 0 || m->K > 512 || m->H[0] <= 0 || m->H[0] > 512 || p->grid <= 0 || !p->out) return -5;
  if (!(p->flags & 2) && p->n_samples <= 0) return -6;
  if (m->input != GFK_IN_CONTEXTUAL && (!p->indptr || !p->indices || !p->values)) return -7;
  if (m->input != GFK_IN_BOW && !p->hctx) return -8;
  const size_t staged = gfk_theta_infer_smem(m);
  if (staged <= 160 * 1024) return launch_nq<true>(m, p, staged, s);
  return launch_nq<false>(m, p, sizeof(float) * inf_act_floats(*m), s);
}
