// Per-document encoder forward: sparse gather of the input layer, hidden MLP,
// encoder dropout and the (pre-batch-norm) mu / log-sigma^2 heads; and the
// standalone backward scatter into the transposed input-layer weight.
//
// Reference math: inference_network.py:76-85 (AVITM), ctm inference_network.py:176-193.
//
// One 256-thread workgroup (4 waves) owns one document, so the bmax rows of a
// minibatch run on bmax CUs in parallel.  The input layer is stored transposed
// ([V, H0] row-major): every non-zero token gathers ONE contiguous 4*H0-byte
// row.  Each wave takes the document's non-zeros 16 at a time: lanes 0-15 load
// 16 (index, count) pairs with one instruction, the pairs are broadcast with
// __shfl and the 16 row loads are issued back to back (16 loads in flight per
// lane instead of a dependent index->row chain per token).  The MLP weights are
// staged into LDS with 16 independent loads per thread, issued BEFORE the
// gather so both round trips overlap.
#include "gfk_common.h"

using namespace gfk;

namespace {

constexpr int ENC_THREADS = 256;
constexpr int CH = 16;        // non-zeros per wave batch

// acc[q] (output j = lane + 64*q) += sum over this wave's non-zeros of x * W[v, j].
// Wave w takes non-zeros [e0 + 64w + 256r, +64): ONE lane-parallel load of the 64
// (index, count) pairs, then the W rows are loaded CH at a time, all in flight.
template <int NQ>
__device__ __forceinline__ void gather_rows(const int32_t* __restrict__ idx,
                                            const float* __restrict__ val, int e0, int e1,
                                            int wave, const float* __restrict__ w, int H,
                                            int lane, float* acc) {
  constexpr int CH = NQ == 1 ? 32 : (NQ == 2 ? 16 : 8);
  for (int base = e0 + wave * 64; base < e1; base += 256) {
    const int e = min(base + lane, e1 - 1);
    const int my_v = idx[e];
    const float my_x = (base + lane < e1) ? val[e] : 0.f;
    const int cnt = min(64, e1 - base);
    for (int g = 0; g < cnt; g += CH) {
      float wv[CH][NQ];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int v = __shfl(my_v, g + i, 64);
#pragma unroll
        for (int q = 0; q < NQ; ++q) wv[i][q] = w[(size_t)v * H + min(lane + 64 * q, H - 1)];
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const float x = __shfl(my_x, g + i, 64);
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += x * wv[i][q];
      }
    }
  }
}

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline int hmax_of(const GfkModel& m) {
  int h = 0;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) h = h > m.H[l] ? h : m.H[l];
  return h;
}

}  // namespace

// Floats of the staged encoder weights: hidden layers (W, b), then heads (W_mu,
// b_mu, W_s, b_s), each padded to a multiple of 4.
__host__ __device__ inline int enc_weights_floats(const GfkModel& m) {
  int n = 0;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < m.n_hidden) n += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
  const int Hl = m.H[m.n_hidden - 1];
  return n + 2 * (pad4(m.K * Hl) + pad4(m.K));
}

extern "C" size_t gfk_encoder_fwd_smem(const GfkModel* m) {
  size_t n = 4 * (size_t)m->H[0] + 2 * (size_t)hmax_of(*m);
  if (m->stage_flags & 1) n += enc_weights_floats(*m);
  return sizeof(float) * n;
}

// grid: bmax workgroups (one per batch row); rows >= nb exit.
// dynamic LDS: red[4*H0] + a_cur[hmax] + a_nxt[hmax] (+ staged weights)
//
// Round trips: (1) kernel arguments (pinned in SGPRs up front), (2) the batch
// prepared by the previous step (nb, doc, CSR extent) + the step counter, with
// the weight staging (LDS-DMA) in flight, (3) the row's (index, count) pairs,
// (4) the W_in rows.  Everything after that is LDS.
extern "C" __global__ void __launch_bounds__(ENC_THREADS)
gfk_encoder_fwd(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  // ---- prologue: every argument field used before the first barrier ----
  int H0 = m.H[0], H1 = m.H[1], H2 = m.H[2], nh = m.n_hidden, K = m.K, sflags = m.stage_flags;
  int bmax = m.bmax;
  const int32_t* nxt = m.ws_next;
  const int32_t* indices = m.indices;
  const float* values = m.values;
  const float* w_in = m.w_in;
  const int32_t* stepp = m.step;
  const float *w_h0 = m.w_h[0], *b_h0 = m.b_h[0], *w_h1 = m.w_h[1], *b_h1 = m.b_h[1];
  const float *w_mu = m.w_mu, *b_mu = m.b_mu, *w_s = m.w_s, *b_s = m.b_s;
  keep(H0, H1, H2, nh, K, sflags, bmax, nxt, indices, values, w_in, stepp, w_h0, b_h0, w_h1, b_h1,
       w_mu, b_mu, w_s, b_s);
  const int Hl = m.H[nh - 1], hm = hmax_of(m);
  float* red = smem;
  float* a_cur = red + 4 * H0;
  float* a_nxt = a_cur + hm;
  const bool staged = sflags & 1;

  // ---- the batch row (prepared by the previous step) and the weight staging ----
  const int nb = nxt[0];
  const int doc = nxt[1 + min(b, bmax - 1)];
  const int e0 = nxt[1 + bmax + 2 * b], e1 = nxt[2 + bmax + 2 * b];
  const int step = *stepp;
  // layout: per hidden layer [W (pad4) | b (pad4)], then W_mu, b_mu, W_s, b_s
  float* wst = a_nxt + hm;
  if (staged) {   // LDS-DMA: all copies in flight at once, drained by the first barrier
    float* p = wst;
#pragma unroll
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
      if (l + 1 < nh) {
        const int hi = l == 0 ? H0 : (l == 1 ? H1 : m.H[l]);
        const int ho = l == 0 ? H1 : (l == 1 ? H2 : m.H[l + 1]);
        const float* W = l == 0 ? w_h0 : (l == 1 ? w_h1 : m.w_h[l]);
        const float* Bv = l == 0 ? b_h0 : (l == 1 ? b_h1 : m.b_h[l]);
        glds_copy(p, W, ho * hi, tid, ENC_THREADS); p += pad4(ho * hi);
        glds_copy(p, Bv, ho, tid, ENC_THREADS); p += pad4(ho);
      }
    }
    glds_copy(p, w_mu, K * Hl, tid, ENC_THREADS); p += pad4(K * Hl);
    glds_copy(p, b_mu, K, tid, ENC_THREADS); p += pad4(K);
    glds_copy(p, w_s, K * Hl, tid, ENC_THREADS); p += pad4(K * Hl);
    glds_copy(p, b_s, K, tid, ENC_THREADS);
  }
  if (b >= nb) {            // drain the LDS-DMA before the workgroup retires
    __syncthreads();
    return;
  }
  if (tid == 0) {           // publish the batch for the rest of the step
    m.ws_doc[b] = doc;
    m.ws_erange[2 * b] = e0;
    m.ws_erange[2 * b + 1] = e1;
    if (b == 0) *m.ws_nb = nb;
  }

  // ---- input layer: BoW gather (+ dense contextual part precomputed in ws_hctx) ----
  const bool has_bow = m.input != GFK_IN_CONTEXTUAL;
  if (has_bow) {
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.f;
    if (H0 <= 64) gather_rows<1>(indices, values, e0, e1, wave, w_in, H0, lane, acc);
    else if (H0 <= 128) gather_rows<2>(indices, values, e0, e1, wave, w_in, H0, lane, acc);
    else if (H0 <= 256) gather_rows<4>(indices, values, e0, e1, wave, w_in, H0, lane, acc);
    else gather_rows<8>(indices, values, e0, e1, wave, w_in, H0, lane, acc);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = lane + 64 * q;
      if (j < H0) red[wave * H0 + j] = acc[q];
    }
  }
  __syncthreads();
  for (int j = tid; j < H0; j += ENC_THREADS) {
    float z = m.b_in[j];
    if (has_bow) z += red[j] + red[H0 + j] + red[2 * H0 + j] + red[3 * H0 + j];
    if (m.input != GFK_IN_BOW) z += m.ws_hctx[(size_t)b * H0 + j];
    const float a = act_f(m.act, z);
    m.ws_z[0][(size_t)b * H0 + j] = z;
    m.ws_a[0][(size_t)b * H0 + j] = a;
    a_cur[j] = a;
  }
  __syncthreads();

  // ---- hidden layers: z_{l+1} = W_l a_l + b_l ----
  float* ain = a_cur;
  float* aout = a_nxt;
  const float* wcur = wst;
  for (int l = 0; l + 1 < nh; ++l) {
    const int Hi = m.H[l], Ho = m.H[l + 1];
    const float* W = staged ? wcur : m.w_h[l];
    const float* Bv = staged ? wcur + pad4(Ho * Hi) : m.b_h[l];
    wcur += pad4(Ho * Hi) + pad4(Ho);
    for (int j = tid; j < Ho; j += ENC_THREADS) {
      float z = Bv[j];
      const float* wr = W + (size_t)j * Hi;
#pragma unroll 8
      for (int i = 0; i < Hi; ++i) z += wr[i] * ain[i];
      const float a = act_f(m.act, z);
      m.ws_z[l + 1][(size_t)b * Ho + j] = z;
      m.ws_a[l + 1][(size_t)b * Ho + j] = a;
      aout[j] = a;
    }
    __syncthreads();
    float* t = ain; ain = aout; aout = t;
  }

  // ---- encoder dropout (p fixed at 0.2 in the reference) ----
  for (int j = tid; j < Hl; j += ENC_THREADS) {
    const float s = drop_scale(m.seed, (uint32_t)step, RNG_DROP_ENC, (uint32_t)(b * Hl + j),
                               m.drop_enc);
    const float hd = ain[j] * s;
    m.ws_mask_h[(size_t)b * Hl + j] = s;
    m.ws_hd[(size_t)b * Hl + j] = hd;
    aout[j] = hd;
  }
  __syncthreads();

  // ---- mu / log-sigma heads (pre-BN) ----
  const float* Wmu = staged ? wcur : w_mu;
  const float* Bmu = staged ? wcur + pad4(K * Hl) : b_mu;
  const float* Ws = staged ? wcur + pad4(K * Hl) + pad4(K) : w_s;
  const float* Bs = staged ? wcur + 2 * pad4(K * Hl) + pad4(K) : b_s;
  for (int t = tid; t < 2 * K; t += ENC_THREADS) {
    const bool is_mu = t < K;
    const int k = is_mu ? t : t - K;
    const float* wr = (is_mu ? Wmu : Ws) + (size_t)k * Hl;
    float z = is_mu ? Bmu[k] : Bs[k];
#pragma unroll 8
    for (int j = 0; j < Hl; ++j) z += wr[j] * aout[j];
    (is_mu ? m.ws_mu_raw : m.ws_ls_raw)[(size_t)b * K + k] = z;
  }
}

// Standalone backward of the sparse input layer (the fused step does this
// inside gfk_posterior_bwd): g_w_in[v, :] += x_bv * dz0[b, :].  Float atomics
// (a word shared by several documents of the batch hits the same row); each
// wave instruction adds one contiguous 4*H0-byte row.  grid: bmax workgroups.
extern "C" __global__ void __launch_bounds__(ENC_THREADS)
gfk_encoder_bwd_scatter(GfkModel m) {
  // grid (bmax, scatter_chunks): workgroup (b, y) takes chunks y, y + gridDim.y, ...
  // of 64 non-zeros of row b; each wave owns 16 of them, so every wave has at
  // most 16 * ceil(H0/64) atomics in flight and the whole scatter is one round.
  const int b = blockIdx.x;
  const int nb = *m.ws_nb;
  if (b >= nb) return;
  const int H0 = m.H[0];
  const int lane = threadIdx.x & 63, wave = uniform(threadIdx.x >> 6);
  const float* dz = m.ws_dz0 + (size_t)b * H0;
  const int e0 = m.ws_erange[2 * b], e1 = m.ws_erange[2 * b + 1];
  for (int base = e0 + (blockIdx.y * 4 + wave) * CH; base < e1; base += gridDim.y * 4 * CH) {
    const int e = min(base + (lane & (CH - 1)), e1 - 1);
    const int my_v = m.indices[e];
    const float my_x = m.values[e];
    const int cnt = min(CH, e1 - base);
    for (int j0 = 0; j0 < H0; j0 += 64) {
      const int j = j0 + lane;
      const float d = dz[min(j, H0 - 1)];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int v = __shfl(my_v, i, 64);
        const float x = __shfl(my_x, i, 64);
        if (i < cnt && j < H0) atomicAdd(m.g_w_in + (size_t)v * H0 + j, x * d);
      }
    }
  }
}

extern "C" int gfk_launch_encoder_fwd(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_encoder_fwd, dim3(m->bmax), dim3(ENC_THREADS), gfk_encoder_fwd_smem(m), s,
                     *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_encoder_bwd(const GfkModel* m, hipStream_t s) {
  const int gy = m->scatter_chunks > 0 ? m->scatter_chunks : 1;
  hipLaunchKernelGGL(gfk_encoder_bwd_scatter, dim3(m->bmax, gy), dim3(ENC_THREADS), 0, s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_encoder_set_smem(size_t bytes) {
  return (int)hipFuncSetAttribute((const void*)gfk_encoder_fwd,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
