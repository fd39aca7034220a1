// Encoder forward, one workgroup per document row: the sparse BoW gather
// z0 = x W_in^T + b_in, the hidden MLP, the encoder dropout and the (pre
// batch-norm) mu / log-sigma^2 heads -- plus all random draws of the row.
//
// Reference math: inference_network.py:76-85 (AVITM), ctm inference_network.py:176-193
// (the dense contextual part of CombinedTM / ZeroShotTM arrives precomputed in
// ws_hctx); the draws are avitm decoder_network.py:102-118 (reparameterisation
// noise, theta dropout) and inference_network.py:82 (encoder dropout).
//
// One workgroup of 16 waves owns one document, so a minibatch of B rows runs on
// B CUs with 16 * B waves.  The input layer is stored TRANSPOSED ([V, H0]
// row-major): every non-zero token gathers one contiguous 4*H0-byte row.  Wave w
// takes non-zeros [e0 + 64w + 1024r, +64): one lane-parallel load of the 64
// (index, count) pairs, then the W rows CH at a time, all in flight (the pair is
// broadcast with v_readlane into SGPRs, so the row address is scalar).  The
// per-wave partial rows are summed through LDS.
//
// The batch itself (nb, doc ids, CSR extents) was prepared by the previous step
// (prepare_next_batch), so the row's CSR extent is one round trip away.  The
// random draws (Philox, keyed by seed/step/element) are produced here, where the
// VALU is otherwise idle waiting on the gather.  Everything up to the heads is
// row-local; the batch coupling (batch-norm) starts in post_fwd.
// (batched descriptor by reference: with the copy (gfk_common.h gfk_model) the narrow
// instance ran 14.5 -> 20 us at M = 8, profiles/r5/ab_batched_copy2.txt)
#include "gfk_common.h"

using namespace gfk;

namespace {

constexpr int ENC_THREADS = 1024;
constexpr int ENC_WAVES = ENC_THREADS / 64;

// acc[q] (output j = lane + 64*q) += sum over this wave's non-zeros of x * W[v, j], for
// the row's non-zeros j in [0, n) of its slot copy (prepare_next_batch).  Non-zeros
// are dealt round-robin over the waves (wave w: j = w + ENC_WAVES * i), so a typical
// row (~100-200 non-zeros) costs every wave one batch of CH W_in row loads in flight;
// this lane's first (index, value) (j = wave + 16 lane) was loaded by the caller with
// the row's extent, so the W_in row loads are the kernel's second round trip.
template <int NQ>
__device__ __forceinline__ void gather_slots(const int32_t* __restrict__ sidx,
                                             const float* __restrict__ sval, int n, int v0,
                                             float x0, int wave, const float* __restrict__ w,
                                             int H, int lane, float* acc) {
  constexpr int CH = NQ == 1 ? 16 : (NQ == 2 ? 8 : 4);
  for (int base = wave; base < n; base += ENC_WAVES * 64) {
    const int le = base + ENC_WAVES * lane;
    int my_v = v0;
    float my_x = le < n ? x0 : 0.f;
    if (base != wave) {                  // rows of more than 1024 non-zeros
      my_v = sidx[min(le, n - 1)];
      my_x = le < n ? sval[min(le, n - 1)] : 0.f;
    }
    const int cnt = min(64, (n - base + ENC_WAVES - 1) / ENC_WAVES);
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

// ZeroShotTM's dense input layer inside the gather: acc[q] += sum over this wave's
// contextual features c (c = wave + 16 i) of x[c] * W[c, j], W = the transposed
// [C, H0] input layer; the same batches of CH row loads in flight as gather_slots.
template <int NQ>
__device__ __forceinline__ void gather_dense(const float* __restrict__ x, int C, int wave,
                                             const float* __restrict__ w, int H, int lane,
                                             float* acc) {
  constexpr int CH = NQ == 1 ? 16 : (NQ == 2 ? 8 : 4);
  for (int base = wave; base < C; base += ENC_WAVES * 64) {
    const int le = base + ENC_WAVES * lane;
    const float my_x = le < C ? x[le] : 0.f;
    const int cnt = min(64, (C - base + ENC_WAVES - 1) / ENC_WAVES);
    for (int g = 0; g < cnt; g += CH) {
      float wv[CH][NQ];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int v = min(base + ENC_WAVES * min(g + i, cnt - 1), C - 1);
        const float* wr = w + (size_t)v * H;
#pragma unroll
        for (int q = 0; q < NQ; ++q) wv[i][q] = wr[min(lane + 64 * q, H - 1)];
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const float xg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(my_x), min(g + i, 63)));
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += (g + i < cnt ? xg : 0.f) * wv[i][q];
      }
    }
  }
}

}  // namespace

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

// Floats of the staged MLP weights: per hidden layer [W (pad4) | b (pad4)], then
// W_mu, b_mu, W_s, b_s (pad4 each) -- the LDS-DMA destination layout.
__host__ __device__ inline int enc_weight_floats(const GfkModel& m) {
  int n = 0;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < m.n_hidden) n += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
  const int Hl = gfk_hlast(m);
  return n + 2 * (pad4(m.K * Hl) + pad4(m.K));
}

__host__ __device__ inline int enc_hmax(const GfkModel& m) {
  int h = 0;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) h = h > m.H[l] ? h : m.H[l];
  return h;
}

// dynamic LDS: red[16][H0] + act[2][hmax] + mask[Hl] + labels[L] (+ staged weights)
extern "C" size_t gfk_enc_in_smem(const GfkModel* m) {
  size_t n = (size_t)ENC_WAVES * m->H[0] + 2 * (size_t)pad4(enc_hmax(*m)) + pad4(m->H[m->n_hidden - 1]) +
             (m->lab_on ? pad4(m->L) : 0);
  if (m->stage_flags & 1) n += enc_weight_floats(*m);
  return sizeof(float) * n;
}

// out[j] = sum_i W[j][i] x[i] (+ bias) for j < n_out: 16 lanes (one DPP row) per
// output split the inputs, 64 outputs per pass of the workgroup.  A ds_read_b32 is
// banked per 32-lane half-wave, whose two 16-lane rows read 16 consecutive words of two
// weight rows: rows j and j + 1 (n_in = 50 words apart) shared banks (11 % LDS conflict
// cycles, k50_counters.md).  The half-wave's second row is j + d instead, with
// d n_in = 16 (mod 32) -- d = 16 / (the largest power of two dividing n_in, <= 16) --
// so the two rows cover all 32 banks once; (P, g) -> (P / d) 2d + P % d + g d maps the
// 32 half-waves x 2 rows onto the pass's 64 outputs one to one.  Each output's sum is
// the same sequence of operations as before (only which lanes compute it changed).
template <class Epi>
__device__ __forceinline__ void rowvec_gemv(const float* W, const float* x, int n_out, int n_in, int tid,
                                            Epi epi) {
  const int s = tid & 15;
  const int tz = n_in & -n_in;                          // lowest set bit of n_in
  const int ld = tz >= 16 ? 0 : 4 - __builtin_ctz(tz);  // log2 d
  const int P = tid >> 5, g = (tid >> 4) & 1;
  const int jo = ((P >> ld) << (ld + 1)) + (P & ((1 << ld) - 1)) + (g << ld);
  for (int j0 = 0; j0 < n_out; j0 += ENC_THREADS / 16) {
    const int j = j0 + jo;
    float acc = 0.f;
    if (j < n_out) {
      const float* wr = W + (size_t)j * n_in;
      // 4 products per lane per round, their 8 LDS reads issued together (clamped
      // addresses, masked values): one LDS round trip per 64 inputs, not per 16
      for (int i0 = 0; i0 < n_in; i0 += 64) {
        float p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = i0 + s + 16 * q, ic = min(i, n_in - 1);
          const float v = wr[ic] * x[ic];
          p[q] = i < n_in ? v : 0.f;
        }
        acc += (p[0] + p[1]) + (p[2] + p[3]);
      }
    }
    acc = row16_sum(acc);
    if (s == 0 && j < n_out) epi(j, acc);
  }
}

// grid: bmax workgroups (one per batch row); rows >= nb exit.
//
// Round trips: the kernel arguments, then ONE round for the prepared batch row
// (nb, doc, CSR extent), the step, the biases and the LDS-DMA staging of every MLP
// weight; then the row's (index, count) pairs and the W_in rows.  After the
// gather the whole MLP (hidden layers, dropout, mu / log-sigma heads) runs out of
// LDS with LDS-only barriers: its global stores are never waited on.
// Staged (compile-time): the MLP weights are read from LDS (ds_read); a runtime
// select between the LDS copy and global memory would make every read a flat load.
// NQM: the widest H0 class compiled in (outputs per lane, 64 NQM >= H0).  The H0 <= 64
// instance (NQM = 1) drops the wide paths' registers (87 -> <= 64 VGPRs): two workgroups
// fit a CU, so a batched launch's M bmax rows (512 at M = 8) run in one round on the 256
// CUs instead of two.
template <bool Staged, bool GB = false, int NQM = 8>
__global__ void __launch_bounds__(ENC_THREADS) __attribute__((amdgpu_waves_per_eu(NQM == 1 ? 8 : 1)))
gfk_enc_in_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = gfk_bx(), tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  int H0 = m.H[0], K = m.K, bmax = m.bmax, nh = m.n_hidden, input = m.input, sflags = m.stage_flags;
  const int32_t *nxt = m.ws_next, *indices = m.indices, *stepp = m.step;
  const float *values = m.values, *w_in = m.w_in, *b_in = m.b_in;
  keep(H0, K, bmax, nh, input, sflags, nxt, indices, stepp, values, w_in, b_in);
  const bool zs = m.ctx_fused == 2;       // ZeroShotTM: dense input layer fused here
  const int Hl = gfk_hlast(m), hm = enc_hmax(m);
  float* red = smem;
  float* act0 = red + ENC_WAVES * H0;
  float* act1 = act0 + pad4(hm);
  float* maskh = act1 + pad4(hm);
  float* labs = maskh + pad4(Hl);         // the row's labels (label head)
  float* wst = labs + (m.lab_on ? pad4(m.L) : 0);
  constexpr bool staged = Staged;

  GFK_STAMP(m, 4);
  // ---- one round: the row, the step, the weights (LDS-DMA), the biases ----
  if (staged) {
    float* p = wst;
#pragma unroll
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
      if (l + 1 < nh) {
        const int nw = m.H[l + 1] * m.H[l], nbias = m.H[l + 1];
        glds_copy(p, m.w_h[l], nw, tid, ENC_THREADS); p += pad4(nw);
        glds_copy(p, m.b_h[l], nbias, tid, ENC_THREADS); p += pad4(nbias);
      }
    }
    glds_copy(p, m.w_mu, K * Hl, tid, ENC_THREADS); p += pad4(K * Hl);
    glds_copy(p, m.b_mu, K, tid, ENC_THREADS); p += pad4(K);
    glds_copy(p, m.w_s, K * Hl, tid, ENC_THREADS); p += pad4(K * Hl);
    glds_copy(p, m.b_s, K, tid, ENC_THREADS);
  }
  const int nb = nxt[0];
  const int doc = nxt[1 + min(b, bmax - 1)];
  const int e0 = nxt[1 + bmax + 2 * b], e1 = nxt[2 + bmax + 2 * b];
  const int step = *stepp;
  const float bias = b_in[min(tid, H0 - 1)];
  // the row's non-zeros from its slots, in the same round: this lane's first gather
  // pair and the (tid, tid - 1) pair of the tile-start table
  const int cap = m.slot_cap;
  const int32_t* sidx = m.ws_sidx + (size_t)min(b, bmax - 1) * cap;
  const float* sval = m.ws_sval + (size_t)min(b, bmax - 1) * cap;
  const int gj = min(wave + ENC_WAVES * lane, cap - 1), tj = min(tid, cap - 1);
  const int gv = sidx[gj];
  const float gx = sval[gj];
  const int tv = sidx[tj], tvp = sidx[max(tj - 1, 0)];
  const int L = m.L;
  const float labv = m.lab_on ? m.labels[(size_t)doc * L + min(tid, L - 1)] : 0.f;
  __shared__ int last_tile;
  if (b >= nb) {            // drain the LDS-DMA before the workgroup retires
    vm_barrier();
    return;
  }
  if (m.lab_on && tid < L) {                 // the batch's label rows (classifier, W_in grads)
    labs[tid] = labv;
    m.ws_lab[(size_t)b * L + tid] = labv;
  }
  if (tid == 0) {           // publish the batch for the rest of the step
    m.ws_doc[b] = doc;
    m.ws_erange[2 * b] = e0;
    m.ws_erange[2 * b + 1] = e1;
    if (b == 0) *m.ws_nb = nb;
  }

  GFK_STAMP(m, 5);
  // ---- sparse gather (ZeroShotTM fused: the dense contextual input layer) ----
  if (zs) {
    float acc[NQM];
#pragma unroll
    for (int q = 0; q < NQM; ++q) acc[q] = 0.f;
    const float* xr = m.ctx + (size_t)doc * m.C;
    if constexpr (NQM == 1) gather_dense<1>(xr, m.C, wave, w_in, H0, lane, acc);
    else {
      if (H0 <= 64) gather_dense<1>(xr, m.C, wave, w_in, H0, lane, acc);
      else if (H0 <= 128) gather_dense<2>(xr, m.C, wave, w_in, H0, lane, acc);
      else if (H0 <= 256) gather_dense<4>(xr, m.C, wave, w_in, H0, lane, acc);
      else gather_dense<8>(xr, m.C, wave, w_in, H0, lane, acc);
    }
#pragma unroll
    for (int q = 0; q < NQM; ++q) {
      const int j = lane + 64 * q;
      if (j < H0) red[wave * H0 + j] = acc[q];
    }
  }
  if (input != GFK_IN_CONTEXTUAL) {
    float acc[NQM];
#pragma unroll
    for (int q = 0; q < NQM; ++q) acc[q] = 0.f;
    const int n = e1 - e0;
    if constexpr (NQM == 1) gather_slots<1>(sidx, sval, n, gv, gx, wave, w_in, H0, lane, acc);
    else {
      if (H0 <= 64) gather_slots<1>(sidx, sval, n, gv, gx, wave, w_in, H0, lane, acc);
      else if (H0 <= 128) gather_slots<2>(sidx, sval, n, gv, gx, wave, w_in, H0, lane, acc);
      else if (H0 <= 256) gather_slots<4>(sidx, sval, n, gv, gx, wave, w_in, H0, lane, acc);
      else gather_slots<8>(sidx, sval, n, gv, gx, wave, w_in, H0, lane, acc);
    }
    if (m.ctx_fused) {      // CombinedTM: the row's contextual partials from ctx_fwd (fixed order)
      const int P = m.ctx_parts > 0 ? m.ctx_parts : m.n_tiles;
      const size_t ps = (size_t)bmax * H0;
      const float* hp = m.ws_hpart + (size_t)b * H0;
      if (NQM == 1 || H0 <= 64) {
        // one column per lane: 16 partials in flight per wave (the per-tile partials of a
        // large vocabulary are ~100 per wave: a round trip per 4 of them was most of the
        // kernel), summed in the same order as below
        constexpr int PU = 16;
        const int jl = min(lane, H0 - 1);
        for (int p0 = wave; p0 < P; p0 += PU * ENC_WAVES) {
          float hv[PU];
#pragma unroll
          for (int u = 0; u < PU; ++u) hv[u] = hp[(size_t)min(p0 + u * ENC_WAVES, P - 1) * ps + jl];
#pragma unroll
          for (int u = 0; u < PU; ++u) acc[0] += p0 + u * ENC_WAVES < P ? hv[u] : 0.f;
        }
      } else
      for (int p0 = wave; p0 < P; p0 += 4 * ENC_WAVES) {
        float hv[4][NQM];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int p = min(p0 + u * ENC_WAVES, P - 1);
#pragma unroll
          for (int q = 0; q < NQM; ++q)
            hv[u][q] = 64 * q < H0 ? hp[(size_t)p * ps + min(lane + 64 * q, H0 - 1)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < NQM; ++q) acc[q] += p0 + u * ENC_WAVES < P ? hv[u][q] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < NQM; ++q) {
      const int j = lane + 64 * q;
      if (j < H0) red[wave * H0 + j] = acc[q];
    }
  }

  // ---- per vocab tile (64 words): the CSR position of the row's first non-zero
  //      (the tail past the row's last tile is filled after the next barrier) ----
  {
    int32_t* ts = m.ws_tstart + (size_t)b * (m.n_tiles + 1);
    const int n = e1 - e0;
    if (tid == 0 && n == 0) last_tile = -1;
    for (int j = tid; j < n; j += ENC_THREADS) {
      const int t = (j == tid ? tv : sidx[j]) >> 6;
      const int tp = j > 0 ? (j == tid ? tvp : sidx[j - 1]) >> 6 : -1;
      for (int u = tp + 1; u <= t; ++u) ts[u] = e0 + j;
      if (j == n - 1) last_tile = t;
    }
  }

  // ---- the row's random draws for this step ----
  for (int t = tid; t < 2 * K + Hl; t += ENC_THREADS) {
    if (t < K) {
      const uint32_t i = (uint32_t)(b * K + t);
      m.ws_eps[i] = randn(m.seed, (uint32_t)step, RNG_EPS, i);
    } else if (t < 2 * K) {
      const uint32_t i = (uint32_t)(b * K + t - K);
      m.ws_mask_t[i] = drop_scale(m.seed, (uint32_t)step, RNG_DROP_THETA, i, m.drop_theta);
    } else {
      const uint32_t i = (uint32_t)(b * Hl + t - 2 * K);
      const float s = drop_scale(m.seed, (uint32_t)step, RNG_DROP_ENC, i, m.drop_enc);
      m.ws_mask_h[i] = s;
      maskh[t - 2 * K] = s;
    }
  }
  vm_barrier();             // gather partials + staged weights
  GFK_STAMP(m, 6);
  {
    int32_t* ts = m.ws_tstart + (size_t)b * (m.n_tiles + 1);
    for (int u = last_tile + 1 + tid; u <= m.n_tiles; u += ENC_THREADS) ts[u] = e1;
  }
  GFK_STAMP(m, 44);

  // ---- input layer: z0 = sum of the wave partials + bias (+ dense contextual part) ----
  const int act = m.act;
  if (tid < H0) {
    float z = bias;
    if (input != GFK_IN_CONTEXTUAL || zs) {
#pragma unroll
      for (int w = 0; w < ENC_WAVES; ++w) z += red[w * H0 + tid];
    }
    if (input != GFK_IN_BOW && !m.ctx_fused) z += m.ws_hctx[(size_t)b * H0 + tid];
    if (m.lab_on && m.lab_in_enc) {          // the label block of the input layer
      const float* wl = w_in + (size_t)m.lab_off * H0 + tid;
      for (int l = 0; l < L; ++l) z += labs[l] * wl[(size_t)l * H0];
    }
    float zs;
    float a = act_train(act, z, m.seed, (uint32_t)step, 0, (uint32_t)(b * H0 + tid), &zs);
    m.ws_z[0][(size_t)b * H0 + tid] = zs;
    m.ws_a[0][(size_t)b * H0 + tid] = a;
    if (nh == 1) {
      a *= maskh[tid];
      m.ws_hd[(size_t)b * H0 + tid] = a;
    }
    act0[tid] = a;
  }
  lds_barrier();
  GFK_STAMP(m, 43);

  // ---- hidden layers ----
  float* ain = act0;
  float* aout = act1;
  const float* wcur = wst;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
    if (l + 1 >= nh) break;
    const int Hi = m.H[l], Ho = m.H[l + 1];
    const float* W = staged ? wcur : m.w_h[l];
    const float* Bv = staged ? wcur + pad4(Ho * Hi) : m.b_h[l];
    wcur += pad4(Ho * Hi) + pad4(Ho);
    const bool last = l + 2 == nh;
    float* zo = m.ws_z[l + 1] + (size_t)b * Ho;
    float* ao = m.ws_a[l + 1] + (size_t)b * Ho;
    float* hdo = m.ws_hd + (size_t)b * Ho;
    rowvec_gemv(W, ain, Ho, Hi, tid, [&](int j, float acc) {
      const float z = acc + Bv[j];
      float zs;
      float a = act_train(act, z, m.seed, (uint32_t)step, l + 1, (uint32_t)(b * Ho + j), &zs);
      zo[j] = zs;
      ao[j] = a;
      if (last) {
        a *= maskh[j];
        hdo[j] = a;
      }
      aout[j] = a;
    });
    GFK_STAMP(m, 45);
    lds_barrier();
    float* t = ain; ain = aout; aout = t;
  }

  GFK_STAMP(m, 7);
  // ---- mu / log-sigma heads (pre batch-norm) ----
  const float* Wmu = staged ? wcur : m.w_mu;
  const float* Bmu = staged ? wcur + pad4(K * Hl) : m.b_mu;
  const float* Ws = staged ? wcur + pad4(K * Hl) + pad4(K) : m.w_s;
  const float* Bs = staged ? wcur + 2 * pad4(K * Hl) + pad4(K) : m.b_s;
  float* mr = m.ws_mu_raw + (size_t)b * K;
  float* lr = m.ws_ls_raw + (size_t)b * K;
  rowvec_gemv(Wmu, ain, K, Hl, tid, [&](int k, float acc) { mr[k] = acc + Bmu[k]; });
  rowvec_gemv(Ws, ain, K, Hl, tid, [&](int k, float acc) { lr[k] = acc + Bs[k]; });
  GFK_STAMP(m, 39);
}

extern "C" int gfk_launch_enc_in(const GfkModel* m, hipStream_t s) {
  if (m->H[0] <= 64 && (m->stage_flags & 1)) {   // narrow, staged: two workgroups per CU
    if (m->n_batch > 1)
      hipLaunchKernelGGL((gfk_enc_in_k<true, true, 1>), gfk_grid(dim3(m->bmax), m), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<true>{gfk_dev(m)});
    else
      hipLaunchKernelGGL((gfk_enc_in_k<true, false, 1>), dim3(m->bmax), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<false>{*m});
    return (int)hipGetLastError();
  }
  if (m->H[0] <= 64) {                           // narrow, weights from L2 (large K plans)
    if (m->n_batch > 1)
      hipLaunchKernelGGL((gfk_enc_in_k<false, true, 1>), gfk_grid(dim3(m->bmax), m), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<true>{gfk_dev(m)});
    else
      hipLaunchKernelGGL((gfk_enc_in_k<false, false, 1>), dim3(m->bmax), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<false>{*m});
    return (int)hipGetLastError();
  }
  if (m->stage_flags & 1)
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_enc_in_k<true, true>), gfk_grid(dim3(m->bmax), m), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_enc_in_k<true, false>), dim3(m->bmax), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<false>{*m}); } while (0);
  else
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_enc_in_k<false, true>), gfk_grid(dim3(m->bmax), m), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_enc_in_k<false, false>), dim3(m->bmax), dim3(ENC_THREADS), gfk_enc_in_smem(m), s, GfkArgT<false>{*m}); } while (0);
  return (int)hipGetLastError();
}

extern "C" int gfk_enc_in_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)gfk_enc_in_k<true>, (const void*)gfk_enc_in_k<true, true>, (const void*)gfk_enc_in_k<false>, (const void*)gfk_enc_in_k<false, true>,
                      (const void*)gfk_enc_in_k<true, false, 1>,
                      (const void*)gfk_enc_in_k<true, true, 1>, (const void*)gfk_enc_in_k<false, false, 1>,
                      (const void*)gfk_enc_in_k<false, true, 1>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" size_t gfk_enc_weight_bytes(const GfkModel* m) {
  return sizeof(float) * (size_t)enc_weight_floats(*m);
}
