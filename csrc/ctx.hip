// CombinedTM contextual path on the fused kernels: adapt_bert and the contextual
// half of the input layer, forward and backward, with the adapt_bert Adam updates
// in the epilogue (reference ctm inference_network.py:160-185:
// z0 = [x_bow | adapt_bert(x_ctx)] W_in^T + b, adapt_bert(x) = x Wa^T + ba).
//
// Shapes: B (bmax) batch rows, V vocabulary, C contextual size, H0 first hidden
// width.  Wa [V, C], ba [V], Wc = rows V..2V-1 of the transposed input layer [2V, H0].
//
//   ctx_fwd (before enc_in), one workgroup per (vocab tile t, 16-row block r):
//       A_rt  = x_ctx[rows r] Wa[tile t]^T + ba[tile t]                      [16, 64]
//       P_rt  = A_rt Wc[tile t]                                              [16, H0]
//     C is walked in chunks of 128: the x_ctx rows and the Wa tile of a chunk are
//     loaded as coalesced float4 rows (two chunks in flight in registers) and
//     staged in LDS for the MFMA; the row blocks of one tile are dealt to the same
//     XCD so Wa[tile t] comes from HBM once per L2.  A is kept for the backward
//     (ws_actx); enc_in adds sum_t P_t to its row's pre-activation (fixed order:
//     deterministic).
//   ctx_bwd (after post_bwd, before win_update), grid n_tiles x kb, (tile t, chunk k):
//       dA_t  = dz0 Wc[tile t]^T                                             [B, 64]
//       g_ba  = sum_b dA_t                              (chunk 0; Adam on ba)
//       g_Wa  = dA_t^T x_ctx[:, chunk k]                (Adam on Wa[tile t, chunk k])
//     the g_Wa tile goes through LDS so the Adam epilogue moves p / m / v as
//     coalesced float4 rows (prefetched before the products).  Wc's own gradient
//     A^T dz0 is a dense tile of win_update (same MFMA + Adam epilogue as the
//     bag-of-words half), which runs after ctx_bwd has read Wc.
//
// All products are fp32 MFMA (v_mfma_f32_16x16x4_f32); operand tiles are staged in
// LDS with strides 2 mod 4 (A-role reads: 16 rows x 2 k per half-wave) or 16 mod 32
// (B-role reads: 2 rows x 16 columns), so every ds_read_b32 hits 32 distinct banks.
// In the backward the C dimension is split across workgroups so the grid covers the
// chip even for a small vocabulary; that split also spreads the Wa Adam traffic
// (p / m / v of V x C floats), which is what bounds it.
#define GFK_BATCHED_COPY 1   // batched kernels copy their descriptor (gfk_common.h gfk_model)
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int CT = 1024;
constexpr int CW = CT / 64;
constexpr int FT = 512;                 // forward workgroup
constexpr int FK = 128, LDK = 130;      // forward C chunk, its LDS stride (2 x odd)
__host__ __device__ inline int rup(int x, int m) { return (x + m - 1) / m * m; }
__host__ __device__ inline int stride_a(int w) {     // 2 x odd
  int s = rup(w, 2);
  return (s / 2) % 2 == 0 ? s + 2 : s;
}
__host__ __device__ inline int stride_b(int w) {     // 16 mod 32 (w: multiple of 16)
  return w % 32 == 16 ? w : w + 16;
}

// forward LDS: x_ctx chunk [16][LDK] + Wa chunk [64][LDK], the 2 C-half partials of
// A [2][16][68], A [16][66], Wc tile [64][ldc]
__host__ __device__ inline int fwd_ldc(const GfkModel& m) { return stride_b(rup(m.H[0], 16)); }
__host__ __device__ inline int fwd_lds_floats(const GfkModel& m) {
  return 80 * LDK + 2 * 16 * 68 + 16 * 66 + 64 * fwd_ldc(m);
}

struct BwdLds {
  int ldz, ldxb, gs, dz, wc, da, xc, g, total;
};
__host__ __device__ inline BwdLds bwd_lds(const GfkModel& m) {
  BwdLds L;
  const int B = m.bmax;
  L.ldz = stride_a(rup(m.H[0], 4));
  L.ldxb = stride_b(m.ctx_ckb);
  L.gs = m.ctx_ckb + 4;                 // g_Wa tile rows: 4 x stride = 16 mod 32
  int o = 0;
  L.dz = o; o += B * L.ldz;
  L.wc = o; o += 64 * L.ldz;
  L.da = o; o += B * 80;
  L.xc = o; o += B * L.ldxb;
  L.g = L.da;                           // reuses dA / x_ctx once the products are done
  L.total = o > L.g + 64 * L.gs ? o : L.g + 64 * L.gs;
  return L;
}

// Split staging: reg_load issues the first NR * NT elements' loads into registers,
// reg_store writes them to LDS later (other loads can be issued in between) and
// copies any remainder (wide shapes) in further groups of NR loads per thread.
template <int NR, int NT = CT, typename Ld>
__device__ __forceinline__ void reg_load(float (&r)[NR], int n, Ld ld) {
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int i = (int)threadIdx.x + u * NT;
    r[u] = i < n ? ld(i) : 0.f;
  }
}
template <int NR, int NT = CT, typename Ld, typename St>
__device__ __forceinline__ void reg_store(const float (&r)[NR], int n, Ld ld, St st) {
#pragma unroll
  for (int u = 0; u < NR; ++u) {
    const int i = (int)threadIdx.x + u * NT;
    if (i < n) st(i, r[u]);
  }
  for (int base = NR * NT + (int)threadIdx.x; base < n; base += NR * NT) {
    float q[NR];
#pragma unroll
    for (int u = 0; u < NR; ++u) q[u] = base + u * NT < n ? ld(base + u * NT) : 0.f;
#pragma unroll
    for (int u = 0; u < NR; ++u)
      if (base + u * NT < n) st(base + u * NT, q[u]);
  }
}

__device__ __forceinline__ void st_f4_as_f2(float* p, const f32x4& x) {   // 8-byte aligned LDS
  reinterpret_cast<float2*>(p)[0] = make_float2(x[0], x[1]);
  reinterpret_cast<float2*>(p)[1] = make_float2(x[2], x[3]);
}
}  // namespace

// grid: 8 * ceil(n_tiles / 8) * (BM / 16) workgroups of 8 waves; workgroup x runs on
// XCD x % 8 and handles tile 8 (x / 8 / RB) + x % 8, row block (x / 8) % RB.
// Wave (vt, kh) = (wave & 3, wave >> 2): 16x16 output tile vt over half kh of each
// chunk.  Staging: thread element u (< 5) of a chunk is float4 (row, q) =
// ((tid + 512 u) / 32, (tid + 512 u) % 32): u = 0 covers the 16 x_ctx rows, u >= 1
// the 64 Wa rows, 32 consecutive lanes per 512-byte row segment.
template <int BM, bool GB = false>
__global__ void __launch_bounds__(FT) gfk_ctx_fwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int RB = BM / 16, SU = 5;
  const int x = gfk_bx(), jx = x >> 3, rb = jx % RB, tile = (jx / RB) * 8 + (x & 7);
  if (tile >= m.n_tiles) return;
  GFK_STAMP(m, 30);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int vt = wave & 3, kh = wave >> 2, r = lane & 15, g = lane >> 4;
  const int V = m.V, C = m.C, H0 = m.H[0];
  const int c0 = tile * 64, nvv = min(64, V - c0), H0P = rup(H0, 16), LDC = fwd_ldc(m);
  float* xs = smem;                      // [16][LDK], then Wa chunk [64][LDK]
  float* red = smem + 80 * LDK;          // [2][16][68]
  float* as = red + 2 * 16 * 68;         // [16][66]
  float* wc = as + 16 * 66;              // [64][LDC]
  const float* wcg = m.w_in + (size_t)V * H0;

  // ---- loads that do not depend on the chunk loop: Wc tile, bias, doc ids ----
  auto ld_wc = [&](int i) {
    const int vv = i / H0P, j = i - vv * H0P;
    return (vv < nvv && j < H0) ? wcg[(size_t)(c0 + vv) * H0 + j] : 0.f;
  };
  auto st_wc = [&](int i, float xv) { const int vv = i / H0P; wc[vv * LDC + i - vv * H0P] = xv; };
  float wcr[8];
  reg_load<8, FT>(wcr, 64 * H0P, ld_wc);
  const int bv = tid & 63;
  const float bias = bv < nvv ? m.b_a[c0 + bv] : 0.f;
  const int q4 = (tid & 31) * 4;
  const int doc = m.ws_next[1 + rb * 16 + (tid >> 5)];   // the batch prepared by the previous step
  const float* xrow = m.ctx + (size_t)doc * C + q4;
  const float* wrow[SU - 1];
  bool wok[SU - 1];
#pragma unroll
  for (int u = 1; u < SU; ++u) {
    const int vv = ((tid + FT * u) >> 5) - 16;
    wok[u - 1] = vv < nvv;
    wrow[u - 1] = m.w_a + (size_t)(c0 + min(vv, nvv - 1)) * C + q4;
  }
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto ld = [&](int c, f32x4 (&rg)[SU]) {
    const int k = c * FK;
    const bool kin = k + q4 < C;          // C % 4 == 0: whole float4 in or out
    rg[0] = kin ? *reinterpret_cast<const f32x4*>(xrow + k) : z4;
#pragma unroll
    for (int u = 1; u < SU; ++u)
      rg[u] = (kin && wok[u - 1]) ? *reinterpret_cast<const f32x4*>(wrow[u - 1] + k) : z4;
  };
  auto st = [&](const f32x4 (&rg)[SU]) {
#pragma unroll
    for (int u = 0; u < SU; ++u) st_f4_as_f2(xs + ((tid + FT * u) >> 5) * LDK + q4, rg[u]);
  };
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const float* ap = xs + r * LDK + kh * 64 + g;
  const float* bp = xs + (16 + vt * 16 + r) * LDK + kh * 64 + g;
  auto mma = [&]() {
#pragma unroll
    for (int k = 0; k < 64; k += 4) acc = mfma16x16x4(ap[k], bp[k], acc);
  };

  // ---- the C loop: chunk c in LDS, c + 1 and c + 2 in flight ----
  const int NC = (C + FK - 1) / FK;
  f32x4 ra[SU], rb2[SU];
  ld(0, ra);
  if (NC > 1) ld(1, rb2);
  reg_store<8, FT>(wcr, 64 * H0P, ld_wc, st_wc);
  st(ra);
  if (NC > 2) ld(2, ra);
  __syncthreads();
  GFK_STAMP(m, 31);
  for (int c = 0; c < NC; c += 2) {
    mma();
    if (c + 1 >= NC) break;
    __syncthreads();
    st(rb2);
    if (c + 3 < NC) ld(c + 3, rb2);
    __syncthreads();
    mma();
    if (c + 2 >= NC) break;
    __syncthreads();
    st(ra);
    if (c + 4 < NC) ld(c + 4, ra);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[(kh * 16 + g * 4 + i) * 68 + vt * 16 + r] = acc[i];
  __syncthreads();
  GFK_STAMP(m, 32);

  // ---- A = sum of the halves + bias: two elements per thread (16 x 64 = 2 FT) ----
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rr = (tid >> 6) + 8 * h;
    float a = red[rr * 68 + bv] + red[(16 + rr) * 68 + bv];
    a = bv < nvv ? a + bias : 0.f;
    as[rr * 66 + bv] = a;
    m.ws_actx[((size_t)tile * m.bmax + rb * 16 + rr) * 64 + bv] = a;
  }
  __syncthreads();

  // ---- P [16, H0] = A Wc_tile ----
  float* hg = m.ws_hpart + ((size_t)tile * m.bmax + rb * 16) * H0;
  for (int jt = wave; jt < H0P / 16; jt += FT / 64) {
    f32x4 p = {0.f, 0.f, 0.f, 0.f};
    const float* pa = as + r * 66 + g;
    const float* pb = wc + g * LDC + jt * 16 + r;
#pragma unroll 4
    for (int k = 0; k < 64; k += 4) p = mfma16x16x4(pa[k], pb[k * LDC], p);
    const int j = jt * 16 + r;
    if (j < H0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) hg[(g * 4 + i) * H0 + j] = p[i];
    }
  }
  GFK_STAMP(m, 33);
}

// Large vocabularies (stage_flags bit 5): ONE workgroup per vocab tile for ALL batch rows
// (B <= 64).  The row-block split above re-stages the tile's whole Wa block [64, C] for
// each 16-row block (4 x at B = 64: 1.2 GB of L2 -> LDS traffic at V = 99k for a
// 9.8 GFLOP product); here every Wa element is staged once and feeds 4x the MFMA work.
// Wave w owns output subtiles (row tile w >> 1, column strips 2 (w & 1), +1) of the
// [64, 64] tile over the full chunk; chunk c + 1 is in flight in registers while c is
// multiplied.  The Wc tile stays in registers through the C loop and is stored into
// the freed chunk buffers afterwards, so the LDS holds one chunk pair (67 KB: two
// workgroups per CU).
constexpr int CTX_FULL = 32;
template <bool GB = false>
__global__ void __launch_bounds__(FT) gfk_ctx_fwd_full_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int BMF = 64, SU = (BMF + 64) * FK / 4 / FT;     // float4 per thread per chunk: 8
  const int tile = gfk_bx();
  if (tile >= m.n_tiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int V = m.V, C = m.C, H0 = m.H[0], nb = *m.ws_nb;
  const int c0 = tile * 64, nvv = min(64, V - c0), H0P = rup(H0, 16), LDC = fwd_ldc(m);
  float* xs = smem;                      // [64 x_ctx rows + 64 Wa rows][LDK]
  float* as = smem;                      // after the loop: A [64][66]
  float* wc = smem + 64 * 66;            //                 Wc tile [64][LDC]
  const float* wcg = m.w_in + (size_t)V * H0;
  auto ld_wc = [&](int i) {
    const int vv = i / H0P, j = i - vv * H0P;
    return (vv < nvv && j < H0) ? wcg[(size_t)(c0 + vv) * H0 + j] : 0.f;
  };
  auto st_wc = [&](int i, float xv) { const int vv = i / H0P; wc[vv * LDC + i - vv * H0P] = xv; };
  float wcr[8];
  reg_load<8, FT>(wcr, 64 * H0P, ld_wc);
  const int bv = tid & 63;
  const float bias = bv < nvv ? m.b_a[c0 + bv] : 0.f;
  // staging element u of a chunk: float4 (row, q) = ((tid + FT u) / 32, (tid + FT u) % 32);
  // rows 0..63 the batch's x_ctx rows (rows >= nb read row 0: finite, never stored),
  // rows 64..127 the tile's Wa rows
  const int q4 = (tid & 31) * 4;
  const float* rowp[SU];
  bool rok[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int row = (tid + FT * u) >> 5;
    if (row < BMF) {
      const int doc = m.ws_next[1 + min(row, m.bmax - 1)];
      rowp[u] = m.ctx + (size_t)doc * C + q4;
      rok[u] = true;
    } else {
      const int vv = row - BMF;
      rowp[u] = m.w_a + (size_t)(c0 + min(vv, nvv - 1)) * C + q4;
      rok[u] = vv < nvv;
    }
  }
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  auto ld = [&](int c, f32x4 (&rg)[SU]) {
    const int k = c * FK;
    const bool kin = k + q4 < C;
#pragma unroll
    for (int u = 0; u < SU; ++u)
      rg[u] = (kin && rok[u]) ? *reinterpret_cast<const f32x4*>(rowp[u] + k) : z4;
  };
  auto st = [&](const f32x4 (&rg)[SU]) {
#pragma unroll
    for (int u = 0; u < SU; ++u) st_f4_as_f2(xs + ((tid + FT * u) >> 5) * LDK + q4, rg[u]);
  };
  const int rt = wave >> 1, cs0 = 2 * (wave & 1);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const float* ap = xs + (rt * 16 + r) * LDK + g;
  const float* bp0 = xs + (BMF + cs0 * 16 + r) * LDK + g;
  const float* bp1 = bp0 + 16 * LDK;
  auto mma = [&]() {
#pragma unroll
    for (int k = 0; k < FK; k += 4) {
      const float a = ap[k];
      acc0 = mfma16x16x4(a, bp0[k], acc0);
      acc1 = mfma16x16x4(a, bp1[k], acc1);
    }
  };
  const int NC = (C + FK - 1) / FK;
  f32x4 ra[SU];
  ld(0, ra);
  st(ra);
  if (NC > 1) ld(1, ra);
  __syncthreads();
  for (int c = 0; c < NC; ++c) {
    mma();
    if (c + 1 >= NC) break;
    __syncthreads();
    st(ra);
    if (c + 2 < NC) ld(c + 2, ra);
    __syncthreads();
  }
  __syncthreads();                       // every wave done with the chunk buffers
  // ---- A = acc + bias -> LDS (for P) and ws_actx (for ctx_bwd / win_update) ----
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f32x4& a4 = h ? acc1 : acc0;
    const int col = (cs0 + h) * 16 + r;
    const float bb = __shfl(bias, col, 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rt * 16 + g * 4 + i;
      const float a = col < nvv ? a4[i] + bb : 0.f;
      as[row * 66 + col] = a;
      if (row < m.bmax) m.ws_actx[((size_t)tile * m.bmax + row) * 64 + col] = a;
    }
  }
  reg_store<8, FT>(wcr, 64 * H0P, ld_wc, st_wc);
  __syncthreads();
  // ---- P [64, H0] = A Wc_tile: subtiles (row tile, column tile) dealt to the waves ----
  float* hg = m.ws_hpart + (size_t)tile * m.bmax * H0;
  const int NJT = H0P / 16;
  for (int t = wave; t < 4 * NJT; t += FT / 64) {
    const int prt = t / NJT, jt = t % NJT;
    f32x4 p = {0.f, 0.f, 0.f, 0.f};
    const float* pa = as + (prt * 16 + r) * 66 + g;
    const float* pb = wc + g * LDC + jt * 16 + r;
#pragma unroll 4
    for (int k = 0; k < 64; k += 4) p = mfma16x16x4(pa[k], pb[k * LDC], p);
    const int j = jt * 16 + r;
    if (j < H0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = prt * 16 + g * 4 + i;
        if (row < m.bmax) hg[(size_t)row * H0 + j] = p[i];
      }
    }
  }
  (void)nb;
}

// Register-streamed forward (stage_flags bit 15; B <= 64, H0 <= 64, at most 32 16-column
// units per workgroup).  The DMA-staged balanced variants of rounds 3-4 (removed in round 6;
// profiles/r4/ab_s8) moved every Wa slice AND the matching x_ctx slice through LDS once per
// 64-column chunk (x_ctx re-staged per
// chunk, a barrier per slice, and at most two slices = 1.7 us of Wa in flight per CU).  Here
// one 16-wave workgroup per CU owns a contiguous range of nu 16-column units; wave w owns
// units w and w + 16 of it, and computes A^T[v, b] = sum_k Wa[v, k] x[b, k] with Wa as the
// MFMA A operand straight from global memory into registers:
//  * lane (r, g) loads Wa[v = 16 unit + r][16 j + 4 g .. + 3] as ONE 128-bit buffer load per
//    16-float block j, consumed by 4 k steps x 4 batch-row tiles (16 MFMAs);
//  * a ring of RS_R = 4 blocks per wave (16 VGPRs) is refilled right after each block is
//    read, with the next block of this unit or the first ones of the wave's next (phase,
//    unit) segment: 4 blocks x 4 waves per SIMD of MFMA work to arrive (~4 us), 64 KB per CU;
//  * x_ctx, the batch's 64 rows, is the B operand from LDS in phases of 256 k (64 KB, two
//    buffers: phase p + 1 arrives by LDS-DMA while phase p is multiplied; quads XOR-swizzled
//    by (row & 15), so a ds_read_b128 of 16 rows x 4 quads hits every bank once); each phase
//    is staged ONCE per workgroup (one barrier per phase, 3 at C = 768) instead of per chunk;
//  * the accumulators of both units (32 VGPRs) live across the phases;
//  * balance: the unit is the grain, so a 25-unit workgroup (V = 99k) would give one SIMD
//    7 units and the others 6.  With nu = 16 + 4 q + 1 (17, 21, 25, 29) the last unit is
//    split by phase instead: phase p of it goes to helper wave 4 q + 1 + p % 3 (SIMDs 1..3,
//    waves with one full unit: their second accumulator), so the SIMDs carry 6, 6 1/3,
//    6 1/3, 6 1/3; the partials meet in LDS in the epilogue (fixed order: deterministic).
// Epilogue: A + bias -> ws_actx and, in [b][v] layout, into the freed LDS; then P^T[h, b] +=
// Wc^T A^T over the workgroup's words on the matrix cores (wave -> subtile (b tile, h tile),
// Wc from global in chunks of 8 k steps, the next chunk in flight): ONE z0 partial per
// workgroup in ws_hpart (ctx_parts = the grid), as the balanced kernels leave it.
constexpr int CTX_RS = 32768;
// RS_R: ring blocks per wave.  Interleaved at V = 99k (profiles/r4/ab_s9): 4 blocks
// 121.4 us, 8 blocks 124.9 us; 4 + the next block's x operands read before this block's
// MFMAs 121.1 us (not kept) -- the ring's depth and the LDS reads are not the limit: the
// busiest SIMD's MFMAs (main + P) are ~75 % of the kernel's cycles
constexpr int RS_T = 1024, RS_KP = 256, RS_R = 4, RS_AL = 512;
static_assert((RS_KP / 16) % RS_R == 0, "a segment's blocks cycle the ring whole");
// x phases / A [64][RS_AL] (the same 128 KB), + 3 split-unit partials [64][16]
__host__ __device__ inline int fwd_rs_lds_floats() { return 2 * 64 * RS_KP + 3 * 64 * 16; }
// BF (matmul_dtype = "bf16"): both GEMMs on v_mfma_f32_16x16x32_bf16 with fp32
// accumulation -- blocks j, j + 1 of a segment form one 32-k step (lane group g: the 8 k
// 16 j + 4 g + i, 16 (j + 1) + 4 g + i of its Wa row AND of x's row, any pairing of k
// works when A and B agree), Wa's pair converted once per step for the 4 row tiles; the
// epilogue's P^T = Wc^T A^T pairs word groups sq, sq + 1 the same way.  8x fewer MFMA
// instructions than the fp32 16x16x4 path, which bounds it (the Wa stream does not).
template <bool GB = false, bool BF = false>
__global__ void __launch_bounds__(RS_T) gfk_ctx_fwd_rs_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  GFK_STAMP(m, 30);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int r = lane & 15, g = lane >> 4;
  const int V = m.V, C = m.C, H0 = m.H[0], bmax = m.bmax;
  const int G = (int)gridDim.x, w = (int)gfk_bx();
  const int U = (V + 15) / 16;
  const int u0 = (int)((int64_t)w * U / G), nu = (int)((int64_t)(w + 1) * U / G) - u0;
  const int NPH = (C + RS_KP - 1) / RS_KP;
  const bool split = nu > 16 && (nu & 3) == 1;
  const int nuf = split ? nu - 1 : nu;              // full units
  const int hw0 = nuf - 15;                         // split: helpers hw0 .. hw0 + 2
  const bool full1 = wave + 16 < nuf;               // a second full unit
  const bool helper = split && wave >= hw0 && wave < hw0 + min(NPH, 3);
  const bool has0 = wave < nuf;
  // (phase, slot) segments of this wave; slot 1 = the second full unit, or a helper's
  // phases p of the split unit (p % 3 == wave - hw0)
  auto has = [&](int p, int t) { return t == 0 ? has0 : (full1 || (helper && p % 3 == wave - hw0)); };
  auto unit_of = [&](int t) { return t == 0 ? u0 + wave : (full1 ? u0 + wave + 16 : u0 + nuf); };
  constexpr uint32_t OOB = 0x80000000u;
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc((void*)m.ctx, 0, 0x7FFFFFFF, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc((void*)m.w_a, 0, (int)((uint32_t)V * (uint32_t)C * 4u), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_f = __builtin_amdgcn_make_buffer_rsrc((void*)m.flat_base, 0, 0x7FFFFFFF, 0x00020000);
  const uint32_t wc_off = (uint32_t)((m.w_in + (size_t)V * H0) - m.flat_base) * 4u;
  const uint32_t ba_off = (uint32_t)(m.b_a - m.flat_base) * 4u;
  // ---- x_ctx phase DMA: wave w moves rows 4 w .. 4 w + 3, one 1 KB row per instruction:
  //      LDS quad `lane` of row b <- global quad lane ^ (b & 15) of the phase ----
  uint32_t xrow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = 4 * wave + i;
    xrow[i] = b < bmax ? (uint32_t)m.ws_next[1 + b] * (uint32_t)C * 4u : OOB;
  }
  auto dma_x = [&](int p, float* buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = 4 * wave + i;
      const int k = p * RS_KP + 4 * (lane ^ (b & 15));
      const uint32_t off = (xrow[i] != OOB && k < C) ? xrow[i] + (uint32_t)k * 4u : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_x, (lds_void_ptr)(buf + b * RS_KP), 16, off, 0, 0, 0);
    }
  };
  // per-lane Wa offset of segment (p, t); past the last segment (p = NPH) and for words >= V
  // out of range: the loads return zeros
  auto seg_off = [&](int p, int t) -> uint32_t {
    if (p >= NPH) return OOB;
    const int v = unit_of(t) * 16 + r;
    return v < V ? ((uint32_t)v * (uint32_t)C + (uint32_t)(p * RS_KP + 4 * g)) * 4u : OOB;
  };
  // the segment after (p, t) in (phase, slot) order (p = NPH: none)
  auto succ = [&](int& p, int& t) {
    do {
      if (++t > 1) { t = 0; ++p; }
    } while (p < NPH && !has(p, t));
  };
  auto ldw = [&](uint32_t off, int j) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_w, off + 64u * j, 0, 0));
  };
  f32x4 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int bt = 0; bt < 4; ++bt) acc[t][bt] = z4;
  dma_x(0, smem);
  int pc = 0, tc = 0;                   // the first segment, then the one after it
  if (!has(0, 0)) succ(pc, tc);
  int pn = pc, tn = tc;
  succ(pn, tn);
  uint32_t offc = seg_off(pc, tc), offn = seg_off(pn, tn);
  f32x4 ring[RS_R];
  // (sched_barrier fences keep the loads in ring order and where they are written: the
  // scheduler otherwise sinks each refill to its use, 8 blocks later, under register
  // pressure -- and vmcnt counts in issue order)
#pragma unroll
  for (int q = 0; q < RS_R; ++q) {
    ring[q] = ldw(offc, q);
    __builtin_amdgcn_sched_barrier(0);
  }
  for (int p = 0; p < NPH; ++p) {
    // phase p's x: issued before every ring load still in flight (RS_R of them, issued
    // after it by any wave with a segment since; a wave without one may have issued none)
    if (has0 || helper) asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else vm_barrier();
    // (4 j + g) ^ r = 16 (j >> 2) + 4 ((j & 3) ^ (r >> 2)) + (g ^ (r & 3)): four lane
    // offsets, the rest immediates
    if (p == 0) GFK_STAMP(m, 31);
    if (p == NPH - 1) GFK_STAMP(m, 143);
    const float* xc = smem + (p & 1) * 64 * RS_KP + r * RS_KP + (g ^ (r & 3)) * 4;
    if (p + 1 < NPH) dma_x(p + 1, smem + ((p + 1) & 1) * 64 * RS_KP);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (has(p, t)) {
        if constexpr (BF) {
#pragma unroll
          for (int j = 0; j < RS_KP / 16; j += 2) {
            f32x4 xv[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int bt = 0; bt < 4; ++bt)
                xv[h][bt] = *reinterpret_cast<const f32x4*>(xc + bt * 16 * RS_KP + 64 * ((j + h) >> 2) + 16 * (((j + h) & 3) ^ (r >> 2)));
            const f32x4 w0v = ring[j % RS_R], w1v = ring[(j + 1) % RS_R];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int h = 0; h < 2; ++h)
              ring[(j + h) % RS_R] = j + h + RS_R < RS_KP / 16 ? ldw(offc, j + h + RS_R) : ldw(offn, j + h + RS_R - RS_KP / 16);
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8 wa = to_bf16x8(w0v, w1v);
#pragma unroll
            for (int bt = 0; bt < 4; ++bt) acc[t][bt] = mfma_bf16x8(wa, to_bf16x8(xv[0][bt], xv[1][bt]), acc[t][bt]);
          }
        } else {
#pragma unroll
        for (int j = 0; j < RS_KP / 16; ++j) {
          f32x4 xv[4];
#pragma unroll
          for (int bt = 0; bt < 4; ++bt)
            xv[bt] = *reinterpret_cast<const f32x4*>(xc + bt * 16 * RS_KP + 64 * (j >> 2) + 16 * ((j & 3) ^ (r >> 2)));
          const f32x4 wv = ring[j % RS_R];
          __builtin_amdgcn_sched_barrier(0);
          ring[j % RS_R] = j + RS_R < RS_KP / 16 ? ldw(offc, j + RS_R) : ldw(offn, j + RS_R - RS_KP / 16);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int bt = 0; bt < 4; ++bt) acc[t][bt] = mfma16x16x4(wv[i], xv[bt][i], acc[t][bt]);
        }
        }
        offc = offn;
        succ(pn, tn);
        offn = seg_off(pn, tn);
      }
    }
  }
  GFK_STAMP(m, 32);
  // ---- epilogue: the first Wc chunk in flight while A (+ bias) goes to ws_actx and LDS ----
  const int NJT = (H0 + 15) / 16;
  const int bt = wave & 3, ht = wave >> 2, hh = ht * 16 + r;
  auto ldwc = [&](f32x4 (&wc)[8], int c) {
#pragma unroll
    for (int sx = 0; sx < 8; ++sx)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int vl = 16 * (8 * c + sx) + 4 * g + i, v = u0 * 16 + vl;
        const uint32_t o = (vl < 16 * nu && v < V && hh < H0) ? wc_off + ((uint32_t)v * (uint32_t)H0 + (uint32_t)hh) * 4u : OOB;
        wc[sx][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_f, o, 0, 0));
      }
  };
  f32x4 wA[8], wB[8];
  if (ht < NJT) ldwc(wA, 0);
  // bias of the wave's full units; the split unit's (its summing wave: hw0)
  const bool summer = split && wave == hw0;
  f32x4 bias[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int v = (t == 0 ? u0 + wave : (full1 ? u0 + wave + 16 : u0 + nuf)) * 16 + 4 * g + i;
      const bool on = t == 0 ? has0 : (full1 || summer);
      bias[t][i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs_f, on && v < V ? ba_off + (uint32_t)v * 4u : OOB, 0, 0));
    }
  lds_barrier();                        // every wave done with the last phase's x
  GFK_STAMP(m, 140);
  float* al = smem;                     // [64 b][RS_AL v], quads XOR (b & 15)
  float* sp = smem + 2 * 64 * RS_KP;    // [3][64 b][16 v] split-unit partials
  // A of unit ul (+ bias) into LDS and ws_actx
  auto put_a = [&](int ul, const f32x4 (&a4)[4], const f32x4& bs) {
    const int v0 = (u0 + ul) * 16 + 4 * g;
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      const int b = b4 * 16 + r;
      f32x4 a;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = v0 + i < V ? a4[b4][i] + bs[i] : 0.f;
      *reinterpret_cast<f32x4*>(al + b * RS_AL + 4 * ((4 * ul + g) ^ r)) = a;
      if (b < bmax) {
        float* dst = m.ws_actx + ((size_t)(v0 >> 6) * bmax + b) * 64 + (v0 & 63);
        if (v0 + 3 < V) *reinterpret_cast<f32x4*>(dst) = a;
        else
#pragma unroll
          for (int i = 0; i < 4; ++i) if (v0 + i < V) dst[i] = a[i];
      }
    }
  };
  if (has0) put_a(wave, acc[0], bias[0]);
  if (full1) put_a(wave + 16, acc[1], bias[1]);
  if (helper) {                         // this helper's phases of the split unit
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4)
      *reinterpret_cast<f32x4*>(sp + ((wave - hw0) * 64 + b4 * 16 + r) * 16 + 4 * g) = acc[1][b4];
  }
  lds_barrier();
  if (summer) {                         // partials summed in helper order (fixed), + bias
    f32x4 a4[4];
#pragma unroll
    for (int b4 = 0; b4 < 4; ++b4) {
      a4[b4] = *reinterpret_cast<const f32x4*>(sp + (b4 * 16 + r) * 16 + 4 * g);
      for (int h = 1; h < min(NPH, 3); ++h) {
        const f32x4 q = *reinterpret_cast<const f32x4*>(sp + (h * 64 + b4 * 16 + r) * 16 + 4 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) a4[b4][i] += q[i];
      }
    }
    put_a(nuf, a4, bias[1]);
  }
  GFK_STAMP(m, 141);
  if (split) lds_barrier();
  GFK_STAMP(m, 142);
  // ---- P^T[h, b] over the workgroup's 16 nu words: k steps v = 16 s + 4 g + i ----
  f32x4 pacc = z4;
  if (ht < NJT) {
    auto part = [&](const f32x4 (&wc)[8], int c) {
      if constexpr (BF) {
        // (word groups past nu: Wc reads 0 there, and A is masked to 0 too)
#pragma unroll
        for (int sx = 0; sx < 8; sx += 2) {
          const int sq = 8 * c + sx;
          if (sq < nu) {
            f32x4 av[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              av[h] = *reinterpret_cast<const f32x4*>(al + (bt * 16 + r) * RS_AL + 4 * ((4 * (sq + h) + g) ^ r));
              if (sq + h >= nu) av[h] = z4;
            }
            pacc = mfma_bf16x8(to_bf16x8(wc[sx], wc[sx + 1]), to_bf16x8(av[0], av[1]), pacc);
          }
        }
      } else {
#pragma unroll
      for (int sx = 0; sx < 8; ++sx) {
        const int sq = 8 * c + sx;
        if (sq < nu) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(al + (bt * 16 + r) * RS_AL + 4 * ((4 * sq + g) ^ r));
#pragma unroll
          for (int i = 0; i < 4; ++i) pacc = mfma16x16x4(wc[sx][i], av[i], pacc);
        }
      }
      }
    };
    for (int c = 0; c < 4; c += 2) {
      if (8 * c >= nu) break;
      if (8 * (c + 1) < nu) ldwc(wB, c + 1);
      part(wA, c);
      if (8 * (c + 1) >= nu) break;
      if (8 * (c + 2) < nu) ldwc(wA, c + 2);
      part(wB, c + 1);
    }
    float* hg = m.ws_hpart + (size_t)w * bmax * H0;
    const int b = bt * 16 + r;
    if (b < bmax) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int h = ht * 16 + g * 4 + e;
        if (h < H0) hg[(size_t)b * H0 + h] = pacc[e];
      }
    }
  }
  GFK_STAMP(m, 33);
}

// grid: n_tiles * ctx_kb workgroups of 16 waves (one per CU).
template <int BM, bool GB = false>
__global__ void __launch_bounds__(CT) gfk_ctx_bwd_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int docs_s[BM];
  GFK_STAMP(m, 34);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int n_tiles = m.n_tiles, tile = gfk_bx() % n_tiles, kc = gfk_bx() / n_tiles;
  const int V = m.V, C = m.C, H0 = m.H[0], ckb = m.ctx_ckb;
  if (tid < BM) docs_s[tid] = m.ws_doc[tid];
  const int c0 = tile * 64, nvv = min(64, V - c0), k0 = kc * ckb, kn = min(ckb, C - k0);
  const int H0Q = rup(H0, 4);
  const BwdLds L = bwd_lds(m);
  float* dzs = smem + L.dz;
  float* wcs = smem + L.wc;
  float* das = smem + L.da;
  float* xcs = smem + L.xc;
  float* gs = smem + L.g;
  const float* wcg = m.w_in + (size_t)V * H0;
  const int nb = *m.ws_nb;
  const bool fused = m.update_mode == 1;
  const AdamCoef ac = adam_coef(m);     // (device loads: issued with the first round)

  // ---- one staging round, every load unconditional (clamped addresses; the masks are
  //      applied when the values reach LDS), so the compiler can count them: dz0 and the
  //      Wc tile, then the x_ctx chunk, then the Adam state p / m / v of the Wa block.
  //      Only the first three are waited for before the products; the 192 KB of Adam
  //      state is still arriving while dA and g_Wa run on the matrix cores. ----
  const float* dz0 = m.ws_dz[0];
  const int nbc = max(nb, 1);
  constexpr int SR = 4;                 // dz0 / Wc elements per thread (H0 <= 64: all of them)
  float rdz[SR], rwc[SR];
#pragma unroll
  for (int u = 0; u < SR; ++u) {
    const int i = tid + CT * u, r = i / H0Q, j = min(i - r * H0Q, H0 - 1);
    rdz[u] = dz0[min(r, nbc - 1) * H0 + j];
    rwc[u] = wcg[(size_t)(c0 + min(r, nvv - 1)) * H0 + j];
  }
  __syncthreads();          // docs_s
  constexpr int XU = (BM * 64 + CT - 1) / CT;   // float4 of the x_ctx chunk per thread
  const int NQ = ckb / 4;
  f32x4 rxc[XU];
#pragma unroll
  for (int u = 0; u < XU; ++u) {
    const int e = tid + CT * u, b = e / NQ, q = e - b * NQ;
    const int bc = min(b, min(nbc, BM) - 1), qc = min(4 * q, kn - 4);
    rxc[u] = *reinterpret_cast<const f32x4*>(m.ctx + (size_t)docs_s[bc] * C + k0 + qc);
  }
  // p / m / v: element u of a thread is (row, q) = (e / NQ, e % NQ), e = tid + 1024 u
  constexpr int MAXQ = 4;               // 64 x 256 / 4 / 1024
  f32x4 pp[MAXQ], pm[MAXQ], pv[MAXQ];
  int prow[MAXQ], pq[MAXQ];
#pragma unroll
  for (int u = 0; u < MAXQ; ++u) {
    const int e = tid + CT * u;
    prow[u] = e / NQ;
    pq[u] = e - prow[u] * NQ;
    const f32x4* p = reinterpret_cast<const f32x4*>(
        m.w_a + (size_t)(c0 + min(prow[u], nvv - 1)) * C + k0 + min(4 * pq[u], kn - 4));
    pp[u] = p[0];
    pm[u] = p[m.off_m / 4];
    pv[u] = p[m.off_v / 4];
  }
#pragma unroll
  for (int u = 0; u < SR; ++u) {
    const int i = tid + CT * u, r = i / H0Q, j = i - r * H0Q;
    if (r < BM) dzs[r * L.ldz + j] = (r < nb && j < H0) ? rdz[u] : 0.f;
    if (r < 64) wcs[r * L.ldz + j] = (r < nvv && j < H0) ? rwc[u] : 0.f;
  }
  for (int i = tid + CT * SR; i < max(BM, 64) * H0Q; i += CT) {   // wide input layers
    const int r = i / H0Q, j = i - r * H0Q;
    if (r < BM) dzs[r * L.ldz + j] = (r < nb && j < H0) ? dz0[r * H0 + j] : 0.f;
    if (r < 64) wcs[r * L.ldz + j] = (r < nvv && j < H0) ? wcg[(size_t)(c0 + r) * H0 + j] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < XU; ++u) {
    const int e = tid + CT * u, b = e / NQ, q = e - b * NQ;
    if (b < BM)
      *reinterpret_cast<f32x4*>(xcs + b * L.ldxb + 4 * q) =
          (b < nb && 4 * q < kn) ? rxc[u] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  GFK_STAMP(m, 35);

  // ---- dA [BM, 64] = dz0 Wc_tile^T ----
  constexpr int RT = BM / 16;
  for (int t = wave; t < RT * 4; t += CW) {
    const int rt = t >> 2, vt = t & 3;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const float* ap = dzs + (rt * 16 + (lane & 15)) * L.ldz + (lane >> 4);
    const float* bp = wcs + (vt * 16 + (lane & 15)) * L.ldz + (lane >> 4);
    for (int k = 0; k < H0Q; k += 4) acc = mfma16x16x4(ap[k], bp[k], acc);
#pragma unroll
    for (int r = 0; r < 4; ++r) das[(rt * 16 + (lane >> 4) * 4 + r) * 80 + vt * 16 + (lane & 15)] = acc[r];
  }
  lds_barrier();
  GFK_STAMP(m, 36);

  // ---- g_ba = column sums of dA (chunk 0): 16 lanes per column; its update (a global
  //      read-modify-write) waits until the end, so nothing here waits on the Wa state ----
  float gba = 0.f;
  if (kc == 0) {
    const int v = tid >> 4, sub = tid & 15;
    for (int b = sub; b < BM; b += 16) gba += das[b * 80 + v];
    gba = row16_sum(gba);
  }
  // ---- g_Wa [64, chunk] = dA^T x_ctx: wave tiles (vt, ct) = (t & 3, t >> 2),
  //      t = wave + 16 u, parked in registers until every wave has read dA / x_ctx ----
  const int NCT = ckb / 16;
  constexpr int MAXU = 4;               // ckb <= 256
  f32x4 gacc[MAXU];
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int t = wave + CW * u, vt = t & 3, ct = t >> 2;
    gacc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ct >= NCT) continue;
    const float* ap = das + (lane >> 4) * 80 + vt * 16 + (lane & 15);
    const float* bp = xcs + (lane >> 4) * L.ldxb + ct * 16 + (lane & 15);
    for (int b = 0; b < BM; b += 4) gacc[u] = mfma16x16x4(ap[b * 80], bp[b * L.ldxb], gacc[u]);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < MAXU; ++u) {
    const int t = wave + CW * u, vt = t & 3, ct = t >> 2;
    if (ct >= NCT) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      gs[(vt * 16 + (lane >> 4) * 4 + r) * L.gs + ct * 16 + (lane & 15)] = gacc[u][r];
  }
  __syncthreads();
  GFK_STAMP(m, 37);

  // ---- the update on coalesced float4 rows ----
  const bool sh = is_shared(m, m.w_a);
#pragma unroll
  for (int u = 0; u < MAXQ; ++u) {
    if (prow[u] >= nvv || 4 * pq[u] >= kn) continue;
    const f32x4 gr = *reinterpret_cast<const f32x4*>(gs + prow[u] * L.gs + 4 * pq[u]);
    f32x4* p = reinterpret_cast<f32x4*>(m.w_a + (size_t)(c0 + prow[u]) * C + k0 + 4 * pq[u]);
    if (!fused) {
      p[m.off_g / 4] = gr;
    } else {
      f32x4 np, mo = pm[u], vo = pv[u];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = mo[r], b2 = vo[r];
        float xv = adam_update(pp[u][r], gr[r], a, b2, ac);
        if (sh && m.fed_scale_on) xv *= m.fed_scale;
        mo[r] = a;
        vo[r] = b2;
        np[r] = xv;
      }
      p[m.off_m / 4] = mo;
      p[m.off_v / 4] = vo;
      p[0] = np;
    }
  }
  if (kc == 0) {
    const int v = tid >> 4;
    if ((tid & 15) == 0 && v < nvv) param_update(m, m.b_a + c0 + v, gba, ac, is_shared(m, m.b_a));
  }
  GFK_STAMP(m, 38);
}

// Persistent pipelined backward (stage_flags bit 12, B <= 64, H0 <= 64): ctx_bgrid
// workgroups of 16 waves (one per CU) walk contiguous ranges of the (tile, chunk) items
// (tile-major, chunks of PK = 128 floats of C), so every CU does the same Wa update
// traffic to within one item and never idles between workgroups: while item i's products
// and Adam epilogue run, item i + 1's Wa p / m / v quads and x_ctx slice are already in
// flight in a second register set (the (tile, chunk) grid started each workgroup's loads
// only after the previous workgroup on its CU had finished its stores, with its 115 KB of
// LDS leaving room for one).  dz0 is staged once per workgroup; dA = dz0 Wc_tile^T (and
// g_ba, on the tile's chunk-0 item) is recomputed only when the tile changes.
constexpr int CTX_BWDPP = 4096;
constexpr int PK = 128;                 // chunk of C per item
struct PPLds {
  int ldz, dz, wc, da, xc, gs, total;
};
__host__ __device__ inline PPLds pp_lds(const GfkModel& m) {
  PPLds L;
  L.ldz = stride_a(rup(m.H[0], 4));
  int o = 0;
  L.dz = o; o += 64 * L.ldz;
  L.wc = o; o += 64 * L.ldz;
  L.da = o; o += 64 * 80;
  L.xc = o; o += 64 * (PK + 16);        // B-role rows: stride 144 = 16 mod 32
  L.gs = o; o += 64 * (PK + 4);         // g_Wa tile rows: 4 x stride = 16 mod 32
  L.total = o;
  return L;
}
template <bool GB = false>
__global__ void __launch_bounds__(CT) gfk_ctx_bwd_pp_k(GfkArgT<GB> ga) {
  const GfkModel& m = gfk_model(ga);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int docs_s[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int V = m.V, C = m.C, H0 = m.H[0], n_tiles = m.n_tiles;
  const int NCK = (C + PK - 1) / PK;
  const int64_t N = (int64_t)n_tiles * NCK;
  const int G = (int)gridDim.x, w = (int)gfk_bx();
  const int i0 = (int)(N * w / G), i1 = (int)(N * (w + 1) / G);
  const int H0Q = rup(H0, 4);
  const PPLds L = pp_lds(m);
  float* dzs = smem + L.dz;
  float* wcs = smem + L.wc;
  float* das = smem + L.da;
  float* xcs = smem + L.xc;
  float* gs = smem + L.gs;
  const float* wcg = m.w_in + (size_t)V * H0;
  const int nb = *m.ws_nb;
  const bool fused = m.update_mode == 1;
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, m.w_a);
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  if (tid < 64) docs_s[tid] = m.ws_doc[min(tid, m.bmax - 1)];
  // ---- dz0 once (rows >= nb zero) ----
  for (int i = tid; i < 64 * H0Q; i += CT) {
    const int r = i / H0Q, j = i - r * H0Q;
    dzs[r * L.ldz + j] = (r < nb && j < H0) ? m.ws_dz[0][r * H0 + j] : 0.f;
  }
  __syncthreads();
  // ---- per-thread element maps: quad u (< 2) of the [64, PK] block = (row, q) ----
  int er[2], eq[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = tid + CT * u;
    er[u] = e >> 5;                      // PK / 4 = 32 quads per row
    eq[u] = e & 31;
  }
  // item loads: Wa p / m / v quads, the x_ctx slice and the tile's Wc rows (for dA when
  // the tile changes; L2 hits) -- clamped addresses, always issued
  auto ld_item = [&](int it, f32x4 (&P)[6], f32x4 (&X)[2], float (&W)[4]) {
    const int t = it / NCK, k0 = (it - t * NCK) * PK;
    const int c0 = t * 64, nvv = min(64, V - c0), kn = min(PK, C - k0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + CT * u, r = i / H0Q, j = i - r * H0Q;
      W[u] = wcg[(size_t)(c0 + min(r, nvv - 1)) * H0 + min(j, H0 - 1)];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const f32x4* p = reinterpret_cast<const f32x4*>(
          m.w_a + (size_t)(c0 + min(er[u], nvv - 1)) * C + k0 + min(4 * eq[u], kn - 4));
      P[3 * u] = p[0];
      P[3 * u + 1] = fused ? p[m.off_m / 4] : z4;
      P[3 * u + 2] = fused ? p[m.off_v / 4] : z4;
      X[u] = *reinterpret_cast<const f32x4*>(m.ctx + (size_t)docs_s[min(er[u], max(nb, 1) - 1)] * C + k0 +
                                             min(4 * eq[u], kn - 4));
    }
  };
  int cur_tile = -1;
  // one item: products + update, with the next item's loads already in flight
  // item part 1: its x_ctx slice into LDS and, for a new tile, dA (the Wc registers are
  // free afterwards: the next item's loads reuse them)
  auto stage = [&](int it, const f32x4 (&X)[2], const float (&W)[4]) {
    const int t = it / NCK, kc = it - t * NCK, k0 = kc * PK;
    const int c0 = t * 64, nvv = min(64, V - c0), kn = min(PK, C - k0);
    // the x_ctx slice -> LDS (rows >= nb, columns >= kn zero)
#pragma unroll
    for (int u = 0; u < 2; ++u)
      *reinterpret_cast<f32x4*>(xcs + er[u] * (PK + 16) + 4 * eq[u]) =
          (er[u] < nb && 4 * eq[u] < kn) ? X[u] : z4;
    if (t != cur_tile) {                 // (uniform) dA for the new tile
      cur_tile = t;
#pragma unroll
      for (int u = 0; u < 4; ++u) {      // 64 x H0Q <= 4096 = 4 CT
        const int i = tid + CT * u, r = i / H0Q, j = i - r * H0Q;
        if (r < 64) wcs[r * L.ldz + j] = (r < nvv && j < H0) ? W[u] : 0.f;
      }
      lds_barrier();
      {
        const int rt = wave >> 2, vt = wave & 3;      // 16 subtiles, one per wave
        f32x4 acc = z4;
        const float* ap = dzs + (rt * 16 + (lane & 15)) * L.ldz + (lane >> 4);
        const float* bp = wcs + (vt * 16 + (lane & 15)) * L.ldz + (lane >> 4);
        for (int k = 0; k < H0Q; k += 4) acc = mfma16x16x4(ap[k], bp[k], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) das[(rt * 16 + (lane >> 4) * 4 + r) * 80 + vt * 16 + (lane & 15)] = acc[r];
      }
    }
  };
  // item part 2: g_ba, g_Wa and the update
  auto compute = [&](int it, const f32x4 (&P)[6]) {
    const int t = it / NCK, kc = it - t * NCK, k0 = kc * PK;
    const int c0 = t * 64, nvv = min(64, V - c0), kn = min(PK, C - k0);
    lds_barrier();                       // x_ctx slice and dA visible
    // ---- g_ba (the tile's chunk-0 item): column sums of dA, 16 lanes per column ----
    if (kc == 0) {
      const int v = tid >> 4, sub = tid & 15;
      float gba = 0.f;
      for (int b = sub; b < 64; b += 16) gba += das[b * 80 + v];
      gba = row16_sum(gba);
      if (sub == 0 && v < nvv) param_update(m, m.b_a + c0 + v, gba, ac, is_shared(m, m.b_a));
    }
    // ---- g_Wa [64, PK] = dA^T x_ctx: subtiles t2 = wave, wave + 16 (vt, ct) = (t2 & 3, t2 >> 2) ----
    f32x4 gacc[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t2 = wave + 16 * u, vt = t2 & 3, ct = t2 >> 2;
      gacc[u] = z4;
      const float* ap = das + (lane >> 4) * 80 + vt * 16 + (lane & 15);
      const float* bp = xcs + (lane >> 4) * (PK + 16) + ct * 16 + (lane & 15);
#pragma unroll 4
      for (int b = 0; b < 64; b += 4) gacc[u] = mfma16x16x4(ap[b * 80], bp[b * (PK + 16)], gacc[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t2 = wave + 16 * u, vt = t2 & 3, ct = t2 >> 2;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        gs[(vt * 16 + (lane >> 4) * 4 + r) * (PK + 4) + ct * 16 + (lane & 15)] = gacc[u][r];
    }
    lds_barrier();
    // ---- the update on coalesced float4 rows ----
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (er[u] >= nvv || 4 * eq[u] >= kn) continue;
      const f32x4 gr = *reinterpret_cast<const f32x4*>(gs + er[u] * (PK + 4) + 4 * eq[u]);
      f32x4* p = reinterpret_cast<f32x4*>(m.w_a + (size_t)(c0 + er[u]) * C + k0 + 4 * eq[u]);
      if (!fused) {
        p[m.off_g / 4] = gr;
      } else {
        f32x4 np, mo = P[3 * u + 1], vo = P[3 * u + 2];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a = mo[r], b2 = vo[r];
          float xv = adam_update(P[3 * u][r], gr[r], a, b2, ac);
          if (sh && m.fed_scale_on) xv *= m.fed_scale;
          mo[r] = a;
          vo[r] = b2;
          np[r] = xv;
        }
        p[m.off_m / 4] = mo;
        p[m.off_v / 4] = vo;
        p[0] = np;
      }
    }
    lds_barrier();                       // before the next item rewrites the slice / dA / g tile
  };
  f32x4 PA[6], XA[2], PB[6], XB[2];
  float W[4];
  if (i0 < i1) ld_item(i0, PA, XA, W);
  for (int it = i0; it < i1; it += 2) {
    stage(it, XA, W);
    if (it + 1 < i1) ld_item(it + 1, PB, XB, W);
    compute(it, PA);
    if (it + 1 >= i1) break;
    stage(it + 1, XB, W);
    if (it + 2 < i1) ld_item(it + 2, PA, XA, W);
    compute(it + 1, PB);
  }
}

__host__ __device__ inline int fwd_full_lds_floats(const GfkModel& m) {
  const int a = 128 * LDK, b = 64 * 66 + 64 * fwd_ldc(m);
  return a > b ? a : b;
}

extern "C" size_t gfk_ctx_smem(const GfkModel* m) {
  size_t a = fwd_lds_floats(*m), b = bwd_lds(*m).total;
  if ((m->stage_flags & CTX_FULL) && (size_t)fwd_full_lds_floats(*m) > a) a = fwd_full_lds_floats(*m);
  if ((m->stage_flags & CTX_RS) && (size_t)fwd_rs_lds_floats() > a) a = fwd_rs_lds_floats();
  if ((m->stage_flags & CTX_BWDPP) && (size_t)pp_lds(*m).total > b) b = pp_lds(*m).total;
  return sizeof(float) * (a > b ? a : b);
}

extern "C" int gfk_ctx_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)gfk_ctx_fwd_k<16>, (const void*)gfk_ctx_fwd_k<16, true>, (const void*)gfk_ctx_fwd_k<32>, (const void*)gfk_ctx_fwd_k<32, true>,
                      (const void*)gfk_ctx_fwd_k<64>, (const void*)gfk_ctx_fwd_k<64, true>, (const void*)gfk_ctx_fwd_k<128>, (const void*)gfk_ctx_fwd_k<128, true>,
                      (const void*)gfk_ctx_bwd_k<16>, (const void*)gfk_ctx_bwd_k<16, true>, (const void*)gfk_ctx_bwd_k<32>, (const void*)gfk_ctx_bwd_k<32, true>,
                      (const void*)gfk_ctx_bwd_k<64>, (const void*)gfk_ctx_bwd_k<64, true>, (const void*)gfk_ctx_bwd_k<128>, (const void*)gfk_ctx_bwd_k<128, true>,
                      (const void*)gfk_ctx_fwd_full_k<false>, (const void*)gfk_ctx_fwd_full_k<true>,
                      (const void*)gfk_ctx_bwd_pp_k<false>, (const void*)gfk_ctx_bwd_pp_k<true>,
                      (const void*)gfk_ctx_fwd_rs_k<false>, (const void*)gfk_ctx_fwd_rs_k<true>,
                      (const void*)gfk_ctx_fwd_rs_k<false, true>, (const void*)gfk_ctx_fwd_rs_k<true, true>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

// Host checks mirror the kernels' assumptions: the backward chunk a multiple of 16
// and <= 256 (prefetch slots), H0 <= 512, float4-aligned contextual rows / Wa.
static bool ctx_ok(const GfkModel* m) {
  return m->ctx_fused && m->ctx && m->ws_actx && m->ws_hpart && m->ctx_ckb > 0 &&
         m->ctx_ckb % 16 == 0 && m->ctx_ckb <= 256 && m->H[0] <= 512 && m->C % 4 == 0 &&
         (uintptr_t)m->ctx % 16 == 0 && (uintptr_t)m->w_a % 16 == 0 && m->off_m % 4 == 0 &&
         m->off_v % 4 == 0 && m->off_g % 4 == 0 &&
         (int64_t)m->ctx_kb * m->ctx_ckb >= m->C;
}

extern "C" int gfk_launch_ctx_fwd(const GfkModel* m, hipStream_t s) {
  if (!ctx_ok(m)) return -9;
  // register-streamed forward: at most 2 units per wave (32 per workgroup), 32-bit buffer
  // offsets into Wa and the flat buffer (engine checks), Wa rows 16-byte aligned
  if ((m->stage_flags & CTX_FULL) && (m->stage_flags & CTX_RS) && m->bmax <= 64 && m->H[0] <= 64 &&
      m->ctx_parts > 0 && ((m->V + 15) / 16 + m->ctx_parts - 1) / m->ctx_parts <= 32 &&
      (int64_t)m->V * m->C * 4 < 0x7FFFFFFFLL) {
    const dim3 g(m->ctx_parts), t(RS_T);
    const size_t sm = sizeof(float) * fwd_rs_lds_floats();
    if (m->mm_bf16)
      do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_rs_k<true, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_rs_k<false, true>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
    else
      do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_rs_k<true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_rs_k<false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
    return (int)hipGetLastError();
  }
  if ((m->stage_flags & CTX_FULL) && m->bmax <= 64) {
    const dim3 g(m->n_tiles), t(FT);
    const size_t sm = sizeof(float) * fwd_full_lds_floats(*m);
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_full_k<true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_full_k<false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
    return (int)hipGetLastError();
  }
  const dim3 g(8 * ((m->n_tiles + 7) / 8) * (m->bmax / 16)), t(FT);
  const size_t sm = sizeof(float) * fwd_lds_floats(*m);
  switch (m->bmax) {
    case 16: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_k<16, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_k<16, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 32: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_k<32, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_k<32, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 64: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_k<64, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_k<64, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 128: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_fwd_k<128, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_fwd_k<128, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_ctx_bwd(const GfkModel* m, hipStream_t s) {
  if (!ctx_ok(m)) return -9;
  if ((m->stage_flags & CTX_BWDPP) && m->bmax <= 64 && m->H[0] <= 64 && m->ctx_bgrid > 0) {
    const dim3 g(m->ctx_bgrid), t(CT);
    const size_t sm = sizeof(float) * pp_lds(*m).total;
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_bwd_pp_k<true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_bwd_pp_k<false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0);
    return (int)hipGetLastError();
  }
  const dim3 g(m->n_tiles * m->ctx_kb), t(CT);
  const size_t sm = sizeof(float) * bwd_lds(*m).total;
  switch (m->bmax) {
    case 16: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_bwd_k<16, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_bwd_k<16, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 32: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_bwd_k<32, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_bwd_k<32, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 64: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_bwd_k<64, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_bwd_k<64, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    case 128: do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_ctx_bwd_k<128, true>), gfk_grid(g, m), t, sm, s, GfkArgT<true>{gfk_dev(m)}); else hipLaunchKernelGGL((gfk_ctx_bwd_k<128, false>), g, t, sm, s, GfkArgT<false>{*m}); } while (0); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
