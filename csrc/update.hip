// The optimizer step of every encoder tensor, each fused with the kernel that
// completes its gradient, plus the next-batch prep.  Workgroup roles:
//   [0, n_tiles)         W_in tiles (below)
//   [n_tiles, +n_w)      small weight tiles: G[j][i] = sum_b dz[b][j] a[b][i] for a
//                        64 x 64 output tile of W_h[l] / W_mu / W_s (MFMA, fused Adam)
//   [.., +n_v)           bias / prior vectors: column sums over the batch (16 lanes
//                        per column, DPP reduction) or the prior gradient, fused Adam
//   last                 prepare_next_batch
// (beta is updated in prodlda_bwd's epilogue.)
//
// dW_in^T[v, :] = sum_b x[b, v] dz0[b, :]  (reference: autograd of
// inference_network.py:76 input_layer).  W_in is stored transposed ([V, H0]), so
// a vocabulary tile of 64 words is a contiguous [64, H0] block.  Instead of
// scattering B * nnz rows with float atomics (order-dependent, and each wave
// serialises on its outstanding-atomic budget), every workgroup owns one tile:
//   * builds the dense x^T tile [64, B] in LDS from the per-row tile start table
//     (ws_tstart, written by enc_in) -- the CSR non-zeros of the tile;
//   * multiplies it with dz0 [B, H0] on the fp32 matrix cores (16 waves, one
//     16x16 output tile each at H0 <= 64);
//   * applies Adam (and the FedAvg pre-scale) to its W_in block in the epilogue,
//     with p / m / v prefetched before the MFMA (fused mode), or stores the
//     gradient (gradient mode).
// Deterministic, no atomics, W_in's gradient is never materialised in fused mode.
// One extra workgroup prepares the next minibatch (gfk_common.h).
#define GFK_BATCHED_COPY 1   // batched kernels copy their descriptor (gfk_common.h gfk_model)
#include "gfk_common.h"

using namespace gfk;

namespace {
// Workgroup size UT: 16 waves when the grid fits the CUs (one round of workgroups: the
// most waves per tile, the shortest critical path -- the K=50 headline); 8 waves for
// large vocabularies, where the W_in tiles ([64, H0] blocks, 16 MFMA subtiles at H0 <= 64)
// outnumber the CUs several times: four workgroups share a CU and one's staging round
// overlaps another's MFMAs and stores.
__host__ __device__ inline int rup(int x, int m) { return (x + m - 1) / m * m; }
// LDS strides for ds_read_b32 MFMA operands (bank = dword % 32 per half-wave):
// A-role reads (lane & 15 -> row, lane >> 4 -> k) want stride = 2 x odd, so 16 rows x
// 2 k land on 32 distinct banks; B-role reads (lane >> 4 -> row, lane & 15 -> column)
// want stride = 16 mod 32, so a half-wave's 2 rows x 16 columns do.
__host__ __device__ inline int stride_a(int w) {
  int s = rup(w, 2);
  if ((s / 2) % 2 == 0) s += 2;
  return s;
}
__host__ __device__ inline int stride_b(int w) {   // w: multiple of 16
  return w % 32 == 16 ? w : w + 16;
}
}  // namespace

// weight jobs stage the batch in chunks of at most WJ_ROWS rows (large batches: several)
constexpr int WJ_ROWS = 128;

extern "C" size_t gfk_win_update_smem(const GfkModel* m) {
  const int B = m->bmax, H0P = rup(m->H[0], 16);
  // (the dense x^T tile path does not run at bmax > 128: the large-batch plan always takes
  // the sparse tiles)
  // (bmax > 128: the chunked dense tile, 128 rows at a time, win_tile_dense_ch)
  const int BR = B > WJ_ROWS ? WJ_ROWS : B;
  size_t a = (size_t)64 * stride_a(BR) + (size_t)BR * stride_b(H0P);
  const size_t b = 2 * (size_t)(B < WJ_ROWS ? B : WJ_ROWS) * 80;
  if (a < 64 * 64) a = 64 * 64;      // the flat epilogue's gradient tile [64, H0 <= 64]
  // the sparse tile (bit 4): dz0, the entry list, the row slots (+ the word mask and list)
  const size_t c = (size_t)B * m->H[0] + 2 * 512 + (B + 1 > 129 ? B + 1 : 129) + 128;
  if (a < c) a = c;
  // the dense contextual tile next to them (fused CombinedTM): dz0 + the A block / G tile,
  // rows at the padded stride (80 floats, win_tile_ctx)
  const size_t d = (size_t)B * 80 +
                   ((size_t)B * 80 > (size_t)64 * m->H[0] ? (size_t)B * 80 : (size_t)64 * m->H[0]);
  if (m->input == GFK_IN_COMBINED && a < d) a = d;
  return sizeof(float) * (a > b ? a : b);
}

// Small weight tile job (see GfkWJob).  LDS: dz[B][LDJ] + a[B][LDJ]
template <int UT>
__device__ __forceinline__ void weight_job(const GfkModel& m, const GfkWJob& J, float* smem) {
  constexpr int UW = UT / 64;
  constexpr int LDJ = 80;            // B-role stride (16 mod 32): conflict-free operand reads
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = m.bmax, nb = *m.ws_nb;
  float* dzs = smem;
  float* as = smem + B * LDJ;
  const bool fused = m.update_mode == 1;
  // prefetch: the lane's 4 outputs of subtiles (jt, it) = (t >> 2, t & 3), t = wave + UW u
  constexpr int WU = 16 / UW;
  float pp[WU][4], pm[WU][4], pv[WU][4];
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int t = wave + UW * u, jt = t >> 2, it = t & 3;
    const int i = J.i0 + it * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = J.j0 + jt * 16 + (lane >> 4) * 4 + r;
      const float* p = J.param + (size_t)min(j, J.rows - 1) * J.cols + min(i, J.cols - 1);
      pp[u][r] = pm[u][r] = pv[u][r] = 0.f;
      if (fused) { pp[u][r] = *p; pm[u][r] = p[m.off_m]; pv[u][r] = p[m.off_v]; }
    }
  }
  // stage the two [B x 64] column slices (rows >= nb zero)
  for (int e0 = 0; e0 < B * 64; e0 += 4 * UT) {
    float vz[4], va[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * UT + tid, b = min(e >> 6, B - 1), c = e & 63;
      vz[u] = J.dz[(size_t)b * J.rows + min(J.j0 + c, J.rows - 1)];
      va[u] = J.a[(size_t)b * J.cols + min(J.i0 + c, J.cols - 1)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * UT + tid, b = e >> 6, c = e & 63;
      if (b < B) {
        dzs[b * LDJ + c] = (b < nb && J.j0 + c < J.rows) ? vz[u] : 0.f;
        as[b * LDJ + c] = (b < nb && J.i0 + c < J.cols) ? va[u] : 0.f;
      }
    }
  }
  lds_barrier();
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, J.param);
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int t = wave + UW * u, jt = t >> 2, it = t & 3;
    const int i = J.i0 + it * 16 + (lane & 15);
    const float* ap = dzs + (lane >> 4) * LDJ + jt * 16 + (lane & 15);
    const float* bp = as + (lane >> 4) * LDJ + it * 16 + (lane & 15);
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < B; k += 8) {
      c0 = mfma16x16x4(ap[k * LDJ], bp[k * LDJ], c0);
      c1 = mfma16x16x4(ap[(k + 4) * LDJ], bp[(k + 4) * LDJ], c1);
    }
    const f32x4 g = c0 + c1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = J.j0 + jt * 16 + (lane >> 4) * 4 + r;
      if (j >= J.rows || i >= J.cols) continue;
      float* p = J.param + (size_t)j * J.cols + i;
      if (!fused) {
        p[m.off_g] = g[r];
      } else {
        float mo = pm[u][r], vo = pv[u][r];
        float np = adam_update(pp[u][r], g[r], mo, vo, ac);
        if (sh && m.fed_scale_on) np *= m.fed_scale;
        p[m.off_m] = mo;
        p[m.off_v] = vo;
        *p = np;
      }
    }
  }
}

// The large-batch plan's weight job (bmax > WJ_ROWS, gradient mode): the two [B x 64] column
// slices staged WJ_ROWS rows at a time, the MFMA accumulators carried over the chunks, the
// gradient stored.  LDS: dz[WJ_ROWS][LDJ] + a[WJ_ROWS][LDJ]
template <int UT>
__device__ __forceinline__ void weight_job_lb(const GfkModel& m, const GfkWJob& J, float* smem) {
  constexpr int UW = UT / 64, WU = 16 / UW;
  constexpr int LDJ = 80;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = m.bmax, nb = *m.ws_nb;
  float* dzs = smem;
  float* as = smem + WJ_ROWS * LDJ;
  f32x4 c0[WU], c1[WU];
#pragma unroll
  for (int u = 0; u < WU; ++u) c0[u] = c1[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int b0 = 0; b0 < B; b0 += WJ_ROWS) {
    if (b0) lds_barrier();             // the previous chunk's operand reads are done
    for (int e0 = 0; e0 < WJ_ROWS * 64; e0 += 4 * UT) {
      float vz[4], va[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * UT + tid, b = b0 + (e >> 6), c = e & 63;
        vz[u] = J.dz[(size_t)b * J.rows + min(J.j0 + c, J.rows - 1)];
        va[u] = J.a[(size_t)b * J.cols + min(J.i0 + c, J.cols - 1)];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = e0 + u * UT + tid, bl = e >> 6, b = b0 + bl, c = e & 63;
        dzs[bl * LDJ + c] = (b < nb && J.j0 + c < J.rows) ? vz[u] : 0.f;
        as[bl * LDJ + c] = (b < nb && J.i0 + c < J.cols) ? va[u] : 0.f;
      }
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < WU; ++u) {
      const int t = wave + UW * u, jt = t >> 2, it = t & 3;
      const float* ap = dzs + (lane >> 4) * LDJ + jt * 16 + (lane & 15);
      const float* bp = as + (lane >> 4) * LDJ + it * 16 + (lane & 15);
      for (int k = 0; k < WJ_ROWS; k += 8) {
        c0[u] = mfma16x16x4(ap[k * LDJ], bp[k * LDJ], c0[u]);
        c1[u] = mfma16x16x4(ap[(k + 4) * LDJ], bp[(k + 4) * LDJ], c1[u]);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < WU; ++u) {
    const int t = wave + UW * u, jt = t >> 2, it = t & 3;
    const int i = J.i0 + it * 16 + (lane & 15);
    const f32x4 g = c0[u] + c1[u];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = J.j0 + jt * 16 + (lane >> 4) * 4 + r;
      if (j < J.rows && i < J.cols) J.param[(size_t)j * J.cols + i + m.off_g] = g[r];
    }
  }
}

// Vector job (see GfkVJob): 16 lanes per element split the batch rows.  LB: the large-batch
// instance (rows in passes of 128)
template <int UT, bool LB = false>
__device__ __forceinline__ void vector_job(const GfkModel& m, const GfkVJob& J) {
  const int tid = threadIdx.x, s = tid & 15;
  const int B = m.bmax, nb = *m.ws_nb;
  const bool fused = m.update_mode == 1;
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, J.param);
  for (int c0 = 0; c0 < J.n; c0 += UT / 16) {
    const int c = c0 + (tid >> 4), cc = min(c, J.n - 1);
    float* p = J.param + cc;
    float pp = 0.f, pm = 0.f, pv = 0.f, g = 0.f;
    if (fused) { pp = *p; pm = p[m.off_m]; pv = p[m.off_v]; }
    if (J.src) {
      constexpr int RU = 8;                  // 8 rows per lane per pass (LB: B / 128 passes)
      float v[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) v[u] = J.src[(size_t)min(s + 16 * u, B - 1) * J.n + cc];
#pragma unroll
      for (int u = 0; u < RU; ++u) g += s + 16 * u < nb ? v[u] : 0.f;
      if constexpr (LB) {
        for (int r0 = 16 * RU; r0 < B; r0 += 16 * RU) {
#pragma unroll
          for (int u = 0; u < RU; ++u) v[u] = J.src[(size_t)min(r0 + s + 16 * u, B - 1) * J.n + cc];
#pragma unroll
          for (int u = 0; u < RU; ++u) g += r0 + s + 16 * u < nb ? v[u] : 0.f;
        }
      }
      g = row16_sum(g);
    } else {
      g = p[m.off_g];
    }
    if (s != 0 || c >= J.n) continue;
    if (!fused) {
      if (J.src) p[m.off_g] = g;
    } else {
      float np = adam_update(pp, g, pm, pv, ac);
      if (sh && m.fed_scale_on) np *= m.fed_scale;
      p[m.off_m] = pm;
      p[m.off_v] = pv;
      *p = np;
    }
  }
}

// Sparse W_in tile (stage_flags bit 4, large vocabularies: a 64-word tile holds only a
// few of the batch's non-zeros, ~7 at V = 112k).  The dense x^T tile + MFMA GEMM of the
// default path spends its staging on zero-filling and scattering a mostly empty [64, B]
// tile; here the tile's non-zeros become an entry list (rows in order, CSR order within a
// row: a scan of the rows' counts gives every row its slot range) and every thread
// accumulates its own elements of the flat [64, H0] block over the list,
//   G[v, h] = sum_{entries (b, v, x), b ascending} x dz0[b, h],
// a fixed order (deterministic, no atomics).  The W_in / m / v block moves as flat quads
// (one round, issued first); Adam (+ FedAvg pre-scale) or the gradient store follows.
// More entries than CAP are taken in passes of CAP (each thread's sums stay in registers).
constexpr int WIN_SPARSE = 16;
constexpr int WIN_BATCH8 = 512;
// VL: the second moment goes through LDS (one LDS-DMA copy of the block, issued with the
// other staging loads) instead of 2 quads of registers per thread, so the tile fits 64
// VGPRs and 4 workgroups per CU (fused mode; the launcher picks it when the block fits the
// kernel's existing LDS budget)
// RS: row slots per thread (64 rows each): 2 up to bmax = 128, GFK_BMAX_LIMIT / 64 for the
// large-batch plan
template <int UT, bool VL = false, int RS = 2>
__device__ __forceinline__ void win_tile_sparse(const GfkModel& m, float* smem, int tile) {
  constexpr int CAP = 512;
  constexpr int TPR = UT / 64;                 // threads per row, 64 rows per pass
  constexpr int FQ = 64 * 64 / 4 / UT;         // quads per thread (H0 <= 64)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = m.bmax, H0 = m.H[0], V = m.V, c0 = tile * 64;
  const int nb = *m.ws_nb;
  float* dz = smem;                            // [B][H0]
  int* ecol = reinterpret_cast<int*>(dz + B * H0);   // [CAP] (row << 8) | local column
  float* ex = reinterpret_cast<float*>(ecol + CAP);  // [CAP]
  int* offs = reinterpret_cast<int*>(ex + CAP);      // [64 RS + 1] rows' first slots, total
  float* vb = smem + ((B * H0 + 2 * CAP + 64 * RS + 1 + 3) & ~3);  // VL: [64 * H0] second moment
  float* wblk = m.w_in + (size_t)c0 * H0;
  const int nel = (min(V, c0 + 64) - c0) * H0;
  const bool fused = m.update_mode == 1;
  const bool al4 = ((uintptr_t)wblk % 16 == 0) && m.off_m % 4 == 0 && m.off_v % 4 == 0 &&
                   m.off_g % 4 == 0;
  auto ld4 = [&](const float* q, int e) {
    if (al4 && e + 3 < nel) return *reinterpret_cast<const f32x4*>(q + e);
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = e + i < nel ? q[e + i] : 0.f;
    return r;
  };
  // ---- one staging round.  Issue order matters (vmcnt counts in order): the rows' tile
  // extents first, so the dependent first-entry loads wait for them alone while the
  // block's p / m / v quads and dz0 stay in flight ----
  const int32_t* tst = m.ws_tstart;
  const int ntp = m.n_tiles + 1;
  const int sub = tid % TPR;
  int xe0[RS], xe1[RS], cnt[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) {             // rows tid / TPR (+ 64 i): the entry loads
    const int r = min(tid / TPR + 64 * i, B - 1);
    xe0[i] = tst[(size_t)r * ntp + tile];
    xe1[i] = tst[(size_t)r * ntp + tile + 1];
  }
#pragma unroll
  for (int i = 0; i < RS; ++i) {             // wave 0: rows lane (+ 64 i): the slot scan
    const int r = min(lane + 64 * i, B - 1);
    cnt[i] = wave == 0 ? tst[(size_t)r * ntp + tile + 1] - tst[(size_t)r * ntp + tile] : 0;
  }
  __builtin_amdgcn_sched_barrier(0);
  f32x4 pp[FQ], pm[FQ], pv[VL ? 1 : FQ];
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int e = 4 * (tid + UT * u);
    pp[u] = pm[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!VL) pv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (fused && e < nel) {
      pp[u] = ld4(wblk, e);
      pm[u] = ld4(wblk + m.off_m, e);
      if constexpr (!VL) pv[u] = ld4(wblk + m.off_v, e);
    }
  }
  if constexpr (VL) {
    if (!fused) {
    } else if (al4) {
      const int n4 = nel & ~3;
      glds_copy(vb, wblk + m.off_v, n4, tid, UT);
      if (tid < nel - n4) vb[n4 + tid] = wblk[m.off_v + n4 + tid];
    } else {
      for (int e = tid; e < nel; e += UT) vb[e] = wblk[m.off_v + e];
    }
  }
  glds_copy(dz, m.ws_dz[0], B * H0, tid, UT);
  __builtin_amdgcn_sched_barrier(0);
  // each thread's first entry of each of its rows (clamped, unconditional)
  int fi[RS];
  float fv[RS];
#pragma unroll
  for (int i = 0; i < RS; ++i) {
    const int e = min(xe0[i] + sub, max(xe1[i] - 1, 0));
    fi[i] = m.indices[e];
    fv[i] = m.values[e];
  }
  if (wave == 0) {             // row counts -> slots, rows in order
    int base = 0;
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const int c = lane + 64 * i < nb ? cnt[i] : 0;
      int x = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
      }
      offs[lane + 64 * i] = base + x - c;
      base += __shfl(x, 63, 64);
    }
    if (lane == 0) offs[64 * RS] = base;
  }
  vm_barrier();
  const int total = offs[64 * RS];
  // this thread's quads: word (row) v0 and column h0 of the first element; a quad spans at
  // most two words (H0 >= 4): elements with h0 + i >= H0 belong to word v0 + 1
  int qv[FQ], qh[FQ];
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int el = 4 * (tid + UT * u);
    qv[u] = el < nel ? el / H0 : -2;
    qh[u] = el % H0;
  }
  f32x4 g[FQ];
#pragma unroll
  for (int u = 0; u < FQ; ++u) g[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the list sums of one pass (fixed order: slots ascending)
  auto sums = [&](int n) {
    for (int j = 0; j < n; ++j) {
      const int cb = ecol[j];
      const float x = ex[j];
      const int col = cb & 255;
      const float* dr = dz + (cb >> 8) * H0;
#pragma unroll
      for (int u = 0; u < FQ; ++u) {
        const int d = col - qv[u];             // 0: this word, 1: the next one
        if (d == 0 || d == 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int h = qh[u] + i - d * H0;  // the element's column in word col
            if (h >= 0 && h < H0 && 4 * (tid + UT * u) + i < nel) g[u][i] = __builtin_fmaf(x, dr[h], g[u][i]);
          }
        }
      }
    }
  };
  // pass 0 from the staged registers (the first entries are already loaded); later passes
  // (more than CAP entries in the tile) re-read the rows' extents, so neither the extents
  // nor the first entries stay live across the sums
#pragma unroll
  for (int i = 0; i < RS; ++i) {
    const int r = tid / TPR + 64 * i;
    if (r >= nb) continue;
    const int o = offs[r] - xe0[i];
    int e = xe0[i] + sub;
    if (e < xe1[i] && o + e < CAP) {
      ecol[o + e] = (r << 8) | (fi[i] - c0);
      ex[o + e] = fv[i];
    }
    for (e += TPR; e < xe1[i] && o + e < CAP; e += TPR) {   // (rows with more than TPR entries)
      ecol[o + e] = (r << 8) | (m.indices[e] - c0);
      ex[o + e] = m.values[e];
    }
  }
  __syncthreads();
  sums(min(CAP, total));
  for (int p0 = CAP; p0 < total; p0 += CAP) {
    __syncthreads();                           // the previous pass's list reads are done
#pragma unroll
    for (int i = 0; i < RS; ++i) {
      const int r = tid / TPR + 64 * i;
      if (r >= nb) continue;
      const int a0 = tst[(size_t)r * ntp + tile], a1 = tst[(size_t)r * ntp + tile + 1];
      const int o = offs[r] - a0;
      for (int e = a0 + sub; e < a1; e += TPR) {
        const int s = o + e - p0;
        if (s >= 0 && s < CAP) {
          ecol[s] = (r << 8) | (m.indices[e] - c0);
          ex[s] = m.values[e];
        }
      }
    }
    __syncthreads();
    sums(min(CAP, total - p0));
  }
  // ---- update (fused: Adam + FedAvg pre-scale) or the gradient ----
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, m.w_in);
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int e = 4 * (tid + UT * u);
    if (e >= nel) break;
    f32x4 np, mo, vo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = pm[u][i], b;
      if constexpr (VL) b = e + i < nel ? vb[e + i] : 0.f;
      else b = pv[u][i];
      const float x = fused ? adam_update(pp[u][i], g[u][i], a, b, ac) : g[u][i];
      np[i] = sh && m.fed_scale_on && fused ? x * m.fed_scale : x;
      mo[i] = a;
      vo[i] = b;
    }
    auto st4 = [&](float* q, const f32x4& x) {
      if (al4 && e + 3 < nel) { *reinterpret_cast<f32x4*>(q + e) = x; return; }
#pragma unroll
      for (int i = 0; i < 4; ++i) if (e + i < nel) q[e + i] = x[i];
    };
    if (!fused) {
      st4(wblk + m.off_g, np);
    } else {
      st4(wblk + m.off_m, mo);
      st4(wblk + m.off_v, vo);
      st4(wblk, np);
    }
  }
}

// CombinedTM's contextual input-layer tile next to the sparse bag-of-words tiles (one
// launch, stage_flags bit 4 with ctx_fused == 1): Wc = rows V..2V-1 of the transposed
// input layer, G[v, h] = sum_{b < nb} A[b, v] dz0[b, h] with A the tile's adapted rows
// (ctx_fwd's ws_actx slab, [B][64]).  Both operand blocks arrive by LDS-DMA in their
// global layout ([B][64] and [B][H0], contiguous) -- no transposing scatter: the MFMA's
// reduction axis is b, and both roles read 16 consecutive columns of 4 rows per wave.
// The gradient tile is parked in the A block's LDS (free after the products) in the
// W block's flat order, and the epilogue moves p / m / v as flat quads prefetched before
// the products, like the sparse tile's.  B <= 64, H0 <= 64.
constexpr int WCS = 80;
template <int UT>
__device__ __forceinline__ void win_tile_ctx(const GfkModel& m, float* smem, int tile) {
  constexpr int UW = UT / 64;
  constexpr int FQ = 64 * 64 / 4 / UT;         // quads per thread (H0 <= 64)
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int B = m.bmax, H0 = m.H[0], V = m.V, c0 = tile * 64;
  const int nb = *m.ws_nb;
  // operand rows at stride WCS = 80 floats (16 mod 32): a half-wave's two rows of 16 columns
  // land on 32 distinct ds_read_b32 banks -- at the blocks' own strides (64, H0 = 50) the two
  // rows shared banks, half of the LDS cycles of the MFMA loop were conflicts (CombinedTM
  // K = 100: SQ_LDS_BANK_CONFLICT 49 % of SQ_LDS_IDX_ACTIVE, profiles/r4)
  float* dz = smem;                                       // [B][WCS]
  float* at = smem + B * WCS;                             // [B][WCS], then G [64][H0]
  float* wblk = m.w_in + (size_t)(V + c0) * H0;
  const int nel = (min(V, c0 + 64) - c0) * H0;
  const bool fused = m.update_mode == 1;
  const bool al4 = ((uintptr_t)wblk % 16 == 0) && m.off_m % 4 == 0 && m.off_v % 4 == 0 &&
                   m.off_g % 4 == 0;
  auto ld4 = [&](const float* q, int e) {
    if (al4 && e + 3 < nel) return *reinterpret_cast<const f32x4*>(q + e);
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = e + i < nel ? q[e + i] : 0.f;
    return r;
  };
  // ---- one staging round: the operand blocks (LDS-DMA, one dword per lane: a row per
  //      wave instruction, at the padded stride), then the W block's p / m / v ----
  {
    const float* ag = m.ws_actx + (size_t)tile * B * 64;
    for (int r = wave; r < B; r += UW) {
      if (lane < H0)
        __builtin_amdgcn_global_load_lds((gbl_void_ptr)(m.ws_dz[0] + r * H0 + lane),
                                         (lds_void_ptr)(dz + r * WCS), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((gbl_void_ptr)(ag + r * 64 + lane),
                                       (lds_void_ptr)(at + r * WCS), 4, 0, 0);
    }
  }
  f32x4 pp[FQ], pm[FQ], pv[FQ];
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int e = 4 * (tid + UT * u);
    pp[u] = pm[u] = pv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (fused && e < nel) {
      pp[u] = ld4(wblk, e);
      pm[u] = ld4(wblk + m.off_m, e);
      pv[u] = ld4(wblk + m.off_v, e);
    }
  }
  vm_barrier();
  // ---- G subtiles (v tile, h tile) = t = wave + UW u: rows b >= nb masked in the A role;
  //      columns h >= H0 read the row's padding (discarded outputs) ----
  const int NT = (H0 + 15) / 16, NST = 4 * NT;
  constexpr int SU = 16 / UW;                   // subtiles per wave (H0 <= 64: <= 16 in all)
  f32x4 acc[SU];
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int t = wave + UW * u;
    acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t >= NST) continue;
    const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
    const float* ap = at + (lane >> 4) * WCS + i0 + (lane & 15);
    const float* bp = dz + (lane >> 4) * WCS + j0 + (lane & 15);
    for (int k = 0; k < B; k += 4) {
      const float a = k + (lane >> 4) < nb ? ap[k * WCS] : 0.f;
      acc[u] = mfma16x16x4(a, bp[k * WCS], acc[u]);
    }
  }
  lds_barrier();                                // every wave is done reading the A block
#pragma unroll
  for (int u = 0; u < SU; ++u) {
    const int t = wave + UW * u;
    if (t >= NST) continue;
    const int i0 = (t / NT) * 16, j = (t % NT) * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (j < H0) at[(i0 + (lane >> 4) * 4 + r) * H0 + j] = acc[u][r];
  }
  lds_barrier();
  // ---- update (fused: Adam + FedAvg pre-scale) or the gradient, flat quads ----
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, m.w_in);
#pragma unroll
  for (int u = 0; u < FQ; ++u) {
    const int e = 4 * (tid + UT * u);
    if (e >= nel) break;
    f32x4 g;
#pragma unroll
    for (int i = 0; i < 4; ++i) g[i] = e + i < nel ? at[e + i] : 0.f;
    f32x4 np, mo, vo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float a = pm[u][i], b = pv[u][i];
      const float x = fused ? adam_update(pp[u][i], g[i], a, b, ac) : g[i];
      np[i] = sh && m.fed_scale_on && fused ? x * m.fed_scale : x;
      mo[i] = a;
      vo[i] = b;
    }
    auto st4 = [&](float* q, const f32x4& x) {
      if (al4 && e + 3 < nel) { *reinterpret_cast<f32x4*>(q + e) = x; return; }
#pragma unroll
      for (int i = 0; i < 4; ++i) if (e + i < nel) q[e + i] = x[i];
    };
    if (!fused) {
      st4(wblk + m.off_g, np);
    } else {
      st4(wblk + m.off_m, mo);
      st4(wblk + m.off_v, vo);
      st4(wblk, np);
    }
  }
}

// grid: n_tiles + n_w + n_v + 1 (+ n_tiles for fused CombinedTM, + ceil(C / 64) for fused
// ZeroShotTM) workgroups of 1024 threads.  The trailing tiles are the contextual input
// layer: CombinedTM's Wc = rows V..2V-1 of the transposed W_in with the dense adapted
// rows A^T (ctx_fwd's output) in place of x^T, or ZeroShotTM's whole [C, H0] layer with
// the batch's contextual rows x_ctx^T -- the same tile GEMM + Adam epilogue.
// dynamic LDS: max(W_in tile: xt[64][stride_a(B)] + dz[B][stride_b(H0P)], weight job: 2 B 80)
// (8-wave shape: at most 64 VGPRs, so the 4 workgroups its 37 KB of LDS allows per CU also
// fit the register file -- the batched instance compiled to 68 VGPRs, 7 waves per SIMD)
template <int UT, bool GB = false>
__global__ void __launch_bounds__(UT, UT == 512 ? 8 : 1) gfk_win_update_k(GfkArgT<GB> ga, GfkUArgT<GB> gua) {
  const GfkModel& m = gfk_model(ga);
  const GfkUpdate& U = gfk_upd(gua);
  constexpr int UW = UT / 64;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nt_here = m.n_tiles;
  {
    const int r = (int)gfk_bx() - nt_here;
    if (r >= 0 && r < U.n_w) { weight_job<UT>(m, U.w[r], smem); return; }
    if (r >= U.n_w && r < U.n_w + U.n_v) { vector_job<UT>(m, U.v[r - U.n_w]); return; }
    if (r == U.n_w + U.n_v) { prepare_next_batch(m, reinterpret_cast<int*>(smem)); return; }
  }
  const bool zs = m.ctx_fused == 2;            // ZeroShotTM: W_in is the dense [C, H0] layer
  if (m.input == GFK_IN_CONTEXTUAL && !zs) return;   // (host GEMMs when not fused)
  const int rr = (int)gfk_bx() - (nt_here + U.n_w + U.n_v + 1);
  const bool ctxt = rr >= 0;                   // a Wc tile (CombinedTM) / W tile (ZeroShotTM)
  if (zs && !ctxt) return;                     // ZeroShotTM has no bag-of-words half
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  int B = m.bmax, H0 = m.H[0], V = zs ? m.C : m.V, n_tiles = m.n_tiles;
  const int32_t *tstart = m.ws_tstart, *indices = m.indices, *nbp = m.ws_nb;
  const float *values = m.values, *dz0 = m.ws_dz[0];
  float* w_in = m.w_in + (ctxt && !zs ? (size_t)m.V * m.H[0] : 0);
  keep(B, H0, V, n_tiles, tstart, indices, nbp, values, dz0, w_in);
  const int H0P = rup(H0, 16);
  const int XS = stride_a(B), ZS = stride_b(H0P);
  float* xt = smem;
  float* dz = smem + 64 * XS;
  const int tile = ctxt ? rr : (int)gfk_bx(), c0 = tile * 64;

  GFK_STAMP(m, 40);
  // ---- staging: dz0 rows (zero padding), zero x^T tile, the tile's CSR extents ----
  const int nb = *nbp;
  if (H0P <= 64) {            // column tid % 64, rows tid / 64 + UT / 64 j: no runtime division
    const int c = tid & 63;
    if (c < H0P)
      for (int r = tid >> 6; r < B; r += UT / 64)
        dz[r * ZS + c] = (c < H0 && r < nb) ? dz0[r * H0 + c] : 0.f;
  } else {
    for (int i = tid; i < B * H0P; i += UT) {
      const int r = i / H0P, c = i % H0P;
      dz[r * ZS + c] = (c < H0 && r < nb) ? dz0[r * H0 + c] : 0.f;
    }
  }
  if (zs) {                   // x_ctx^T tile: the batch rows' contextual features
    for (int i = tid; i < B * 64; i += UT) {
      const int b = i >> 6, v = i & 63;
      xt[v * XS + b] = (b < nb && c0 + v < V) ? m.ctx[(size_t)m.ws_doc[b] * V + c0 + v] : 0.f;
    }
  } else if (ctxt) {          // A^T tile: the adapted rows (slab 0 of ctx_fwd's output)
    const float* ag = m.ws_actx + (size_t)tile * B * 64;
    for (int i = tid; i < B * 64; i += UT) {
      const int b = i >> 6, v = i & 63;
      xt[v * XS + b] = b < nb ? ag[i] : 0.f;
    }
  } else {
    for (int i = tid; i < 64 * XS; i += UT) xt[i] = 0.f;
  }
  // 16 threads per row: the row's non-zeros inside this tile (rows tid/16 + 32 i,
  // i < B / 32 -- the tile-start loads of every row are issued in the staging round)
  constexpr int XR = 128 / (UT / 16);          // row slots per thread (bmax <= 128)
  const int row = tid >> 4, sub = tid & 15;
  int xe0[XR], xe1[XR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int r = row + i * (UT / 16);
    xe0[i] = xe1[i] = 0;
    if (!ctxt && r < nb && r < B) {
      const int32_t* ts = tstart + (size_t)r * (n_tiles + 1) + tile;
      xe0[i] = ts[0];
      xe1[i] = ts[1];
    }
  }
  // prefetch the optimizer state of this lane's outputs: subtiles t = wave + UW u
  // (16x16 each; H0 <= 64 -> at most 16 subtiles, one pass; wider layers take passes
  // of UW * PU subtiles below, the later ones prefetched after the scatter)
  const int MT = 4, NT = H0P / 16;
  constexpr int PU = 16 / UW;
  float pp[PU][4], pm[PU][4], pv[PU][4];
  const bool fused = m.update_mode == 1;
  // FLAT (H0 <= 64, one pass): a tile's W_in block [64, H0] is contiguous, so the
  // epilogue moves p / m / v as flat quads (float4 when 16-B aligned): every load /
  // store instruction covers whole cache lines, instead of the MFMA output layout's
  // 4 rows x 64 B.  The gradient tile goes through LDS (the x^T buffer, free after the
  // MFMAs).  Quad q of the block is thread (q % UT)'s slot q / UT.
  // (the 8-wave large-vocabulary shape only: with one round of 16-wave workgroups the
  // extra LDS pass and barriers measured slower than the bytes they save)
  const bool flat = UT == 512 && NT <= 4;
  const int nel = (min(V, c0 + 64) - c0) * H0;          // the block's elements
  float* wblk = w_in + (size_t)c0 * H0;
  const bool al4 = ((uintptr_t)wblk % 16 == 0) && m.off_m % 4 == 0 && m.off_v % 4 == 0 &&
                   m.off_g % 4 == 0;
  auto ld4 = [&](const float* q, int e) {      // elements e..e+3 of the block (bounded)
    if (al4 && e + 3 < nel) return *reinterpret_cast<const f32x4*>(q + e);
    f32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = e + i < nel ? q[e + i] : 0.f;
    return r;
  };
  constexpr int FQ = 64 * 64 / 4 / UT;         // quads per thread (H0 <= 64)
  static_assert(FQ <= PU, "flat epilogue reuses the prefetch registers");
  if (flat) {
#pragma unroll
    for (int u = 0; u < FQ; ++u) {
      const int e = 4 * (tid + UT * u);
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, b = a, c = a;
      if (fused && e < nel) { a = ld4(wblk, e); b = ld4(wblk + m.off_m, e); c = ld4(wblk + m.off_v, e); }
#pragma unroll
      for (int i = 0; i < 4; ++i) { pp[u][i] = a[i]; pm[u][i] = b[i]; pv[u][i] = c[i]; }
    }
  }
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    if (flat) break;
    const int t = wave + UW * u;
    const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
    const int j = min(j0 + (lane & 15), H0 - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = min(c0 + i0 + (lane >> 4) * 4 + r, V - 1);
      float* p = w_in + (size_t)v * H0 + j;
      pp[u][r] = pm[u][r] = pv[u][r] = 0.f;
      if (t < MT * NT && fused) {
        pp[u][r] = *p;
        pm[u][r] = p[m.off_m];
        pv[u][r] = p[m.off_v];
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int r = row + i * (UT / 16);
    for (int e = xe0[i] + sub; e < xe1[i]; e += 16) xt[(indices[e] - c0) * XS + r] = values[e];
  }
  __syncthreads();

  GFK_STAMP(m, 41);
  // ---- G[v, j] = sum_b xt[v, b] dz[b, j] and the update ----
  const AdamCoef ac = adam_coef(m);
  const bool sh = is_shared(m, w_in);
  f32x4 gk[PU];
  for (int pass = 0; pass * UW * PU < MT * NT; ++pass) {
  if (pass > 0) {             // wide input layers (H0 > 64): the next subtiles' state
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int t = pass * UW * PU + wave + UW * u;
      const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
      const int j = min(j0 + (lane & 15), H0 - 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int v = min(c0 + i0 + (lane >> 4) * 4 + r, V - 1);
        float* p = w_in + (size_t)v * H0 + j;
        pp[u][r] = pm[u][r] = pv[u][r] = 0.f;
        if (t < MT * NT && fused) {
          pp[u][r] = *p;
          pm[u][r] = p[m.off_m];
          pv[u][r] = p[m.off_v];
        }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int t = pass * UW * PU + wave + UW * u;
    if (t >= MT * NT) break;
    const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
    const float* ap = xt + (i0 + (lane & 15)) * XS + (lane >> 4);
    const float* bp = dz + (lane >> 4) * ZS + j0 + (lane & 15);
    f32x4 c0v = {0.f, 0.f, 0.f, 0.f}, c1v = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < B; k += 8) {
      c0v = mfma16x16x4(ap[k], bp[k * ZS], c0v);
      c1v = mfma16x16x4(ap[k + 4], bp[(k + 4) * ZS], c1v);
    }
    const f32x4 g = c0v + c1v;
    const int j = j0 + (lane & 15);
    if (flat) {               // park the gradient in registers until every wave is done
      gk[u] = g;
      continue;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = c0 + i0 + (lane >> 4) * 4 + r;
      if (v >= V || j >= H0) continue;
      float* p = w_in + (size_t)v * H0 + j;
      if (!fused) {
        p[m.off_g] = g[r];
      } else {
        float mo = pm[u][r], vo = pv[u][r];
        float np = adam_update(pp[u][r], g[r], mo, vo, ac);
        if (sh && m.fed_scale_on) np *= m.fed_scale;
        p[m.off_m] = mo;
        p[m.off_v] = vo;
        *p = np;
      }
    }
  }
  }
  if (flat) {
    // the gradient tile [64, H0] into x^T's buffer in the block's own (flat) order
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int t = wave + UW * u;
      if (t >= MT * NT) break;
      const int i0 = (t / NT) * 16, j0 = (t % NT) * 16, j = j0 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (j < H0) xt[(i0 + (lane >> 4) * 4 + r) * H0 + j] = gk[u][r];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < FQ; ++u) {
      const int e = 4 * (tid + UT * u);
      if (e >= nel) break;
      const f32x4 g = *reinterpret_cast<const f32x4*>(xt + e);
      f32x4 np, mo, vo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float a = pm[u][i], b = pv[u][i];
        float x = fused ? adam_update(pp[u][i], g[i], a, b, ac) : g[i];
        np[i] = sh && m.fed_scale_on && fused ? x * m.fed_scale : x;
        mo[i] = a;
        vo[i] = b;
      }
      auto st4 = [&](float* q, const f32x4& x) {
        if (al4 && e + 3 < nel) { *reinterpret_cast<f32x4*>(q + e) = x; return; }
#pragma unroll
        for (int i = 0; i < 4; ++i) if (e + i < nel) q[e + i] = x[i];
      };
      if (!fused) {
        st4(wblk + m.off_g, np);
      } else {
        st4(wblk + m.off_m, mo);
        st4(wblk + m.off_v, vo);
        st4(wblk, np);
      }
    }
  }
  GFK_STAMP(m, 42);
}

// The large-batch plan's dense W_in tile (bmax > 128, gradient mode, H0 <= 64): the W_in
// tile body above with the batch taken in chunks of 128 rows -- per chunk the x^T tile
// [64][130] is rebuilt from the chunk rows' tile extents and dz0's chunk [128][ZS] staged,
// the MFMA accumulators carrying over (the small vocabularies' dense tiles: at V = 4.5k
// a 64-word tile holds ~700 of a 256-row batch's non-zeros, which the entry-list walk of the
// sparse tile serialises).  LDS: 64 x 130 + 128 x stride_b(H0) floats.
template <int UT>
__device__ __forceinline__ void win_tile_dense_ch(const GfkModel& m, float* smem, int tile) {
  constexpr int UW = UT / 64, RC = WJ_ROWS;
  constexpr int PU = 16 / UW;                  // subtiles per wave (H0 <= 64: 16 in all)
  constexpr int XR = RC / (UT / 16);           // row slots per thread per chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int B = m.bmax, H0 = m.H[0], V = m.V, n_tiles = m.n_tiles, c0 = tile * 64;
  const int nb = *m.ws_nb;
  const int H0P = rup(H0, 16), NT = H0P / 16, MT = 4;
  const int XS = stride_a(RC), ZS = stride_b(H0P);
  float* xt = smem;
  float* dz = smem + 64 * XS;
  const float* dz0 = m.ws_dz[0];
  const int row = tid >> 4, sub = tid & 15;
  f32x4 g[PU];
#pragma unroll
  for (int u = 0; u < PU; ++u) g[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int b0 = 0; b0 < B; b0 += RC) {
    if (b0) __syncthreads();                   // the previous chunk's operand reads are done
    {
      const int c = tid & 63;
      if (c < H0P)
        for (int r = tid >> 6; r < RC; r += UT / 64)
          dz[r * ZS + c] = (c < H0 && b0 + r < nb) ? dz0[(size_t)(b0 + r) * H0 + c] : 0.f;
    }
    for (int i = tid; i < 64 * XS; i += UT) xt[i] = 0.f;
    int xe0[XR], xe1[XR];
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int r = b0 + row + i * (UT / 16);
      xe0[i] = xe1[i] = 0;
      if (r < nb) {
        const int32_t* ts = m.ws_tstart + (size_t)r * (n_tiles + 1) + tile;
        xe0[i] = ts[0];
        xe1[i] = ts[1];
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int rl = row + i * (UT / 16);
      for (int e = xe0[i] + sub; e < xe1[i]; e += 16) xt[(m.indices[e] - c0) * XS + rl] = m.values[e];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int t = wave + UW * u;
      if (t >= MT * NT) break;
      const int i0 = (t / NT) * 16, j0 = (t % NT) * 16;
      const float* ap = xt + (i0 + (lane & 15)) * XS + (lane >> 4);
      const float* bp = dz + (lane >> 4) * ZS + j0 + (lane & 15);
      f32x4 c0v = {0.f, 0.f, 0.f, 0.f}, c1v = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < RC; k += 8) {
        c0v = mfma16x16x4(ap[k], bp[k * ZS], c0v);
        c1v = mfma16x16x4(ap[k + 4], bp[(k + 4) * ZS], c1v);
      }
      g[u] += c0v + c1v;
    }
  }
  float* w_in = m.w_in;
#pragma unroll
  for (int u = 0; u < PU; ++u) {
    const int t = wave + UW * u;
    if (t >= MT * NT) break;
    const int i0 = (t / NT) * 16, j = (t % NT) * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = c0 + i0 + (lane >> 4) * 4 + r;
      if (v < V && j < H0) w_in[(size_t)v * H0 + j + m.off_g] = g[u][r];
    }
  }
}

// the large-batch plan's update kernel with dense W_in tiles: job workgroups first, then the
// n_tiles chunked tiles
template <int UT>
__global__ void __launch_bounds__(UT) gfk_win_lb_k(GfkArgT<false> ga, GfkUArgT<false> gua) {
  const GfkModel& m = ga.m;
  const GfkUpdate& U = gua.u;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int r = (int)blockIdx.x;
  if (r < U.n_w) { weight_job_lb<UT>(m, U.w[r], smem); return; }
  if (r < U.n_w + U.n_v) { vector_job<UT, true>(m, U.v[r - U.n_w]); return; }
  if (r == U.n_w + U.n_v) { prepare_next_batch(m, reinterpret_cast<int*>(smem)); return; }
  win_tile_dense_ch<UT>(m, smem, r - (U.n_w + U.n_v + 1));
}

// the sparse W_in tiles (stage_flags bit 4) as their own kernel: its register budget is
// its own (the job paths of gfk_win_update_k need ~86 VGPRs)
// grid: n_w + n_v + 1 job workgroups FIRST (they start with the tiles, not after them),
// then the n_tiles sparse W_in tiles (+ n_tiles dense contextual tiles: fused CombinedTM)
template <int UT, bool GB = false, bool VL = false, bool CTX = false, int RS = 2>
__global__ void __launch_bounds__(UT, VL ? 4096 / UT : 1) gfk_win_sparse_k(GfkArgT<GB> ga, GfkUArgT<GB> gua) {
  const GfkModel& m = gfk_model(ga);
  const GfkUpdate& U = gfk_upd(gua);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int r = (int)gfk_bx();
  if (r < U.n_w) {
    if constexpr (RS > 2) weight_job_lb<UT>(m, U.w[r], smem);
    else weight_job<UT>(m, U.w[r], smem);
    return;
  }
  if (r < U.n_w + U.n_v) { vector_job<UT, (RS > 2)>(m, U.v[r - U.n_w]); return; }
  if (r == U.n_w + U.n_v) { prepare_next_batch(m, reinterpret_cast<int*>(smem)); return; }
  const int t = r - (U.n_w + U.n_v + 1);
  if constexpr (CTX) {
    if (t >= m.n_tiles) { win_tile_ctx<UT>(m, smem, t - m.n_tiles); return; }
  }
  win_tile_sparse<UT, VL, RS>(m, smem, t);
}

// the sparse tile's LDS second-moment variant: fused mode, and the block fits the LDS the
// kernel is given anyway (gfk_win_update_smem: no occupancy lost to LDS); gradient mode and
// the large-batch plan keep the second moment in registers
static bool win_sparse_vl(const GfkModel* m) {
  if (m->update_mode != 1) return false;
  if (m->bmax > 128) return false;      // (the large-batch instance keeps it in registers)
  const size_t need = sizeof(float) * ((((size_t)m->bmax * m->H[0] + 2 * 512 + 129 + 3) & ~(size_t)3) +
                                       (size_t)64 * m->H[0]);
  return need <= gfk_win_update_smem(m);
}

#define GFK_WIN_SPARSE_LAUNCH(VL, CTX)                                                               \
  do {                                                                                           \
    if (m->n_batch > 1)                                                                          \
      hipLaunchKernelGGL((gfk_win_sparse_k<512, true, VL, CTX>), gfk_grid(gs, m), dim3(512),     \
                         gfk_win_update_smem(m), s, GfkArgT<true>{gfk_dev(m)},                   \
                         GfkUArgT<true>{reinterpret_cast<const GfkUpdate*>(m->dev_upd)});        \
    else                                                                                         \
      hipLaunchKernelGGL((gfk_win_sparse_k<512, false, VL, CTX>), gs, dim3(512),                 \
                         gfk_win_update_smem(m), s, GfkArgT<false>{*m}, GfkUArgT<false>{*u});    \
  } while (0)

#define GFK_WIN_SPARSE_LB_LAUNCH()                                                                   \
  do {                                                                                           \
    constexpr int RSL = GFK_BMAX_LIMIT / 64;                                                     \
    if (m->n_batch > 1)                                                                          \
      hipLaunchKernelGGL((gfk_win_sparse_k<512, true, false, false, RSL>), gfk_grid(gs, m),     \
                         dim3(512), gfk_win_update_smem(m), s, GfkArgT<true>{gfk_dev(m)},        \
                         GfkUArgT<true>{reinterpret_cast<const GfkUpdate*>(m->dev_upd)});        \
    else                                                                                         \
      hipLaunchKernelGGL((gfk_win_sparse_k<512, false, false, false, RSL>), gs, dim3(512),       \
                         gfk_win_update_smem(m), s, GfkArgT<false>{*m}, GfkUArgT<false>{*u});    \
  } while (0)

extern "C" int gfk_launch_win_update(const GfkModel* m, const GfkUpdate* u, hipStream_t s) {
  const int extra = m->ctx_fused == 1 ? m->n_tiles : (m->ctx_fused == 2 ? (m->C + 63) / 64 : 0);
  if (m->stage_flags & WIN_SPARSE) {
    // bag-of-words inputs, or fused CombinedTM (its contextual half as dense tiles after
    // the sparse ones: B <= 64 so the operand blocks fit the kernel's LDS)
    const bool comb = m->input == GFK_IN_COMBINED && m->ctx_fused == 1;
    if (m->H[0] > 64 || m->bmax > (comb ? 64 : GFK_BMAX_LIMIT) || !(m->input == GFK_IN_BOW || comb))
      return -1;
    const dim3 gs(u->n_w + u->n_v + 1 + m->n_tiles * (comb ? 2 : 1));
    if (m->bmax > 128)
      GFK_WIN_SPARSE_LB_LAUNCH();
    else if (comb && win_sparse_vl(m))
      GFK_WIN_SPARSE_LAUNCH(true, true);
    else if (comb)
      GFK_WIN_SPARSE_LAUNCH(false, true);
    else if (win_sparse_vl(m))
      GFK_WIN_SPARSE_LAUNCH(true, false);
    else
      GFK_WIN_SPARSE_LAUNCH(false, false);
    return (int)hipGetLastError();
  }
  if (m->bmax > 128) {                 // large batches: the chunked dense tiles
    if (m->H[0] > 64 || m->update_mode != 0 || m->input != GFK_IN_BOW || m->n_batch > 1) return -1;
    const dim3 gl(u->n_w + u->n_v + 1 + m->n_tiles);
    hipLaunchKernelGGL((gfk_win_lb_k<1024>), gl, dim3(1024), gfk_win_update_smem(m), s, GfkArgT<false>{*m}, GfkUArgT<false>{*u});
    return (int)hipGetLastError();
  }
  const dim3 g(m->n_tiles + u->n_w + u->n_v + 1 + extra);
  // more W_in tiles than two rounds of 16-wave workgroups (dec_grid = the CUs' slots), or the
  // batched launch of several clients' tiles asks for the 8-wave shape (stage_flags bit 9,
  // set by BatchedSteps when all clients' tiles together exceed two rounds)
  if ((m->n_tiles > 2 * m->dec_grid && m->n_tiles > 512) || (m->stage_flags & WIN_BATCH8))
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_win_update_k<512, true>), gfk_grid(g, m), dim3(512), gfk_win_update_smem(m), s, GfkArgT<true>{gfk_dev(m)}, GfkUArgT<true>{reinterpret_cast<const GfkUpdate*>(m->dev_upd)}); else hipLaunchKernelGGL((gfk_win_update_k<512, false>), g, dim3(512), gfk_win_update_smem(m), s, GfkArgT<false>{*m}, GfkUArgT<false>{*u}); } while (0);
  else
    do { if (m->n_batch > 1) hipLaunchKernelGGL((gfk_win_update_k<1024, true>), gfk_grid(g, m), dim3(1024), gfk_win_update_smem(m), s, GfkArgT<true>{gfk_dev(m)}, GfkUArgT<true>{reinterpret_cast<const GfkUpdate*>(m->dev_upd)}); else hipLaunchKernelGGL((gfk_win_update_k<1024, false>), g, dim3(1024), gfk_win_update_smem(m), s, GfkArgT<false>{*m}, GfkUArgT<false>{*u}); } while (0);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// gfk_win_fold_k: the encoder update of M batched clients with their FedAvg fold in the
// epilogue (csrc/gfk_common.h GfkFold; the decoder half is prodlda.hip gfk_bwd_fold_k).
// Workgroup roles (256 threads), each walking the M clients in order and adding every
// client's pre-scaled Adam result to a register accumulator, written once at the end:
//   W_in      (tile, 16-column hidden slice): the x^T tile rebuilt from the client's tile
//             extents, dz0's slice, the 16x16 MFMA subtiles of gfk_win_update_k (B-step 8,
//             two accumulators), Adam with the client's m / v;
//   W         (weight job, 16-row slice): weight_job's products on the slice;
//   V         (vector job, 16-element pass): vector_job's column sums / the prior gradient;
//   left      pieces of the shared prefix no job owns (batch-norm running statistics,
//             already pre-scaled by the forward): the plain client-order sum;
//   prep      one per client: prepare_next_batch.
// The next client's loads are in flight while the current one computes; the vector and
// leftover roles load 8 clients at once.  Per client the arithmetic of the batched
// gfk_win_update_k<512> (dense x^T tiles: H0 <= 64, bmax == 64, bag-of-words input), then
// gfk_local_fedavg's client-order sum: bit-identical to that pair (tests/test_fold_gpu.py).
namespace {
constexpr int WF_NT = 256;
constexpr int WF_XS = 66;               // x^T tile stride: stride_a(64)
constexpr int WF_ZS = 16;               // a 16-column operand slice: rows 16 banks apart
constexpr int WF_LDJ = 80;
constexpr int WF_FG = 8;                // clients loaded at once by the vector / leftover roles
typedef const __attribute__((address_space(4))) GfkModel GfkModelC;
typedef const __attribute__((address_space(4))) GfkUpdate GfkUpdateC;
__device__ __forceinline__ GfkModelC& wf_model(const GfkFold& f, int c) {
  return ((GfkModelC*)(uintptr_t)f.models)[c];
}
__device__ __forceinline__ GfkUpdateC& wf_upd(const GfkFold& f, int c) {
  return ((GfkUpdateC*)(uintptr_t)f.upds)[c];
}
typedef const __attribute__((address_space(4))) GfkFoldClient GfkFoldClientC;
// a client's packed pointers (csrc/gfk_common.h GfkFoldClient): a few batched scalar loads
__device__ __forceinline__ GfkFoldClientC& wf_cl(const GfkFold& f, int c) {
  return ((GfkFoldClientC*)(uintptr_t)f.cl)[c];
}
__device__ __forceinline__ AdamCoef wf_coefp(GfkFoldClientC& P, float c0, float c1) {
  AdamCoef c;
  c.b1 = P.b1; c.b2 = P.b2; c.eps = P.eps; c.wd = P.wd;
  c.step = c0;
  c.ibc2 = c1;
  return c;
}

#ifdef GFK_STAMPS
#define WF_STAMP(slot)                                                            \
  do {                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                            \
    if (blockIdx.x == 0 && threadIdx.x == 0 && wf_model(f, 0).dbg)               \
      wf_model(f, 0).dbg[slot] = __builtin_amdgcn_s_memtime();                    \
    __builtin_amdgcn_sched_barrier(0);                                            \
  } while (0)
#else
#define WF_STAMP(slot) do { } while (0)
#endif
// W_in (tile, hidden slice js).  The tile extents run two clients ahead (the dependent
// first-non-zero loads one ahead), every store of the loop is an unconditional buffer store
// (elements outside the shapes get an offset past the descriptor): the loop top waits for the
// prefetched loads only, not for the previous client's stores.
__device__ __forceinline__ void wf_win(const GfkFold& f, float* smem, int tile, int js) {
  float* xt = smem;                       // [64][WF_XS]  x^T tile (zero outside the scatter)
  float* dzs = xt + 64 * WF_XS;           // [64][WF_ZS]  dz0[:, j0 .. j0 + 15]
  GfkModelC& m0 = wf_model(f, 0);
  const int M = f.M, V = m0.V, H0 = m0.H[0], n_tiles = m0.n_tiles, c0 = tile * 64, j0 = 16 * js;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = tid >> 2, sub = tid & 3;          // staging: row, 4 threads per row
  const int i0 = 16 * wave, jc = j0 + (lane & 15);  // MFMA subtile rows (words), output column
  const int nrec = V * H0 * 4;
  for (int i = tid; i < 64 * WF_XS / 4; i += WF_NT) reinterpret_cast<f32x4*>(xt)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the shared values of this thread's 4 outputs (every client's copy holds them)
  int eo[4], st[4];
  float pp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int v = c0 + i0 + (lane >> 4) * 4 + r;
    eo[r] = min(v, V - 1) * H0 + min(jc, H0 - 1);
    st[r] = v < V && jc < H0 ? 4 * eo[r] : 0x7FFF0000;
    pp[r] = m0.w_in[eo[r]];
  }
  struct Pre {
    int xe0, xe1, nb, xc[2];
    float xv[2], dz[4], pm[4], pv[4], cf0, cf1;
  };
  auto issue_ts = [&](int c, int& e0, int& e1) {
    const int32_t* ts = wf_cl(f, c).tstart + (size_t)row * (n_tiles + 1) + tile;
    e0 = ts[0];
    e1 = ts[1];
  };
  auto issue_nz = [&](int c, Pre& p) {
    GfkFoldClientC& P = wf_cl(f, c);
    const int32_t* indices = P.indices;
    const float* values = P.values;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = min(p.xe0 + sub + 4 * i, max(p.xe1 - 1, 0));
      p.xc[i] = indices[e];
      p.xv[i] = values[e];
    }
  };
  auto issue = [&](int c, Pre& p) {
    GfkFoldClientC& P = wf_cl(f, c);
    const int32_t* nbp = P.nb;
    const float *coef = P.coef, *dz0 = P.dz0, *wm = P.w_in_m, *wv = P.w_in_v;
    p.nb = *nbp;
    p.cf0 = coef[0];
    p.cf1 = coef[1];
    const float* d0 = dz0 + (size_t)row * H0;
#pragma unroll
    for (int i = 0; i < 4; ++i) p.dz[i] = d0[min(j0 + 4 * sub + i, H0 - 1)];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p.pm[r] = wm[eo[r]];
      p.pv[r] = wv[eo[r]];
    }
  };
  // a client's operands into LDS: dz0's slice (rows >= nb and columns >= H0 zero) and the
  // x^T scatter.  Runs at the end of the previous client's turn (and in the prologue): the
  // wait for its loads sits right behind that client's stores, the loop top never waits
  auto stage = [&](const Pre& p, int c) {
    const bool live = row < p.nb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = j0 + 4 * sub + i;
      dzs[row * WF_ZS + 4 * sub + i] = (j < H0 && live) ? p.dz[i] : 0.f;
    }
    const int xe1 = live ? p.xe1 : 0;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (p.xe0 + sub + 4 * i < xe1) xt[(p.xc[i] - c0) * WF_XS + row] = p.xv[i];
    GfkFoldClientC& P = wf_cl(f, c);
    for (int e = p.xe0 + sub + 8; e < xe1; e += 4) xt[(P.indices[e] - c0) * WF_XS + row] = P.values[e];
    // every other register of the client settles here (empty asm uses: the waits land now,
    // behind the previous client's stores, not inside the next turn)
    asm volatile("" ::"v"(p.nb), "v"(p.cf0), "v"(p.cf1), "v"(p.pm[0]), "v"(p.pm[1]), "v"(p.pm[2]), "v"(p.pm[3]));
    asm volatile("" ::"v"(p.pv[0]), "v"(p.pv[1]), "v"(p.pv[2]), "v"(p.pv[3]));
  };
  Pre cu, nx;
  int tn0, tn1, ts2a, ts2b;               // the tile extents of clients c + 1, c + 2
  issue_ts(0, cu.xe0, cu.xe1);
  issue(0, cu);
  issue_nz(0, cu);
  issue_ts(min(1, M - 1), tn0, tn1);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  WF_STAMP(300);
  lds_barrier();                          // the zeroed x^T tile
  stage(cu, 0);
  asm volatile("" ::"v"(tn0), "v"(tn1));  // (settled before the loop as at its latch)
  lds_barrier();
  WF_STAMP(301);
  for (int c = 0; c < M; ++c) {
    WF_STAMP(302 + 8 * c);
    GfkModelC& mc = wf_model(f, c);
    // ---- the next client's loads (unconditional, client indices clamped: a conditional
    //      load merging into a loop-carried register is a copy that waits for every load) ----
    {
      const int c1 = min(c + 1, M - 1);
      nx.xe0 = tn0;
      nx.xe1 = tn1;
      issue_nz(c1, nx);
      issue(c1, nx);
      issue_ts(min(c + 2, M - 1), ts2a, ts2b);
    }
    WF_STAMP(303 + 8 * c);
    // ---- G[v, j] = sum_b xt[v, b] dz[b, j] (gfk_win_update_k's subtile sequence) ----
    const float* ap = xt + (i0 + (lane & 15)) * WF_XS + (lane >> 4);
    const float* bp = dzs + (lane >> 4) * WF_ZS + (lane & 15);
    f32x4 c0v = {0.f, 0.f, 0.f, 0.f}, c1v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 64; k += 8) {
      c0v = mfma16x16x4(ap[k], bp[k * WF_ZS], c0v);
      c1v = mfma16x16x4(ap[k + 4], bp[(k + 4) * WF_ZS], c1v);
    }
    const f32x4 g = c0v + c1v;
    WF_STAMP(304 + 8 * c);
    lds_barrier();                        // every product read its operands
    WF_STAMP(305 + 8 * c);
    // ---- undo the scatter (the next client's tile starts from zeros); a row with more than
    //      8 entries in the tile clears its whole column instead of re-loading its entries ----
    {
      const int xe1 = row < cu.nb ? cu.xe1 : 0;
      if (xe1 - cu.xe0 > 8) {
        for (int v = sub; v < 64; v += 4) xt[v * WF_XS + row] = 0.f;
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          if (cu.xe0 + sub + 4 * i < xe1) xt[(cu.xc[i] - c0) * WF_XS + row] = 0.f;
      }
    }
    // ---- Adam with this client's moments, its pre-scale, the client-order sum ----
    GfkFoldClientC& P = wf_cl(f, c);
    const AdamCoef ac = wf_coefp(P, cu.cf0, cu.cf1);
    const float fs = P.win_sc;            // (1 where W_in is not shared: x * 1 = x)
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)P.w_in_m, 0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)P.w_in_v, 0, nrec, 0x00020000);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mo = cu.pm[r], vo = cu.pv[r];
      const float np = adam_update(pp[r], g[r], mo, vo, ac);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mo), rm, st[r], 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vo), rv, st[r], 0, 0);
      acc[r] = fold_add(acc[r], np, fs, c == 0);
    }
    WF_STAMP(306 + 8 * c);
    lds_barrier();                        // the undo is done before the next scatter
    WF_STAMP(307 + 8 * c);
    stage(nx, min(c + 1, M - 1));
    cu = nx;
    tn0 = ts2a;
    tn1 = ts2b;
    asm volatile("" ::"v"(tn0), "v"(tn1));
    WF_STAMP(308 + 8 * c);
    lds_barrier();
  }
  WF_STAMP(299);
  const int nw = f.mode == 1 ? 1 : M;
  for (int c = 0; c < nw; ++c) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wf_cl(f, c).w_in, 0, nrec, 0x00020000);
#pragma unroll
    for (int r = 0; r < 4; ++r) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r]), rw, st[r], 0, 0);
  }
}

// weight job jb, output rows J.j0 + 16 jt ..
__device__ __forceinline__ void wf_weight(const GfkFold& f, float* smem, int jb, int jt) {
  float* dzs = smem;                      // [64][WF_ZS] dz[:, row slice]
  float* as = smem + 64 * WF_ZS;          // [64][WF_LDJ] a[:, i0 .. i0 + 63]
  GfkModelC& m0 = wf_model(f, 0);
  GfkUpdateC& u0 = wf_upd(f, 0);
  const int M = f.M, B = m0.bmax;
  const int rows = u0.w[jb].rows, cols = u0.w[jb].cols, jr0 = u0.w[jb].j0 + 16 * jt, ic0 = u0.w[jb].i0;
  if (jr0 >= rows) return;
  const int tid = threadIdx.x, lane = tid & 63, it = tid >> 6;
  const int b = tid >> 2, sub = tid & 3;
  const int ic = ic0 + it * 16 + (lane & 15);
  const int nrec = rows * cols * 4;
  int eo[4], st[4];
  float pp[4];
  {
    const float* p0 = u0.w[jb].param;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jr0 + (lane >> 4) * 4 + r;
      eo[r] = min(j, rows - 1) * cols + min(ic, cols - 1);
      st[r] = j < rows && ic < cols ? 4 * eo[r] : 0x7FFF0000;
      pp[r] = p0[eo[r]];
    }
  }
  struct Pre {
    int nb;
    float dz[4], a[16], pm[4], pv[4], cf0, cf1;
  };
  auto issue = [&](int c, Pre& p) {
    GfkFoldClientC& P = wf_cl(f, c);
    const int32_t* nbp = P.nb;
    const float *coef = P.coef, *dzp = P.wdz[jb], *ap0 = P.wa[jb], *pm0 = P.wm[jb], *pv0 = P.wv[jb];
    p.nb = *nbp;
    p.cf0 = coef[0];
    p.cf1 = coef[1];
    const int bb = min(b, B - 1);
    const float* dz = dzp + (size_t)bb * rows;
    const float* a = ap0 + (size_t)bb * cols;
#pragma unroll
    for (int i = 0; i < 4; ++i) p.dz[i] = dz[min(jr0 + 4 * sub + i, rows - 1)];
#pragma unroll
    for (int i = 0; i < 16; ++i) p.a[i] = a[min(ic0 + 16 * sub + i, cols - 1)];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p.pm[r] = pm0[eo[r]];
      p.pv[r] = pv0[eo[r]];
    }
  };
  Pre nx;
  issue(0, nx);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < M; ++c) {
    GfkModelC& mc = wf_model(f, c);
    const Pre cu = nx;
    const bool live = b < cu.nb;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dzs[b * WF_ZS + 4 * sub + i] = (live && jr0 + 4 * sub + i < rows) ? cu.dz[i] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      as[b * WF_LDJ + 16 * sub + i] = (live && ic0 + 16 * sub + i < cols) ? cu.a[i] : 0.f;
    lds_barrier();
    issue(min(c + 1, M - 1), nx);          // (unconditional: see wf_win)
    const float* ap = dzs + (lane >> 4) * WF_ZS + (lane & 15);
    const float* bp = as + (lane >> 4) * WF_LDJ + it * 16 + (lane & 15);
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < B; k += 8) {
      c0 = mfma16x16x4(ap[k * WF_ZS], bp[k * WF_LDJ], c0);
      c1 = mfma16x16x4(ap[(k + 4) * WF_ZS], bp[(k + 4) * WF_LDJ], c1);
    }
    const f32x4 g = c0 + c1;
    GfkFoldClientC& P = wf_cl(f, c);
    const AdamCoef ac = wf_coefp(P, cu.cf0, cu.cf1);
    const float fs = P.wsc[jb];
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)P.wm[jb], 0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)P.wv[jb], 0, nrec, 0x00020000);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mo = cu.pm[r], vo = cu.pv[r];
      const float np = adam_update(pp[r], g[r], mo, vo, ac);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mo), rm, st[r], 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(vo), rv, st[r], 0, 0);
      acc[r] = fold_add(acc[r], np, fs, c == 0);
    }
    lds_barrier();                        // the products read their operands
  }
  const int nw = f.mode == 1 ? 1 : M;
  for (int c = 0; c < nw; ++c) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)wf_cl(f, c).wp[jb], 0, nrec, 0x00020000);
#pragma unroll
    for (int r = 0; r < 4; ++r) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r]), rw, st[r], 0, 0);
  }
}

// vector job jv, elements 16 pass .. 16 pass + 15 (16 lanes each)
__device__ __forceinline__ void wf_vector(const GfkFold& f, int jv, int pass) {
  GfkModelC& m0 = wf_model(f, 0);
  GfkUpdateC& u0 = wf_upd(f, 0);
  const int M = f.M, B = m0.bmax, n = u0.v[jv].n;
  const int tid = threadIdx.x, s = tid & 15;
  const int c = 16 * pass + (tid >> 4);
  if (16 * pass >= n) return;
  const int cc = min(c, n - 1);
  const float pp = u0.v[jv].param[cc];
  const bool has_src = u0.v[jv].src != nullptr;
  float acc = 0.f;
  for (int g0 = 0; g0 < M; g0 += WF_FG) {
    float v[WF_FG][8], pm[WF_FG], pv[WF_FG], gr[WF_FG], cf0[WF_FG], cf1[WF_FG];
    int nb[WF_FG];
#pragma unroll
    for (int i = 0; i < WF_FG; ++i) {
      const int ci = min(g0 + i, M - 1);
      GfkFoldClientC& P = wf_cl(f, ci);
      const int32_t* nbp = P.nb;
      const float *coef = P.coef, *vm = P.vm[jv], *vv = P.vv[jv], *vg = P.vg[jv], *src = P.vsrc[jv];
      nb[i] = *nbp;
      cf0[i] = coef[0];
      cf1[i] = coef[1];
      pm[i] = vm[cc];
      pv[i] = vv[cc];
      gr[i] = 0.f;
      if (has_src) {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[i][u] = src[(size_t)min(s + 16 * u, B - 1) * n + cc];
      } else {
        gr[i] = vg[cc];
      }
    }
#pragma unroll
    for (int i = 0; i < WF_FG; ++i) {
      if (g0 + i >= M) break;
      GfkFoldClientC& P = wf_cl(f, g0 + i);
      float g = gr[i];
      if (has_src) {
        g = 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u) g += s + 16 * u < nb[i] ? v[i][u] : 0.f;
        g = row16_sum(g);
      }
      if (s != 0 || c >= n) continue;
      float mo = pm[i], vo = pv[i];
      const float np = adam_update(pp, g, mo, vo, wf_coefp(P, cf0[i], cf1[i]));
      P.vm[jv][cc] = mo;
      P.vv[jv][cc] = vo;
      acc = fold_add(acc, np, P.vsc[jv], g0 + i == 0);
    }
  }
  if (s != 0 || c >= n) return;
  const int nw = f.mode == 1 ? 1 : M;
  for (int ci = 0; ci < nw; ++ci) wf_cl(f, ci).vp[jv][cc] = acc;
}

// leftover piece r: f.left[2 r] (first float, a multiple of 4), f.left[2 r + 1] floats (<= 1024)
__device__ __forceinline__ void wf_left(const GfkFold& f, int r) {
  const int64_t off = f.left[2 * r];
  const int len = (int)f.left[2 * r + 1];
  const int e = 4 * threadIdx.x;
  if (e >= len) return;
  const int M = f.M;
  const bool full = e + 3 < len;
  f32x4 tot = {0.f, 0.f, 0.f, 0.f};
  for (int g0 = 0; g0 < M; g0 += WF_FG) {
    f32x4 v[WF_FG];
#pragma unroll
    for (int i = 0; i < WF_FG; ++i) {
      const float* p = wf_cl(f, min(g0 + i, M - 1)).flat + off + e;
      if (full) {
        v[i] = *reinterpret_cast<const f32x4*>(p);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[i][k] = e + k < len ? p[k] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < WF_FG; ++i) {
      if (g0 + i >= M) break;
      tot = g0 + i == 0 ? v[i] : tot + v[i];
    }
  }
  const int nw = f.mode == 1 ? 1 : M;
  for (int c = 0; c < nw; ++c) {
    float* p = wf_cl(f, c).flat + off + e;
    if (full) {
      *reinterpret_cast<f32x4*>(p) = tot;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) if (e + k < len) p[k] = tot[k];
    }
  }
}
}  // namespace

extern "C" __global__ void __launch_bounds__(WF_NT) gfk_win_fold_k(GfkFold f) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  GfkModelC& m0 = wf_model(f, 0);
  GfkUpdateC& u0 = wf_upd(f, 0);
  const int n_tiles = m0.n_tiles, nj = f.nj;
  const int n_win = 8 * nj * ((n_tiles + 7) / 8);
  int r = blockIdx.x;
  WF_STAMP(298);
  if (r < n_win) {                  // a tile's nj slices on one XCD (they read the same x^T)
    const int x8 = r & 7, jj = r >> 3, js = jj % nj, tile = (jj / nj) * 8 + x8;
    if (tile < n_tiles) wf_win(f, smem, tile, js);
    return;
  }
  r -= n_win;
  if (r < 4 * u0.n_w) { wf_weight(f, smem, r >> 2, r & 3); return; }
  r -= 4 * u0.n_w;
  if (r < 4 * u0.n_v) { wf_vector(f, r >> 2, r & 3); return; }
  r -= 4 * u0.n_v;
  if (r < f.n_left) { wf_left(f, r); return; }
  r -= f.n_left;
  if (r < f.M) prepare_next_batch(f.models[r], reinterpret_cast<int*>(smem));
}

extern "C" size_t gfk_win_fold_smem() {
  const size_t a = 64 * WF_XS + 64 * WF_ZS, b = 64 * WF_ZS + 64 * WF_LDJ, c = 2 * GFK_BMAX_LIMIT;
  return sizeof(float) * (a > b ? (a > c ? a : c) : (b > c ? b : c));
}

extern "C" int gfk_win_fold_launch(const GfkModel* m0, const GfkUpdate* u0, const GfkFold* f, hipStream_t s) {
  if (m0->input != GFK_IN_BOW || m0->H[0] > 64 || m0->bmax != 64 || m0->update_mode != 1 ||
      (m0->stage_flags & (WIN_SPARSE | GFK_LB)) || m0->lab_on || f->M < 1 ||
      !f->models || !f->upds || !f->cl || f->nj != (m0->H[0] + 15) / 16 || (f->n_left > 0 && !f->left))
    return -1;
  for (int j = 0; j < u0->n_v; ++j)
    if (u0->v[j].n > 64) return -1;
  const int n_win = 8 * f->nj * ((m0->n_tiles + 7) / 8);
  const dim3 g(n_win + 4 * u0->n_w + 4 * u0->n_v + f->n_left + f->M);
  hipLaunchKernelGGL(gfk_win_fold_k, g, dim3(WF_NT), gfk_win_fold_smem(), s, *f);
  return (int)hipGetLastError();
}

extern "C" int gfk_win_update_set_smem(size_t bytes) {
  // the attribute is per function and process-wide: only ever raise it, so an engine
  // built earlier with a larger footprint keeps launching after a smaller one is set up
  static size_t cur = 0;
  if (bytes <= cur) return 0;
  cur = bytes;
  const void* ks[] = {(const void*)gfk_win_update_k<512, false>, (const void*)gfk_win_update_k<512, true>,
                      (const void*)gfk_win_update_k<1024, false>, (const void*)gfk_win_update_k<1024, true>,
                      (const void*)gfk_win_sparse_k<512, false>, (const void*)gfk_win_sparse_k<512, true>,
                      (const void*)gfk_win_sparse_k<512, false, true>, (const void*)gfk_win_sparse_k<512, true, true>,
                      (const void*)gfk_win_sparse_k<512, false, false, true>, (const void*)gfk_win_sparse_k<512, true, false, true>,
                      (const void*)gfk_win_sparse_k<512, false, true, true>, (const void*)gfk_win_sparse_k<512, true, true, true>,
                      (const void*)gfk_win_sparse_k<512, false, false, false, GFK_BMAX_LIMIT / 64>,
                      (const void*)gfk_win_sparse_k<512, true, false, false, GFK_BMAX_LIMIT / 64>,
                      (const void*)gfk_win_lb_k<1024>};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}
