// Batch-coupled part of the encoder: batch-norm of the mu / log-sigma^2 heads,
// reparameterised sample, softmax(theta), theta dropout, KL -- and the whole
// encoder backward down to the sparse input layer.
//
// Reference math: inference_network.py:76-85, decoder_network.py:102-118,
// avitm.py:207-229, torch.nn.BatchNorm1d training semantics (biased variance to
// normalise, unbiased variance into running_var, momentum 0.1).
//
// MI355X decomposition.  Batch-norm couples the rows only through per-column
// statistics, which are tiny ([2K] sums over <= 128 rows).  So instead of one
// workgroup doing everything (one CU's VALU + a chain of dependent global loads
// per phase), the rows are split over G = bmax/4 workgroups of 4 waves, one wave
// per row:
//   posterior_fwd : every workgroup re-derives the column statistics from the
//                   (L2-resident) raw heads of ALL rows, then does the heavy
//                   per-element work (Philox, exp, softmax) for its 4 rows only.
//   posterior_bwd_rows : per own row: softmax / reparameterisation / KL
//                   backward -> dmu, dls; each workgroup writes a partial slab
//                   of the column sums the BN backward needs (plain stores, no
//                   atomics, reduced in a fixed order => deterministic).
//   posterior_bwd_mlp : reduces the slabs, finishes the BN backward for its own
//                   rows, back-propagates through the heads and hidden MLP
//                   (weights staged in LDS) down to dz0, and writes its rows'
//                   share of every MLP weight gradient into its own gradient
//                   slab (plain stores; Adam sums the slabs in a fixed order).
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int PT = 256;            // threads per posterior workgroup
constexpr int RPB = 4;             // rows per workgroup (one wave per row)
constexpr int NSUM = 9;            // column sums per K-column (see posterior_bwd_rows)

__host__ __device__ inline int hmax_of(const GfkModel& m) {
  int h = 0;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l)
    if (l < m.n_hidden) h = h > m.H[l] ? h : m.H[l];
  return h;
}

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline int mlp_weight_floats(const GfkModel& m) {
  int n = 0;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
    if (l + 1 < m.n_hidden) n += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
  const int Hl = m.H[m.n_hidden - 1];
  return n + 2 * (pad4(m.K * Hl) + pad4(m.K));
}
}  // namespace

// Prepares the NEXT minibatch (the step counter has already been advanced):
// nb, the doc ids, and each row's CSR extent into ws_next.  This is a chain of
// four dependent global reads (step -> plan -> doc -> indptr); it runs in an
// extra workgroup of posterior_bwd_mlp, off the step's critical path, so the
// next encoder_fwd starts from one round trip.  Rows past the batch repeat its
// first doc so dense gathers over bmax rows stay in bounds.
__device__ void prepare_next_batch(const GfkModel& m) {
  const int step = *m.step;
  int32_t* nxt = m.ws_next;
  if (step >= m.n_steps) {
    if (threadIdx.x == 0) nxt[0] = 0;
    return;
  }
  const int nb = m.plan_size[step];
  const int base = m.plan_start[step];
  for (int b = threadIdx.x; b < m.bmax; b += blockDim.x) {
    const int doc = m.plan_order[base + (b < nb ? b : 0)];
    const int e0 = m.indptr[doc], e1 = m.indptr[doc + 1];
    nxt[1 + b] = doc;
    nxt[1 + m.bmax + 2 * b] = e0;
    nxt[2 + m.bmax + 2 * b] = e1;
  }
  if (threadIdx.x == 0) nxt[0] = nb;
}

extern "C" __global__ void gfk_batch_prep(GfkModel m) { prepare_next_batch(m); }

// Publishes the prepared batch (doc ids for every row < bmax, nb) before the
// dense contextual GEMMs of the CTM encoders, which run on all bmax rows.
extern "C" __global__ void gfk_batch_docs(GfkModel m) {
  const int32_t* nxt = m.ws_next;
  for (int b = threadIdx.x; b < m.bmax; b += blockDim.x) m.ws_doc[b] = nxt[1 + b];
  if (threadIdx.x == 0) *m.ws_nb = nxt[0];
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
extern "C" size_t gfk_posterior_fwd_smem(const GfkModel* m) {
  return sizeof(float) * (2 * (size_t)m->bmax * m->K + 4 * (size_t)m->K);
}

// grid: bmax/4 workgroups.  dynamic LDS: mr[bmax*K] + lr[bmax*K] + mean[2K] + rstd[2K]
extern "C" __global__ void __launch_bounds__(PT) gfk_posterior_fwd(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  int K = m.K, bmax = m.bmax;
  const float *mu_raw = m.ws_mu_raw, *ls_raw = m.ws_ls_raw;
  float *mu_rm = m.mu_rm, *mu_rv = m.mu_rv, *s_rm = m.s_rm, *s_rv = m.s_rv;
  const int32_t *nbp = m.ws_nb, *stepp = m.step;
  keep(K, bmax, mu_raw, ls_raw, mu_rm, mu_rv, s_rm, s_rv, nbp, stepp);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  float* mr = smem;
  float* lr = mr + bmax * K;
  float* cmean = lr + bmax * K;
  float* crstd = cmean + 2 * K;
  GFK_STAMP(m, 0);
  // all loads up front: raw heads of every row by LDS-DMA (rows >= nb are never
  // read back), the running statistics, the counters
  glds_copy(mr, mu_raw, bmax * K, tid, PT);
  glds_copy(lr, ls_raw, bmax * K, tid, PT);
  float rm_old = 0.f, rv_old = 0.f;
  if (blockIdx.x == 0 && tid < 2 * K) {
    const int c = tid < K ? tid : tid - K;
    rm_old = (tid < K ? mu_rm : s_rm)[c];
    rv_old = (tid < K ? mu_rv : s_rv)[c];
  }
  const int nb = *nbp;
  const int step = *stepp;
  const int row = blockIdx.x * RPB + wave;
  if (m.kind == GFK_LDA) {
    // NeuralLDA: per-topic log-sum-exp over V from the vocab-tile partials;
    // topics are dealt to the (workgroup, wave) pairs of the whole grid
    for (int k = blockIdx.x * (PT / 64) + wave; k < K; k += gridDim.x * (PT / 64)) {
      float mx = -INFINITY, se = 0.f;
      for (int g = lane; g < m.dec_grid; g += 64) {
        const float* p = m.ws_row_part + ((size_t)g * K + k) * 2;
        lse_merge(mx, se, p[0], p[1]);
      }
      wave_lse(mx, se);
      if (lane == 0) m.ws_lse[k] = mx + logf(se);
    }
  }
  __syncthreads();
  GFK_STAMP(m, 1);
  // ---- column statistics over the batch (every workgroup, redundantly) ----
  for (int t = tid; t < 2 * K; t += PT) {
    const float* x = (t < K ? mr : lr) + (t < K ? t : t - K);
    float s = 0.f;
#pragma unroll 8
    for (int b = 0; b < nb; ++b) s += x[b * K];
    const float mean = s / (float)nb;
    float q = 0.f;
#pragma unroll 8
    for (int b = 0; b < nb; ++b) { const float d = x[b * K] - mean; q += d * d; }
    const float var = q / (float)nb;
    const float rstd = rsqrtf(var + m.bn_eps);
    cmean[t] = mean;
    crstd[t] = rstd;
    if (blockIdx.x == 0) {   // t == tid here: 2K <= 512 < PT is not required, see below
      const int c = t < K ? t : t - K;
      float* rm = t < K ? m.mu_rm : m.s_rm;
      float* rv = t < K ? m.mu_rv : m.s_rv;
      const float mom = m.bn_momentum;
      const float unb = nb > 1 ? var * (float)nb / (float)(nb - 1) : var;
      const float ro = t == tid ? rm_old : rm[c], vo = t == tid ? rv_old : rv[c];
      rm[c] = (1.f - mom) * ro + mom * mean;
      rv[c] = (1.f - mom) * vo + mom * unb;
      m.ws_bn_rstd[t] = rstd;
    }
  }
  if (blockIdx.x == 0 && tid == 0) { *m.nbt_mu += 1; *m.nbt_s += 1; }
  __syncthreads();
  GFK_STAMP(m, 2);
  // ---- own row: reparameterise, softmax, dropout, KL ----
  if (row < nb) {
    float logpv_sum = 0.f;
    for (int k = lane; k < K; k += 64) logpv_sum += logf(m.prior_var[k]);
    logpv_sum = wave_sum(logpv_sum);
    float zmax = -INFINITY, kl = 0.f;
    constexpr int KQ = 4;   // K <= 256
    float zq[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int k = lane + 64 * q;
      zq[q] = -INFINITY;
      if (k < K) {
        const int i = row * K + k;
        const float mu = (mr[i] - cmean[k]) * crstd[k];
        const float ls = (lr[i] - cmean[K + k]) * crstd[K + k];
        const float e = randn(m.seed, (uint32_t)step, RNG_EPS, (uint32_t)i);
        const float sd = expf(0.5f * ls);
        const float z = mu + e * sd;
        m.ws_mu[i] = mu;
        m.ws_ls[i] = ls;
        m.ws_eps[i] = e;
        zq[q] = z;
        zmax = fmaxf(zmax, z);
        const float pv = m.prior_var[k], dm = m.prior_mean[k] - mu;
        kl += sd * sd / pv + dm * dm / pv - ls;
      }
    }
    zmax = wave_max(zmax);
    kl = wave_sum(kl);
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
        const int i = row * K + k;
        const float th = zq[q] * inv;
        const float s = drop_scale(m.seed, (uint32_t)step, RNG_DROP_THETA, (uint32_t)i, m.drop_theta);
        m.ws_theta[i] = th;
        m.ws_mask_t[i] = s;
        m.ws_thetad[row * m.kt + k] = th * s;
      }
    }
    if (lane == 0) m.ws_kl[row] = 0.5f * (kl - (float)K + logpv_sum);
  }
  GFK_STAMP(m, 3);
}

// ---------------------------------------------------------------------------
// backward, part 1: per-row softmax / reparameterisation / KL backward
// ---------------------------------------------------------------------------
// Column sums written per workgroup g into ws_colpart[g][NSUM][K]:
//   0: sum dmu   1: sum dmu*mu   2: sum dls   3: sum dls*ls   4: sum mu   5: sum ls
//   6: sum exp(ls)   7: sum (pm - mu)^2   8: sum theta_d * dtheta_d   (NeuralLDA c_k)
// d theta_d arrives as n_dpart partial slabs [n_dpart][bmax][K] (one per decoder
// vocab tile for ProdLDA, plain stores, so the sum below is in a fixed order and
// the step is deterministic); the own rows' slices are pulled into LDS by
// LDS-DMA, DPC tiles per round.
__host__ __device__ inline int dpart_chunk(const GfkModel& m) {
  const int cap = (96 * 1024) / (int)(sizeof(float) * RPB * m.K);
  return m.n_dpart < cap ? m.n_dpart : (cap > 0 ? cap : 1);
}

extern "C" size_t gfk_posterior_bwd_rows_smem(const GfkModel* m) {
  return sizeof(float) * ((size_t)RPB * NSUM * m->K + (size_t)RPB * m->K +
                          (size_t)dpart_chunk(*m) * RPB * m->K);
}

// dynamic LDS: part[RPB][NSUM][K] + dsum[RPB*K] + stage[DPC][RPB*K]
extern "C" __global__ void __launch_bounds__(PT) gfk_posterior_bwd_rows(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int r0 = blockIdx.x * RPB;
  const int row = r0 + wave;
  const float wk = m.kl_weight;
  float* part = smem;                 // [RPB][NSUM][K]
  float* dsum = part + RPB * NSUM * K;
  float* stg = dsum + RPB * K;
  const int DPC = dpart_chunk(m);
  const int nrk = RPB * K;
  GFK_STAMP(m, 8);
  // ---- one staging round: d theta_d partials (LDS-DMA) + the own row's stash ----
  float acc = 0.f;                    // thread t < nrk sums element t of the own rows
  for (int p0 = 0; p0 < m.n_dpart; p0 += DPC) {
    const int np = min(DPC, m.n_dpart - p0);
    for (int p = wave; p < np; p += PT / 64)   // one wave per slab copy
      glds_copy(stg + p * nrk, m.ws_dthetad + ((size_t)(p0 + p) * m.bmax + r0) * K, nrk, lane, 64);
    if (p0 + DPC < m.n_dpart) {       // more rounds follow: drain this one now
      __syncthreads();
      if (tid < nrk)
        for (int p = 0; p < np; ++p) acc += stg[p * nrk + tid];
      __syncthreads();
    }
  }
  const int nb = *m.ws_nb;
  constexpr int KQ = 4;
  float dt[KQ], th[KQ], td[KQ], mu[KQ], ls[KQ], ep[KQ], pm[KQ], pv[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {   // all loads first
    const int k = min(lane + 64 * q, K - 1);
    const int i = min(row, nb - 1) * K + k;
    dt[q] = m.ws_mask_t[i];
    th[q] = m.ws_theta[i];
    td[q] = m.ws_thetad[min(row, nb - 1) * m.kt + k];
    mu[q] = m.ws_mu[i];
    ls[q] = m.ws_ls[i];
    ep[q] = m.ws_eps[i];
    pm[q] = m.prior_mean[k];
    pv[q] = m.prior_var[k];
  }
  __syncthreads();
  {
    const int p0 = ((m.n_dpart - 1) / DPC) * DPC, np = m.n_dpart - p0;
    if (tid < nrk) {
      for (int p = 0; p < np; ++p) acc += stg[p * nrk + tid];
      dsum[tid] = acc;
    }
    for (int t = tid + PT; t < nrk; t += PT) {   // K > 64: more elements than threads
      float a2 = 0.f;
      for (int p = 0; p < m.n_dpart; ++p)
        a2 += m.ws_dthetad[((size_t)p * m.bmax + r0) * K + t];
      dsum[t] = a2;
    }
  }
  __syncthreads();
  float dtd[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) dtd[q] = dsum[wave * K + min(lane + 64 * q, K - 1)];
  const bool live = row < nb;
  float c = 0.f;
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    dt[q] *= dtd[q];              // through theta dropout
    if (lane + 64 * q < K) c += dt[q] * th[q];
  }
  c = wave_sum(c);
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int k = lane + 64 * q;
    if (k >= K) continue;
    const float dz = th[q] * (dt[q] - c);
    const float sd = expf(0.5f * ls[q]);
    const float dmu = dz + wk * (mu[q] - pm[q]) / pv[q];
    const float dls = dz * ep[q] * 0.5f * sd + wk * 0.5f * (sd * sd / pv[q] - 1.f);
    float* p = part + wave * NSUM * K + k;
    if (live) {
      m.ws_dmu[row * K + k] = dmu;
      m.ws_dls[row * K + k] = dls;
      const float dmm = pm[q] - mu[q];
      p[0] = dmu; p[K] = dmu * mu[q]; p[2 * K] = dls; p[3 * K] = dls * ls[q];
      p[4 * K] = mu[q]; p[5 * K] = ls[q]; p[6 * K] = sd * sd; p[7 * K] = dmm * dmm;
      p[8 * K] = td[q] * dtd[q];
    } else {
#pragma unroll
      for (int s = 0; s < NSUM; ++s) p[s * K] = 0.f;
    }
  }
  // loss of the minibatch and the counters of the next replay (workgroup 0)
  if (blockIdx.x == 0 && wave == 0) {
    float l = 0.f;
    for (int b = lane; b < nb; b += 64) l += wk * m.ws_kl[b] + m.ws_rl[b];
    l = wave_sum(l);
    if (lane == 0) {
      const int step = *m.step;
      m.loss_hist[step] = l;
      *m.step = step + 1;
      *m.adam_t += 1;
    }
  }
  __syncthreads();
  for (int t = tid; t < NSUM * K; t += PT) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < RPB; ++r) s += part[r * NSUM * K + t];
    m.ws_colpart[(size_t)blockIdx.x * NSUM * K + t] = s;
  }
  GFK_STAMP(m, 9);
}

// ---------------------------------------------------------------------------
// backward, part 2: BN backward of the heads, heads / MLP backward, dz0 and the
// weight gradients of the MLP (per-workgroup slabs, reduced by Adam)
// ---------------------------------------------------------------------------
// LDS plan of posterior_bwd_mlp (floats, every piece padded to 4 so each is a
// valid LDS-DMA destination)
struct MlpLds {
  int cp, cs, rstd, dmu, dls, mu, ls, mask, hd, z, a, dh, dh2, w, total;   // z, a: layer 0 base
  bool stage_cp;
};

__host__ __device__ inline MlpLds mlp_lds(const GfkModel& m) {
  MlpLds L;
  const int K = m.K, nh = m.n_hidden, Hl = m.H[nh - 1], G = m.bmax / RPB, hm = hmax_of(m);
  int o = 0;
  L.stage_cp = (size_t)G * NSUM * K * sizeof(float) <= 64 * 1024;
  L.cp = o; o += L.stage_cp ? pad4(G * NSUM * K) : 0;
  L.cs = o; o += pad4(NSUM * K);
  L.rstd = o; o += pad4(2 * K);
  L.dmu = o; o += RPB * K;
  L.dls = o; o += RPB * K;
  L.mu = o; o += RPB * K;
  L.ls = o; o += RPB * K;
  L.mask = o; o += RPB * Hl;
  L.hd = o; o += RPB * Hl;
  L.z = o;
#pragma unroll
  for (int l = 0; l < GFK_MAX_LAYERS; ++l) if (l < nh) o += RPB * m.H[l];
  L.a = o;
#pragma unroll
  for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) if (l + 1 < nh) o += RPB * m.H[l];
  L.dh = o; o += RPB * hm;
  L.dh2 = o; o += RPB * hm;
  L.w = o; o += (m.stage_flags & 1) ? mlp_weight_floats(m) : 0;
  L.total = o;
  return L;
}

// offset of layer l's [RPB x H[l]] block inside the z / a stashes
__device__ __forceinline__ int layer_off(const GfkModel& m, int l) {
  int o = 0;
#pragma unroll
  for (int i = 0; i < GFK_MAX_LAYERS; ++i) if (i < l) o += RPB * m.H[i];
  return o;
}

extern "C" size_t gfk_posterior_bwd_mlp_smem(const GfkModel* m) {
  return sizeof(float) * (size_t)mlp_lds(*m).total;
}

// grid: bmax/4 workgroups of 4 waves; workgroup g owns rows [4g, 4g+4).
// Every global read is issued in ONE staging round (LDS-DMA): the column-sum
// slabs of all workgroups, the own rows' heads / BN outputs / masks /
// pre-activations / activations, and (when they fit) the MLP weights.  After
// that the kernel only touches LDS until its stores.
extern "C" __global__ void __launch_bounds__(PT) gfk_posterior_bwd_mlp(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (blockIdx.x == gridDim.x - 1) {   // the extra workgroup: next step's batch
    prepare_next_batch(m);
    return;
  }
  // prologue: pin the argument fields of the staging round in SGPRs
  int K = m.K, nh = m.n_hidden, H0 = m.H[0], H1 = m.H[1], H2 = m.H[2], sflags = m.stage_flags;
  const float *w_mu = m.w_mu, *w_s = m.w_s, *colpart = m.ws_colpart, *bn_rstd = m.ws_bn_rstd;
  const float *g_dmu = m.ws_dmu, *g_dls = m.ws_dls, *g_mu = m.ws_mu, *g_ls = m.ws_ls;
  const float *g_mask = m.ws_mask_h, *g_hd = m.ws_hd, *g_z0 = m.ws_z[0], *g_z1 = m.ws_z[1];
  const float *g_a0 = m.ws_a[0], *w_h0 = m.w_h[0];
  const int32_t* nbp = m.ws_nb;
  keep(K, nh, H0, H1, H2, sflags, w_mu, w_s, colpart, bn_rstd, g_dmu, g_dls, g_mu, g_ls, g_mask, g_hd,
       g_z0, g_z1, g_a0, w_h0, nbp);
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int Hl = m.H[nh - 1], hm = hmax_of(m);
  const int G = gridDim.x - 1;
  const int r0 = blockIdx.x * RPB;
  const float wk = m.kl_weight;
  const MlpLds L = mlp_lds(m);
  float* cs = smem + L.cs;
  float* dmr = smem + L.dmu;   // dmu, then (in place) d mu_raw
  float* dlr = smem + L.dls;
  float* dh = smem + L.dh;
  float* dh2 = smem + L.dh2;
  float* wst = smem + L.w;
  const bool staged = sflags & 1;
  const size_t so = (size_t)blockIdx.x * m.slab_stride;   // this workgroup's gradient slab
  GFK_STAMP(m, 10);
  // ---- the staging round ----
  if (staged) {
    float* p = wst;
#pragma unroll
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l) {
      if (l + 1 < nh) {
        const int nw = m.H[l + 1] * m.H[l];
        glds_copy(p, l == 0 ? w_h0 : m.w_h[l], nw, tid, PT); p += pad4(nw) + pad4(m.H[l + 1]);
      }
    }
    glds_copy(p, w_mu, K * Hl, tid, PT); p += pad4(K * Hl) + pad4(K);
    glds_copy(p, w_s, K * Hl, tid, PT);
  }
  if (L.stage_cp) glds_copy(smem + L.cp, colpart, G * NSUM * K, tid, PT);
  glds_copy(smem + L.rstd, bn_rstd, 2 * K, tid, PT);
  glds_copy(smem + L.dmu, g_dmu + (size_t)r0 * K, RPB * K, tid, PT);
  glds_copy(smem + L.dls, g_dls + (size_t)r0 * K, RPB * K, tid, PT);
  glds_copy(smem + L.mu, g_mu + (size_t)r0 * K, RPB * K, tid, PT);
  glds_copy(smem + L.ls, g_ls + (size_t)r0 * K, RPB * K, tid, PT);
  glds_copy(smem + L.mask, g_mask + (size_t)r0 * Hl, RPB * Hl, tid, PT);
  glds_copy(smem + L.hd, g_hd + (size_t)r0 * Hl, RPB * Hl, tid, PT);
  {
    int o = 0;
#pragma unroll
    for (int l = 0; l < GFK_MAX_LAYERS; ++l) {
      if (l < nh) {
        const float* zl = l == 0 ? g_z0 : (l == 1 ? g_z1 : m.ws_z[l]);
        const float* al = l == 0 ? g_a0 : m.ws_a[l];
        glds_copy(smem + L.z + o, zl + (size_t)r0 * m.H[l], RPB * m.H[l], tid, PT);
        if (l + 1 < nh) glds_copy(smem + L.a + o, al + (size_t)r0 * m.H[l], RPB * m.H[l], tid, PT);
        o += RPB * m.H[l];
      }
    }
  }
  float pm = 0.f, pv = 1.f;
  if (blockIdx.x == 0 && tid < K) { pm = m.prior_mean[tid]; pv = m.prior_var[tid]; }
  const int nb = *nbp;
  __syncthreads();
  // ---- column sums: fixed-order reduction of the per-workgroup slabs ----
  for (int t = tid; t < NSUM * K; t += PT) {
    float s = 0.f;
    if (L.stage_cp) {
      const float* cp = smem + L.cp;
      for (int g = 0; g < G; ++g) s += cp[g * NSUM * K + t];
    } else {
      for (int g = 0; g < G; ++g) s += m.ws_colpart[(size_t)g * NSUM * K + t];
    }
    cs[t] = s;
  }
  __syncthreads();
  GFK_STAMP(m, 11);
  const float inv_nb = 1.f / (float)nb;
  const float* rstd = smem + L.rstd;
  // ---- head-bias and prior gradients (workgroup 0; the other slabs hold 0) ----
  for (int t = tid; t < 2 * K; t += PT) {
    const bool is_mu = t < K;
    const int k = is_mu ? t : t - K;
    float g = 0.f;
    if (blockIdx.x == 0) {
      const float s1 = cs[(is_mu ? 0 : 2) * K + k], s2 = cs[(is_mu ? 1 : 3) * K + k];
      const float sx = cs[(is_mu ? 4 : 5) * K + k];
      // sum_b rstd (dy - s1/nb - xh s2/nb) = rstd (s1 - s1 - sx s2 / nb)
      g = rstd[t] * (s1 - s1 - sx * s2 * inv_nb);
    }
    (is_mu ? m.s_b_mu : m.s_b_s)[so + k] = g;
  }
  if (blockIdx.x == 0 && tid < K) {
    const int k = tid;
    if (m.learn_priors) {
      const float smu = cs[4 * K + k], svar = cs[6 * K + k], sdm2 = cs[7 * K + k];
      m.g_prior_mean[k] = wk * ((float)nb * pm - smu) / pv;
      m.g_prior_var[k] = wk * 0.5f * ((float)nb / pv - svar / (pv * pv) - sdm2 / (pv * pv));
    }
    if (m.kind == GFK_LDA) m.ws_ck[k] = cs[8 * K + k];
  }
  // ---- BN backward of the heads for the own rows (in place) ----
  for (int t = tid; t < RPB * 2 * K; t += PT) {
    const int r = t / (2 * K), c2 = t % (2 * K);
    const bool is_mu = c2 < K;
    const int k = is_mu ? c2 : c2 - K;
    const int i = r * K + k;
    float* dy = is_mu ? dmr : dlr;
    const float xh = (is_mu ? smem + L.mu : smem + L.ls)[i];
    const float s1 = cs[(is_mu ? 0 : 2) * K + k] * inv_nb, s2 = cs[(is_mu ? 1 : 3) * K + k] * inv_nb;
    dy[i] = r0 + r < nb ? rstd[c2] * (dy[i] - s1 - xh * s2) : 0.f;
  }
  __syncthreads();
  GFK_STAMP(m, 12);
  // ---- heads: weight gradients (own rows' share, slab stores) and d hd ----
  const float* Wmu = m.w_mu;
  const float* Ws = m.w_s;
  if (staged) {
    const float* wcur = wst;
#pragma unroll
    for (int l = 0; l + 1 < GFK_MAX_LAYERS; ++l)
      if (l + 1 < nh) wcur += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
    Wmu = wcur;
    Ws = wcur + pad4(K * Hl) + pad4(K);
  }
  {
    const float* hdv = smem + L.hd;
    const float* mask = smem + L.mask;
    const MatView Amu{dmr, 1, K, K, RPB}, As{dlr, 1, K, K, RPB};   // A[k][q] = dy[q][k]
    const MatView Bh{hdv, Hl, 1, RPB, Hl};                         // B[q][j] = hd[q][j]
    float *gwm = m.s_w_mu + so, *gws = m.s_w_s + so;
    mfma_gemm(K, Hl, RPB, Amu, Bh, wave, PT / 64, [&](int k, int j, float v) { gwm[k * Hl + j] = v; });
    mfma_gemm(K, Hl, RPB, As, Bh, wave, PT / 64, [&](int k, int j, float v) { gws[k * Hl + j] = v; });
    // d hd = dmu_raw W_mu + dls_raw W_s (one GEMM over the concatenated 2K), through the dropout
    const MatView Dm{dmr, K, 1, RPB, K}, Ds{dlr, K, 1, RPB, K};
    const MatView Wm{Wmu, Hl, 1, K, Hl}, Wsv{Ws, Hl, 1, K, Hl};
    const int nt = (Hl + 15) >> 4;
    for (int s = wave; s < nt; s += PT / 64) {
      const int j0 = s * 16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int ai = lane & 15, bj = j0 + (lane & 15), kk = lane >> 4;
      for (int k0 = 0; k0 < K; k0 += 4) {
        acc = mfma16x16x4(Dm.at(ai, k0 + kk), Wm.at(k0 + kk, bj), acc);
        acc = mfma16x16x4(Ds.at(ai, k0 + kk), Wsv.at(k0 + kk, bj), acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = (lane >> 4) * 4 + r;
        if (q < RPB && bj < Hl) dh[q * hm + bj] = acc[r] * mask[q * Hl + bj];
      }
    }
  }
  __syncthreads();
  GFK_STAMP(m, 13);
  // ---- hidden layers, last to first (own rows) ----
  for (int l = nh - 2; l >= 0; --l) {
    const int Hi = m.H[l], Ho = m.H[l + 1];
    const float* W = m.w_h[l];
    if (staged) {
      const float* p = wst;
#pragma unroll
      for (int ll = 0; ll + 1 < GFK_MAX_LAYERS; ++ll)
        if (ll < l) p += pad4(m.H[ll + 1] * m.H[ll]) + pad4(m.H[ll + 1]);
      W = p;
    }
    const float* zl = smem + L.z + layer_off(m, l + 1);
    for (int t = tid; t < RPB * Ho; t += PT) {
      const int q = t / Ho, j = t % Ho;
      dh[q * hm + j] = r0 + q < nb ? dh[q * hm + j] * act_d(m.act, zl[q * Ho + j]) : 0.f;
    }
    __syncthreads();
    {
      const MatView dZt{dh, 1, hm, Ho, RPB};          // A[j][q] = dz[q][j]
      const MatView Av{smem + L.a + layer_off(m, l), Hi, 1, RPB, Hi};  // B[q][i] = a_l[q][i]
      float* gw = m.s_w_h[l] + so;
      mfma_gemm(Ho, Hi, RPB, dZt, Av, wave, PT / 64, [&](int j, int i, float v) { gw[j * Hi + i] = v; });
    }
    for (int j = tid; j < Ho; j += PT) {
      float g = 0.f;
#pragma unroll
      for (int q = 0; q < RPB; ++q) g += dh[q * hm + j];
      m.s_b_h[l][so + j] = g;
    }
    {
      const MatView dZ{dh, hm, 1, RPB, Ho};    // A[q][j]
      const MatView Wv{W, Hi, 1, Ho, Hi};      // B[j][i] = W[j][i]
      mfma_gemm(RPB, Hi, Ho, dZ, Wv, wave, PT / 64, [&](int q, int i, float v) { dh2[q * hm + i] = v; });
    }
    __syncthreads();
    float* tmp = dh; dh = dh2; dh2 = tmp;
  }
  // ---- input layer: dz0 (consumed by the input-layer scatter) and its bias ----
  {
    const float* z0 = smem + L.z;
    for (int t = tid; t < RPB * H0; t += PT) {
      const int q = t / H0, j = t % H0, row = r0 + q;
      const float g = row < nb ? dh[q * hm + j] * act_d(m.act, z0[q * H0 + j]) : 0.f;
      dh[q * hm + j] = g;
      m.ws_dz0[(size_t)row * H0 + j] = g;
    }
  }
  __syncthreads();
  for (int j = tid; j < H0; j += PT) {
    float g = 0.f;
#pragma unroll
    for (int q = 0; q < RPB; ++q) g += dh[q * hm + j];
    m.s_b_in[so + j] = g;
  }
  GFK_STAMP(m, 14);
}

extern "C" int gfk_launch_batch_prep(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_batch_prep, dim3(1), dim3(256), 0, s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_batch_docs(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_batch_docs, dim3(1), dim3(256), 0, s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_posterior_fwd(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_posterior_fwd, dim3(m->bmax / RPB), dim3(PT), gfk_posterior_fwd_smem(m), s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_posterior_bwd(const GfkModel* m, hipStream_t s) {
  hipLaunchKernelGGL(gfk_posterior_bwd_rows, dim3(m->bmax / RPB), dim3(PT),
                     gfk_posterior_bwd_rows_smem(m), s, *m);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(gfk_posterior_bwd_mlp, dim3(m->bmax / RPB + 1), dim3(PT),
                     gfk_posterior_bwd_mlp_smem(m), s, *m);
  return (int)hipGetLastError();
}

extern "C" int gfk_posterior_set_smem(size_t bytes) {
  const void* ks[] = {(const void*)gfk_posterior_fwd, (const void*)gfk_posterior_bwd_rows,
                      (const void*)gfk_posterior_bwd_mlp};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" size_t gfk_posterior_bwd_smem(const GfkModel* m) {
  const size_t a = gfk_posterior_bwd_rows_smem(m), b = gfk_posterior_bwd_mlp_smem(m);
  return a > b ? a : b;
}

extern "C" size_t gfk_mlp_weight_bytes(const GfkModel* m) {
  return sizeof(float) * (size_t)mlp_weight_floats(*m);
}
