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
//                   (weights staged in LDS), scatters the sparse input-layer
//                   gradient of its rows, and adds its rows' share of every
//                   weight gradient (float atomics, 16-way at B=64).
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int PT = 256;            // threads per posterior workgroup
constexpr int RPB = 4;             // rows per workgroup (one wave per row)
constexpr int NSUM = 9;            // column sums per K-column (see posterior_bwd_rows)
constexpr int CH = 16;             // non-zeros per wave batch in the input-layer scatter

__host__ __device__ inline int hmax_of(const GfkModel& m) {
  int h = 0;
  for (int l = 0; l < m.n_hidden; ++l) h = h > m.H[l] ? h : m.H[l];
  return h;
}

__host__ __device__ inline int pad4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline int mlp_weight_floats(const GfkModel& m) {
  int n = 0;
  for (int l = 0; l + 1 < m.n_hidden; ++l) n += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
  const int Hl = m.H[m.n_hidden - 1];
  return n + 2 * (pad4(m.K * Hl) + pad4(m.K));
}
}  // namespace

// Writes the doc ids of the current minibatch for every row < bmax (rows past
// the batch repeat row 0 so gathers stay in bounds).  Used before the dense
// contextual GEMMs of the CTM encoders, which run on all bmax rows.
extern "C" __global__ void gfk_batch_docs(GfkModel m) {
  const int step = *m.step;
  const int nb = m.plan_size[step];
  const int base = m.plan_start[step];
  for (int b = threadIdx.x; b < m.bmax; b += blockDim.x)
    m.ws_doc[b] = m.plan_order[base + (b < nb ? b : 0)];
  if (threadIdx.x == 0) *m.ws_nb = nb;
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
  const int K = m.K, bmax = m.bmax, tid = threadIdx.x;
  const int lane = tid & 63, wave = uniform(tid >> 6);
  float* mr = smem;
  float* lr = mr + bmax * K;
  float* cmean = lr + bmax * K;
  float* crstd = cmean + 2 * K;
  GFK_STAMP(m, 0);
  // all loads up front: raw heads of every row by LDS-DMA (rows >= nb are never
  // read back), the running statistics, the counters
  glds_copy(mr, m.ws_mu_raw, bmax * K, tid, PT);
  glds_copy(lr, m.ws_ls_raw, bmax * K, tid, PT);
  float rm_old = 0.f, rv_old = 0.f;
  if (blockIdx.x == 0 && tid < 2 * K) {
    const int c = tid < K ? tid : tid - K;
    rm_old = (tid < K ? m.mu_rm : m.s_rm)[c];
    rv_old = (tid < K ? m.mu_rv : m.s_rv)[c];
  }
  const int nb = *m.ws_nb;
  const int step = *m.step;
  const int row = blockIdx.x * RPB + wave;
  // theta_d's gradient is accumulated with atomics by the decoder backward: clear own rows
  if (row < bmax)
    for (int k = lane; k < K; k += 64) m.ws_dthetad[(size_t)row * K + k] = 0.f;
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
        m.ws_thetad[i] = th * s;
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
extern "C" size_t gfk_posterior_bwd_rows_smem(const GfkModel* m) {
  return sizeof(float) * ((size_t)RPB * NSUM * m->K);
}

extern "C" __global__ void __launch_bounds__(PT) gfk_posterior_bwd_rows(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int nb = *m.ws_nb;
  const int row = blockIdx.x * RPB + wave;
  const float wk = m.kl_weight;
  float* part = smem;     // [RPB][NSUM][K]
  GFK_STAMP(m, 8);
  constexpr int KQ = 4;
  float dt[KQ], th[KQ], td[KQ], dtd[KQ], mu[KQ], ls[KQ], ep[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {   // all loads first
    const int k = min(lane + 64 * q, K - 1);
    const int i = min(row, nb - 1) * K + k;
    dtd[q] = m.ws_dthetad[i];
    dt[q] = m.ws_mask_t[i];
    th[q] = m.ws_theta[i];
    td[q] = m.ws_thetad[i];
    mu[q] = m.ws_mu[i];
    ls[q] = m.ws_ls[i];
    ep[q] = m.ws_eps[i];
  }
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
    const float pm = m.prior_mean[k], pv = m.prior_var[k];
    const float dz = th[q] * (dt[q] - c);
    const float sd = expf(0.5f * ls[q]);
    const float dmu = dz + wk * (mu[q] - pm) / pv;
    const float dls = dz * ep[q] * 0.5f * sd + wk * 0.5f * (sd * sd / pv - 1.f);
    float* p = part + wave * NSUM * K + k;
    if (live) {
      m.ws_dmu[row * K + k] = dmu;
      m.ws_dls[row * K + k] = dls;
      const float dmm = pm - mu[q];
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
// backward, part 2: BN backward of the heads, heads / MLP backward, sparse
// input-layer scatter, weight gradients
// ---------------------------------------------------------------------------
extern "C" size_t gfk_posterior_bwd_mlp_smem(const GfkModel* m) {
  const int hm = hmax_of(*m);
  size_t n = (size_t)NSUM * m->K + 2 * (size_t)RPB * m->K + 3 * (size_t)RPB * hm;
  if (m->stage_flags & 1) n += mlp_weight_floats(*m);
  return sizeof(float) * n;
}

// dynamic LDS: cs[NSUM*K] + dmr[RPB*K] + dlr[RPB*K] + dh[RPB*hm] + dh2[RPB*hm] + av[RPB*hm]
//              (+ staged weights)
extern "C" __global__ void __launch_bounds__(PT) gfk_posterior_bwd_mlp(GfkModel m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int K = m.K, tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int nh = m.n_hidden, Hl = m.H[nh - 1], H0 = m.H[0], hm = hmax_of(m);
  const int G = gridDim.x;
  const int r0 = blockIdx.x * RPB;
  const float wk = m.kl_weight;
  float* cs = smem;
  float* dmr = cs + NSUM * K;
  float* dlr = dmr + RPB * K;
  float* dh = dlr + RPB * K;
  float* dh2 = dh + RPB * hm;
  float* av = dh2 + RPB * hm;
  float* wst = av + RPB * hm;
  const bool staged = m.stage_flags & 1;
  GFK_STAMP(m, 10);
  // ---- loads up front: weights, slabs, own-row stash ----
  if (staged) {
    float* p = wst;
    for (int l = 0; l + 1 < nh; ++l) {
      const int nw = m.H[l + 1] * m.H[l];
      glds_copy(p, m.w_h[l], nw, tid, PT); p += pad4(nw) + pad4(m.H[l + 1]);
    }
    glds_copy(p, m.w_mu, K * Hl, tid, PT); p += pad4(K * Hl) + pad4(K);
    glds_copy(p, m.w_s, K * Hl, tid, PT);
  }
  glds_copy(av, m.ws_hd + (size_t)r0 * Hl, RPB * Hl, tid, PT);   // own rows' dropped hidden
  for (int t = tid; t < NSUM * K; t += PT) {
    constexpr int U = 8;
    float s = 0.f;
    for (int g0 = 0; g0 < G; g0 += U) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u] = m.ws_colpart[(size_t)min(g0 + u, G - 1) * NSUM * K + t];
#pragma unroll
      for (int u = 0; u < U; ++u) s += (g0 + u < G) ? v[u] : 0.f;
    }
    cs[t] = s;
  }
  const int nb = *m.ws_nb;
  __syncthreads();
  GFK_STAMP(m, 11);
  const float inv_nb = 1.f / (float)nb;
  // ---- workgroup 0: head-bias and prior gradients from the column sums ----
  if (blockIdx.x == 0) {
    for (int t = tid; t < 2 * K; t += PT) {
      const bool is_mu = t < K;
      const int k = is_mu ? t : t - K;
      const float rstd = m.ws_bn_rstd[t];
      const float s1 = cs[(is_mu ? 0 : 2) * K + k], s2 = cs[(is_mu ? 1 : 3) * K + k];
      const float sx = cs[(is_mu ? 4 : 5) * K + k];
      // sum_b rstd (dy - s1/nb - xh s2/nb) = rstd (s1 - s1 - sx s2 / nb)
      (is_mu ? m.g_b_mu : m.g_b_s)[k] = rstd * (s1 - s1 - sx * s2 * inv_nb);
    }
    if (m.learn_priors) {
      for (int k = tid; k < K; k += PT) {
        const float pm = m.prior_mean[k], pv = m.prior_var[k];
        const float smu = cs[4 * K + k], svar = cs[6 * K + k], sdm2 = cs[7 * K + k];
        m.g_prior_mean[k] = wk * ((float)nb * pm - smu) / pv;
        m.g_prior_var[k] = wk * 0.5f * ((float)nb / pv - svar / (pv * pv) - sdm2 / (pv * pv));
      }
    }
    if (m.kind == GFK_LDA)
      for (int k = tid; k < K; k += PT) m.ws_ck[k] = cs[8 * K + k];
  }
  // ---- BN backward of the heads for the own rows ----
  for (int t = tid; t < RPB * 2 * K; t += PT) {
    const int r = t / (2 * K), c2 = t % (2 * K);
    const int row = r0 + r;
    const bool is_mu = c2 < K;
    const int k = is_mu ? c2 : c2 - K;
    float v = 0.f;
    if (row < nb) {
      const size_t i = (size_t)row * K + k;
      const float dy = (is_mu ? m.ws_dmu : m.ws_dls)[i];
      const float xh = (is_mu ? m.ws_mu : m.ws_ls)[i];
      const float s1 = cs[(is_mu ? 0 : 2) * K + k] * inv_nb, s2 = cs[(is_mu ? 1 : 3) * K + k] * inv_nb;
      v = m.ws_bn_rstd[c2] * (dy - s1 - xh * s2);
    }
    (is_mu ? dmr : dlr)[r * K + k] = v;
  }
  __syncthreads();
  GFK_STAMP(m, 12);
  // ---- heads: weight gradients (own rows' share) and d hd ----
  const float* Wmu = staged ? wst : m.w_mu;
  const float* Ws = m.w_s;
  {
    const float* wcur = wst;
    for (int l = 0; l + 1 < nh; ++l) wcur += pad4(m.H[l + 1] * m.H[l]) + pad4(m.H[l + 1]);
    if (staged) { Wmu = wcur; Ws = wcur + pad4(K * Hl) + pad4(K); }
  }
  {
    // weight gradients: the own rows' share sum_q dy[q]^T hd[q] (one MFMA k-step)
    const MatView Amu{dmr, 1, K, K, RPB}, As{dlr, 1, K, K, RPB};   // A[k][q] = dy[q][k]
    const MatView Bh{av, Hl, 1, RPB, Hl};                          // B[q][j] = hd[q][j]
    float *gwm = m.g_w_mu, *gws = m.g_w_s;
    mfma_gemm(K, Hl, RPB, Amu, Bh, wave, PT / 64, [&](int k, int j, float v) {
      atomicAdd(gwm + k * Hl + j, v);
    });
    mfma_gemm(K, Hl, RPB, As, Bh, wave, PT / 64, [&](int k, int j, float v) {
      atomicAdd(gws + k * Hl + j, v);
    });
    // d hd = dmu_raw W_mu + dls_raw W_s, through the encoder dropout
    const MatView Dm{dmr, K, 1, RPB, K}, Ds{dlr, K, 1, RPB, K};
    const MatView Wm{Wmu, Hl, 1, K, Hl}, Wsv{Ws, Hl, 1, K, Hl};
    mfma_gemm(RPB, Hl, K, Dm, Wm, wave, PT / 64, [&](int q, int j, float v) { dh[q * hm + j] = v; });
    __syncthreads();
    mfma_gemm(RPB, Hl, K, Ds, Wsv, wave, PT / 64, [&](int q, int j, float v) {
      const int row = r0 + q;
      const float mk = row < nb ? m.ws_mask_h[(size_t)row * Hl + j] : 0.f;
      dh[q * hm + j] = (dh[q * hm + j] + v) * mk;
    });
  }
  __syncthreads();
  GFK_STAMP(m, 13);
  // ---- hidden layers, last to first (own rows) ----
  for (int l = nh - 2; l >= 0; --l) {
    const int Hi = m.H[l], Ho = m.H[l + 1];
    const float* W = m.w_h[l];
    if (staged) {
      const float* p = wst;
      for (int ll = 0; ll < l; ++ll) p += pad4(m.H[ll + 1] * m.H[ll]) + pad4(m.H[ll + 1]);
      W = p;
    }
    for (int t = tid; t < RPB * Ho; t += PT) {
      const int q = t / Ho, j = t % Ho, row = r0 + q;
      const float z = m.ws_z[l + 1][(size_t)min(row, m.bmax - 1) * Ho + j];
      dh[q * hm + j] = row < nb ? dh[q * hm + j] * act_d(m.act, z) : 0.f;
    }
    for (int t = tid; t < RPB * Hi; t += PT) {
      const int q = t / Hi, i = t % Hi, row = r0 + q;
      av[q * hm + i] = m.ws_a[l][(size_t)min(row, m.bmax - 1) * Hi + i];
    }
    __syncthreads();
    {
      const MatView dZt{dh, 1, hm, Ho, RPB};   // A[j][q] = dz[q][j]
      const MatView Av{av, hm, 1, RPB, Hi};    // B[q][i] = a_l[q][i]
      float* gw = m.g_w_h[l];
      mfma_gemm(Ho, Hi, RPB, dZt, Av, wave, PT / 64, [&](int j, int i, float v) {
        atomicAdd(gw + j * Hi + i, v);
      });
    }
    for (int j = tid; j < Ho; j += PT) {
      float g = 0.f;
#pragma unroll
      for (int q = 0; q < RPB; ++q) g += dh[q * hm + j];
      atomicAdd(m.g_b_h[l] + j, g);
    }
    {
      const MatView dZ{dh, hm, 1, RPB, Ho};    // A[q][j]
      const MatView Wv{W, Hi, 1, Ho, Hi};      // B[j][i] = W[j][i]
      mfma_gemm(RPB, Hi, Ho, dZ, Wv, wave, PT / 64, [&](int q, int i, float v) { dh2[q * hm + i] = v; });
    }
    __syncthreads();
    float* tmp = dh; dh = dh2; dh2 = tmp;
  }
  // ---- input layer: dz0, its bias, and the sparse scatter into W_in^T ----
  for (int t = tid; t < RPB * H0; t += PT) {
    const int q = t / H0, j = t % H0, row = r0 + q;
    float g = 0.f;
    if (row < nb) g = dh[q * hm + j] * act_d(m.act, m.ws_z[0][(size_t)row * H0 + j]);
    dh[q * hm + j] = g;
    if (row < m.bmax) m.ws_dz0[(size_t)row * H0 + j] = g;
  }
  __syncthreads();
  for (int j = tid; j < H0; j += PT) {
    float g = 0.f;
#pragma unroll
    for (int q = 0; q < RPB; ++q) g += dh[q * hm + j];
    atomicAdd(m.g_b_in + j, g);
  }
  GFK_STAMP(m, 14);
  if (m.input != GFK_IN_CONTEXTUAL) {   // wave q scatters row r0 + q
    const int row = r0 + wave;
    if (row < nb) {
      const int doc = m.ws_doc[row];
      const int e0 = m.indptr[doc], e1 = m.indptr[doc + 1];
      for (int base = e0; base < e1; base += 256) {
        int vq[4];
        float xq[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // up to 256 (index, count) pairs in one round trip
          const int e = min(base + 64 * q + lane, e1 - 1);
          vq[q] = m.indices[e];
          xq[q] = m.values[e];
        }
        const int cnt = min(256, e1 - base);
        for (int j0 = 0; j0 < H0; j0 += 64) {
          const int j = j0 + lane;
          const float d = dh[wave * hm + min(j, H0 - 1)];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = min(64, cnt - 64 * q);
            for (int i = 0; i < n; ++i) {
              const int v = __shfl(vq[q], i, 64);
              const float x = __shfl(xq[q], i, 64);
              if (j < H0) atomicAdd(m.g_w_in + (size_t)v * H0 + j, x * d);
            }
          }
        }
      }
    }
  }
  GFK_STAMP(m, 15);
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
  hipLaunchKernelGGL(gfk_posterior_bwd_mlp, dim3(m->bmax / RPB), dim3(PT),
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
