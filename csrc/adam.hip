// Fused multi-tensor Adam over the flat parameter buffer + FedAvg pre-scale.
//
// torch.optim.Adam semantics (reference avitm.py:141-143: betas=(momentum, 0.99),
// eps 1e-8, no weight decay by default):
//   m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2
//   p = p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// One launch covers every parameter tensor (segments of the flat buffer), reads
// the step count t from device memory (graph-replay safe), clears the gradient
// it consumed (so scatter-accumulated gradients start from zero next step) --
// or, for the small MLP tensors, sums the per-workgroup gradient slabs written by
// posterior_bwd_mlp in a fixed order (so those gradients need no atomics) -- and,
// on segments flagged for FedAvg, multiplies the result by w_i = n_i / sum n so
// the following all-reduce(SUM) directly yields the sample-weighted average.
// float4 vectorised: segment bounds are multiples of 4 floats.
#include "gfk_common.h"

namespace {
constexpr int ADAM_THREADS = 256;
}

// Workgroups are dealt to segments in proportion to their size (blocks
// [seg_block[s], seg_block[s+1]) own segment s), so a thread touches one segment
// only; slab gradients are summed with all loads of a float4 issued at once.
extern "C" __global__ void __launch_bounds__(ADAM_THREADS) gfk_adam_kernel(GfkAdam a) {
  GFK_STAMP(a, 32);
  const int t = *a.t;
  const float bc1 = 1.f - powf(a.beta1, (float)t);
  const float bc2 = 1.f - powf(a.beta2, (float)t);
  const float step_size = a.lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  // find this block's segment: lane i reads segment i's first block (host
  // precomputed, one vector load), a ballot counts the segments starting at or
  // before this block.  One round trip instead of a scalar chain per segment.
  const int lane = threadIdx.x & 63;
  const int nseg = a.n_seg;
  const int fb = lane < nseg ? a.seg_first_block[lane] : 0x7fffffff;
  const uint64_t le = __ballot(fb <= (int)blockIdx.x);
  const int s = __popcll(le) - 1;
  if (s < 0 || s >= nseg) return;
  const int64_t first = a.seg_first_block[s];
  GFK_STAMP(a, 33);
  const int64_t s0 = a.seg_start[s], n4 = (a.seg_end[s] - s0) >> 2;
  const int flags = a.seg_flags[s];
  const bool do_adam = flags & 1, do_scale = flags & 2;
  const float* slab = a.seg_slab[s];
  constexpr int PER = 4;   // float4s per thread
  const int64_t base = ((int64_t)blockIdx.x - first) * ADAM_THREADS * PER + threadIdx.x;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int64_t i = base + u * ADAM_THREADS;
    if (i >= n4) continue;
    const int64_t o = s0 + 4 * i;
    float4 p = *reinterpret_cast<float4*>(a.p + o);
    if (do_adam) {
      float4 g;
      if (slab) {   // fixed-order reduction of the per-workgroup partial gradients
        constexpr int MAXS = 32;
        float4 q[MAXS];
#pragma unroll
        for (int j = 0; j < MAXS; ++j)
          q[j] = *reinterpret_cast<const float4*>(slab + (int64_t)min(j, a.n_slab - 1) * a.slab_stride +
                                                  4 * i);
        g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < MAXS; ++j)
          if (j < a.n_slab) { g.x += q[j].x; g.y += q[j].y; g.z += q[j].z; g.w += q[j].w; }
      } else {
        g = *reinterpret_cast<float4*>(a.g + o);
      }
      float4 m = *reinterpret_cast<float4*>(a.m + o);
      float4 v = *reinterpret_cast<float4*>(a.v + o);
      float* pp = &p.x; float* gg = &g.x; float* mm = &m.x; float* vv = &v.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gj = gg[j];
        if (a.weight_decay != 0.f) gj += a.weight_decay * pp[j];
        mm[j] += (1.f - a.beta1) * (gj - mm[j]);
        vv[j] = a.beta2 * vv[j] + (1.f - a.beta2) * gj * gj;
        const float denom = sqrtf(vv[j]) / bc2_sqrt + a.eps;
        pp[j] -= step_size * mm[j] / denom;
      }
      *reinterpret_cast<float4*>(a.m + o) = m;
      *reinterpret_cast<float4*>(a.v + o) = v;
      if (!slab) *reinterpret_cast<float4*>(a.g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (do_scale) { p.x *= a.scale; p.y *= a.scale; p.z *= a.scale; p.w *= a.scale; }
    if (do_adam || do_scale) *reinterpret_cast<float4*>(a.p + o) = p;
  }
  GFK_STAMP(a, 34);
}

// Weighted in-place scale of a flat range (FedAvg pre-scale outside Adam, e.g.
// for the gradient-averaging mode or non-Adam solvers).
extern "C" __global__ void gfk_scale_kernel(float* p, int64_t n, float s) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] *= s;
}

extern "C" int gfk_launch_adam(const GfkAdam* a, int grid, hipStream_t s) {
  hipLaunchKernelGGL(gfk_adam_kernel, dim3(grid), dim3(ADAM_THREADS), 0, s, *a);
  return (int)hipGetLastError();
}

extern "C" int gfk_launch_scale(float* p, int64_t n, float sc, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(gfk_scale_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, p, n, sc);
  return (int)hipGetLastError();
}
