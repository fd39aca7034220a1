// Fused multi-tensor Adam over the flat parameter buffer + FedAvg pre-scale.
//
// torch.optim.Adam semantics (reference avitm.py:141-143: betas=(momentum, 0.99),
// eps 1e-8, no weight decay by default):
//   m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2
//   p = p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// One launch covers every parameter tensor (segments of the flat buffer), reads
// the step count t from device memory (graph-replay safe), clears the gradient
// it consumed (so scatter-accumulated gradients start from zero next step) and,
// on segments flagged for FedAvg, multiplies the result by w_i = n_i / sum n so
// the following all-reduce(SUM) directly yields the sample-weighted average.
// float4 vectorised: segment bounds are multiples of 4 floats.
#include "gfk_common.h"

namespace {
constexpr int ADAM_THREADS = 256;
}

extern "C" __global__ void __launch_bounds__(ADAM_THREADS) gfk_adam_kernel(GfkAdam a) {
  const int t = *a.t;
  const float bc1 = 1.f - powf(a.beta1, (float)t);
  const float bc2 = 1.f - powf(a.beta2, (float)t);
  const float step_size = a.lr / bc1;
  const float bc2_sqrt = sqrtf(bc2);
  const int64_t nthreads = (int64_t)gridDim.x * ADAM_THREADS;
  const int64_t gtid = (int64_t)blockIdx.x * ADAM_THREADS + threadIdx.x;
  for (int s = 0; s < a.n_seg; ++s) {
    const int64_t s0 = a.seg_start[s], n4 = (a.seg_end[s] - s0) >> 2;
    const int flags = a.seg_flags[s];
    const bool do_adam = flags & 1, do_scale = flags & 2;
    for (int64_t i = gtid; i < n4; i += nthreads) {
      const int64_t o = s0 + 4 * i;
      float4 p = *reinterpret_cast<float4*>(a.p + o);
      if (do_adam) {
        float4 g = *reinterpret_cast<float4*>(a.g + o);
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
        *reinterpret_cast<float4*>(a.g + o) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (do_scale) { p.x *= a.scale; p.y *= a.scale; p.z *= a.scale; p.w *= a.scale; }
      if (do_adam || do_scale) *reinterpret_cast<float4*>(a.p + o) = p;
    }
  }
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
