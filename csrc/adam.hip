// Fused multi-tensor Adam over the flat parameter buffer + FedAvg pre-scale.
//
// Gradient mode of the fused step (and non-fused tensors).  torch.optim.Adam
// semantics (reference avitm.py:141-143: betas=(momentum, 0.99),
// eps 1e-8, no weight decay by default):
//   m = m + (1-b1)(g - m);  v = b2 v + (1-b2) g^2
//   p = p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
// One launch covers every parameter tensor (segments of the flat buffer), reads
// the step count t from device memory (graph-replay safe), clears the gradient
// it consumed, and,
// on segments flagged for FedAvg, multiplies the result by w_i = n_i / sum n so
// the following all-reduce(SUM) directly yields the sample-weighted average.
// float4 vectorised: segment bounds are multiples of 4 floats.
#define GFK_BATCHED_COPY 1   // batched kernels copy their descriptor (gfk_common.h gfk_model)
#include "gfk_common.h"

using namespace gfk;

namespace {
constexpr int ADAM_THREADS = 256;
}

extern "C" __global__ void __launch_bounds__(ADAM_THREADS) gfk_adam_kernel(GfkAdam a) {
  adam_block(a, blockIdx.x, threadIdx.x, ADAM_THREADS);
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
