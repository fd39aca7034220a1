// Latency microbenchmarks (diagnostic, not part of the framework):
//  chase    : one lane follows a pointer ring; cycles (s_memtime) and 100 MHz
//             ticks (s_memrealtime) per dependent load
//  sload    : dependent scalar loads (kernel-argument style) through a ring
//  writer   : a kernel writing a buffer, so the next chase reads data produced
//             by another kernel (other XCDs' L2)
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void chase_kernel(const int* __restrict__ ring, int n, uint64_t* out) {
  if (threadIdx.x != 0) return;
  int idx = 0;
  // warm the first element's translation
  idx = __builtin_nontemporal_load(ring);
  idx = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) idx = __atomic_load_n(ring + idx, __ATOMIC_RELAXED);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  out[0] = t1 - t0;
  out[1] = r1 - r0;
  out[2] = idx;
}

extern "C" __global__ void sload_kernel(const int* __restrict__ ring, int n, uint64_t* out) {
  int idx = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < n; ++i) idx = __builtin_amdgcn_readfirstlane(ring[idx]);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; out[2] = idx; }
}

extern "C" __global__ void writer_kernel(int* ring, int n, int stride) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    ring[i] = ((i / stride + 1) * stride) % n;   // same ring, rewritten
}

extern "C" __global__ void empty_kernel() {}

extern "C" int launch_chase(const int* ring, int n, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(chase_kernel, dim3(1), dim3(64), 0, s, ring, n, out);
  return (int)hipGetLastError();
}
extern "C" int launch_sload(const int* ring, int n, uint64_t* out, hipStream_t s) {
  hipLaunchKernelGGL(sload_kernel, dim3(1), dim3(64), 0, s, ring, n, out);
  return (int)hipGetLastError();
}
extern "C" int launch_writer(int* ring, int n, int stride, hipStream_t s) {
  hipLaunchKernelGGL(writer_kernel, dim3(512), dim3(256), 0, s, ring, n, stride);
  return (int)hipGetLastError();
}
extern "C" int launch_empty(int grid, hipStream_t s) {
  hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(64), 0, s);
  return (int)hipGetLastError();
}

// writes n floats (grid-stride), optionally with non-temporal stores
extern "C" __global__ void wr_kernel(float* p, int n, int nt) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (nt) __builtin_nontemporal_store(1.0f, p + i);
    else p[i] = 1.0f;
  }
}
// reads n floats written by the previous kernel and writes one value per block
extern "C" __global__ void rd_kernel(const float* p, int n, float* out) {
  float s = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += p[i];
  if (s == 12345.f) out[blockIdx.x] = s;
}
extern "C" int launch_wr(float* p, int n, int nt, int grid, hipStream_t s) {
  hipLaunchKernelGGL(wr_kernel, dim3(grid), dim3(256), 0, s, p, n, nt);
  return (int)hipGetLastError();
}
extern "C" int launch_rd(const float* p, int n, float* out, int grid, hipStream_t s) {
  hipLaunchKernelGGL(rd_kernel, dim3(grid), dim3(256), 0, s, p, n, out);
  return (int)hipGetLastError();
}
