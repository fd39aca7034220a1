// Kernel-argument size microbenchmark (diagnostic): per-kernel time inside a
// hipGraph for (a) a tiny argument list, (b) a 1.5 KB struct passed by value
// (the fused step's GfkModel style), (c) a pointer to the same struct in device
// memory; each kernel reads two fields and writes one value per workgroup.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

struct Big {
  float* out;
  int a[380];
  int b;
};

__global__ void k_small(float* out, int a, int b) {
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(a + b);
}
__global__ void k_big(Big m) {
  if (threadIdx.x == 0) m.out[blockIdx.x] = (float)(m.a[7] + m.b);
}
__global__ void k_ptr(const Big* __restrict__ m) {
  if (threadIdx.x == 0) m->out[blockIdx.x] = (float)(m->a[7] + m->b);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <class F>
static int timed(const char* name, hipStream_t s, F launch, int grid) {
  const int N = 200;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < N; ++i) launch();
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("%-28s grid %4d: %.3f us/kernel\n", name, grid, 1000.f * ms / (10 * N));
  return 0;
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  float* out;
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  Big h{};
  h.out = out;
  h.b = 3;
  Big* d;
  CK(hipMalloc(&d, sizeof(Big)));
  CK(hipMemcpy(d, &h, sizeof(Big), hipMemcpyHostToDevice));
  printf("sizeof(Big) = %zu\n", sizeof(Big));
  for (int grid : {64, 256}) {
    timed("small args", s, [&] { hipLaunchKernelGGL(k_small, dim3(grid), dim3(256), 0, s, out, 1, 2); }, grid);
    timed("1.5 KB struct by value", s, [&] { hipLaunchKernelGGL(k_big, dim3(grid), dim3(256), 0, s, h); }, grid);
    timed("pointer to device struct", s, [&] { hipLaunchKernelGGL(k_ptr, dim3(grid), dim3(256), 0, s, d); }, grid);
  }
  return 0;
}
