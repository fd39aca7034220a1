// Achievable HBM bandwidth of the beta Adam read-modify-write (p, m, v of a [K, V]
// fp32 matrix, 64-column vocab tiles) under three access patterns:
//   mfma   : the MFMA output layout of prodlda_bwd (lane -> 4 rows x 1 column; a wave
//            instruction touches 4 rows x 64 B), quarter-K ranges, 512 threads
//   rows4  : the same tiles, float4 per lane along a row (a wave instruction: 4 rows x
//            256 B), quarter-K ranges, 512 threads
//   flat4  : one flat float4 stream over the three arrays (the ceiling)
// Each kernel reads p, m, v and writes all three once (no LDS, no compute to speak of).
#include <hip/hip_runtime.h>

__device__ __forceinline__ float upd(float p, float& m, float& v) {
  m = 0.9f * m + 0.1f * p;
  v = 0.99f * v + 0.01f * p * p;
  return p - 1e-3f * m / (sqrtf(v) + 1e-8f);
}

// grid: slabs * 4; workgroup g: quarter q = g % 4 of tiles g/4, g/4 + slabs, ...
__global__ void __launch_bounds__(512) rmw_mfma(float* p, float* m, float* v, int K, int V,
                                                int n_tiles) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = blockIdx.x % 4, slab = blockIdx.x / 4, nslab = gridDim.x / 4;
  const int ksub = (K + 15) / 16, ks0 = q * ksub / 4, nks = (q + 1) * ksub / 4 - ks0;
  for (int tile = slab; tile < n_tiles; tile += nslab) {
    const int c0 = tile * 64;
    float pm[2][4], mm[2][4], vm[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 8 * u, ks = ks0 + t / 4, cs = t % 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = min(ks * 16 + (lane >> 4) * 4 + r, K - 1);
        const size_t o = (size_t)k * V + min(c0 + cs * 16 + (lane & 15), V - 1);
        pm[u][r] = p[o]; mm[u][r] = m[o]; vm[u][r] = v[o];
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = wave + 8 * u, ks = ks0 + t / 4, cs = t % 4;
      if (t >= 4 * nks) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = ks * 16 + (lane >> 4) * 4 + r, c = c0 + cs * 16 + (lane & 15);
        if (k >= K || c >= V) continue;
        const size_t o = (size_t)k * V + c;
        float mo = mm[u][r], vo = vm[u][r];
        const float np = upd(pm[u][r], mo, vo);
        p[o] = np; m[o] = mo; v[o] = vo;
      }
    }
  }
}

__global__ void __launch_bounds__(512) rmw_rows4(float* p, float* m, float* v, int K, int V,
                                                 int n_tiles) {
  const int tid = threadIdx.x;
  const int q = blockIdx.x % 4, slab = blockIdx.x / 4, nslab = gridDim.x / 4;
  const int ksub = (K + 15) / 16, ks0 = q * ksub / 4, nks = (q + 1) * ksub / 4 - ks0;
  const int k0 = 16 * ks0, nk = min(16 * nks, K - k0);
  for (int tile = slab; tile < n_tiles; tile += nslab) {
    const int c0 = tile * 64;
    // 16 lanes per row (float4 each), 32 rows per pass, up to 64 rows: 2 passes
    float4 pp[2], mm[2], vv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int k = k0 + min(tid / 16 + 32 * u, nk - 1), c = c0 + 4 * (tid % 16);
      const size_t o = (size_t)k * V + min(c, V - 4);
      pp[u] = *reinterpret_cast<const float4*>(p + o);
      mm[u] = *reinterpret_cast<const float4*>(m + o);
      vv[u] = *reinterpret_cast<const float4*>(v + o);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int kr = tid / 16 + 32 * u, c = c0 + 4 * (tid % 16);
      if (kr >= nk || c >= V) continue;
      const size_t o = (size_t)(k0 + kr) * V + c;
      float* a = &pp[u].x; float* b = &mm[u].x; float* d = &vv[u].x;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = upd(a[j], b[j], d[j]);
      *reinterpret_cast<float4*>(p + o) = pp[u];
      *reinterpret_cast<float4*>(m + o) = mm[u];
      *reinterpret_cast<float4*>(v + o) = vv[u];
    }
  }
}

// rows1: the pipelined prodlda backward's pattern -- one dword per lane along a row (a wave
// instruction: one row x 256 B), 8 rows per thread, quarter-K ranges, 512 threads
__global__ void __launch_bounds__(512) rmw_rows1(float* p, float* m, float* v, int K, int V,
                                                 int n_tiles) {
  const int tid = threadIdx.x;
  const int q = blockIdx.x % 4, slab = blockIdx.x / 4, nslab = gridDim.x / 4;
  const int ksub = (K + 15) / 16, ks0 = q * ksub / 4, nks = (q + 1) * ksub / 4 - ks0;
  const int k0 = 16 * ks0, nk = min(16 * nks, K - k0);
  for (int tile = slab; tile < n_tiles; tile += nslab) {
    const int c = min(tile * 64 + (tid & 63), V - 1);
    float pp[8], mm[8], vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t o = (size_t)(k0 + min(tid / 64 + 8 * u, nk - 1)) * V + c;
      pp[u] = p[o]; mm[u] = m[o]; vv[u] = v[o];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int kr = tid / 64 + 8 * u;
      if (kr >= nk || tile * 64 + (tid & 63) >= V) continue;
      const size_t o = (size_t)(k0 + kr) * V + c;
      const float np = upd(pp[u], mm[u], vv[u]);
      p[o] = np; m[o] = mm[u]; v[o] = vv[u];
    }
  }
}

__global__ void __launch_bounds__(256) rmw_flat4(float4* p, float4* m, float4* v, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 a = p[i], b = m[i], d = v[i];
    float* x = &a.x; float* y = &b.x; float* z = &d.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = upd(x[j], y[j], z[j]);
    p[i] = a; m[i] = b; v[i] = d;
  }
}

extern "C" int launch(int which, float* p, float* m, float* v, int K, int V, int grid,
                      hipStream_t s) {
  const int n_tiles = (V + 63) / 64;
  if (which == 0) hipLaunchKernelGGL(rmw_mfma, dim3(grid), dim3(512), 0, s, p, m, v, K, V, n_tiles);
  else if (which == 1) hipLaunchKernelGGL(rmw_rows4, dim3(grid), dim3(512), 0, s, p, m, v, K, V, n_tiles);
  else if (which == 3) hipLaunchKernelGGL(rmw_rows1, dim3(grid), dim3(512), 0, s, p, m, v, K, V, n_tiles);
  else hipLaunchKernelGGL(rmw_flat4, dim3(grid), dim3(256), 0, s, (float4*)p, (float4*)m, (float4*)v,
                          (long)K * V / 4);
  return (int)hipGetLastError();
}
