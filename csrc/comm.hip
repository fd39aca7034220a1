// Deterministic two-shot all-reduce (SUM) over xGMI peer memory, for the
// per-round FedAvg of the pre-scaled shared state (reference server.py:477-487:
// sum_i n_i W_i / sum n, here sum_i (w_i W_i) with w_i applied by the update
// kernels).
//
// Every rank owns a double-buffered stage [2][world * chunk] floats and a flag
// array [2 phases][nblk][8] (uncached), both IPC-mapped into every peer.  The
// n floats are cut into `world` chunks; chunk c is cut into `nblk` slices, and
// workgroup b of every rank handles slice b of each chunk, so every data
// dependency is per (workgroup, slice) and no grid-wide barrier is needed:
//   phase 0  copy slice b of all chunks into my stage (write-through, system
//            scope), then tell every rank (flag[0][b][me] = epoch);
//   phase 1  once all ranks published: chunk me, slice b = sum over ranks in
//            RANK ORDER (bit-identical everywhere: each chunk is summed by
//            exactly one rank), into my stage and my output; flag[1][b][me];
//   phase 2  once all ranks reduced: copy the other chunks' slice b from their
//            owners' stages into my output.
// Round e uses stage buffer e & 1: a rank starts overwriting a buffer only
// after every rank passed the next round's phase 0, i.e. finished reading it.
// The per-workgroup epoch lives in device memory (so hipGraph replays advance
// it); every wait is bounded: on timeout the workgroup records an error word and
// finishes (the host checks it), it never hangs the device.
//
// In-place mode (large shared states, e.g. beta at V ~ 100k: 90 MB): the data buffer
// itself is IPC-mapped into every peer, so phase 0 is only the publish (no copy of the
// whole state into the stage: 2 S of local HBM traffic saved); phase 1 writes the reduced
// chunk back into the data with system-scope stores; and a phase 3 publish / await keeps
// every rank from returning -- and its next step from overwriting its data -- before all
// peers have read their chunks from it.  The system release in the phase-0 publish writes
// the step kernels' dirty L2 lines back, so the peers' system-scope loads see them.
//
// Visibility across devices (MI355X_MICROARCH.md inter-workgroup rules, lifted
// to system scope): payload stores sc0 sc1 (write-through) -> s_waitcnt
// vmcnt(0) -> barrier -> system release -> one lane per rank stores the flag at
// system scope; consumers poll relaxed at system scope, one system acquire, then
// sc0 sc1 loads of the payload.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int CMAX = 8;          // ranks (one node)
constexpr int CT = 256;          // threads per workgroup
constexpr int AUX_SYS = 17;      // cache policy sc0 | sc1: system coherence

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
}  // namespace

struct GfkComm {
  float* stage[2][CMAX];         // every rank's stage buffers (own one included); in-place:
                                 // every rank's DATA buffer (both entries)
  uint32_t* flags[CMAX];         // every rank's flag array [2 (3 in-place)][nblk][CMAX]
  uint32_t* epoch;               // own per-workgroup round counter [nblk]
  int32_t* err;                  // own error word (timeouts)
  int32_t rank, world, nblk, spin_limit;
  int64_t n, chunk, slice;       // floats; chunk, slice multiples of 4
  int32_t inplace, pad;          // 1: the data buffers themselves are IPC-mapped (no stage)
  // bf16-delta wire (gfk_xgmi_allreduce_bf16d): the stages hold bf16; ref = this rank's copy
  // of the last averaged state (n floats), wgt = this rank's FedAvg weight sum
  float* ref;
  float wgt;
  int32_t wire;                  // 0: fp32 sum (gfk_xgmi_allreduce), 1: bf16 deltas
};

namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ float4 ld_sys(__amdgpu_buffer_rsrc_t r, int64_t i) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 4), 0, AUX_SYS);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}

__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, int64_t i, float4 f) {
  u32x4 v;
  v.x = __float_as_uint(f.x); v.y = __float_as_uint(f.y);
  v.z = __float_as_uint(f.z); v.w = __float_as_uint(f.w);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(i * 4), 0, AUX_SYS);
}

__device__ __forceinline__ float ld_sys1(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4), 0, AUX_SYS));
}

__device__ __forceinline__ void st_sys1(__amdgpu_buffer_rsrc_t r, int64_t i, float f) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(f), r, (int)(i * 4), 0, AUX_SYS);
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// All storing waves drained, then one lane per destination rank raises the flag.
// The flag goes through this rank's IPC mapping of the peer's flag array, which may be
// cached in this XCD's L2 (same-device mappings of coarse-grained memory are; a peer GPU's
// lines may be too): the store is followed by an L2 write-back, so the flag reaches
// memory now and not at the next write-back of this L2.  Without it a 2-rank rehearsal
// on one GPU intermittently left a rank spinning to the wait bound (g9 / g16 / g17: error
// 2 on one rank, every epoch and flag correct once the other kernel's end-of-kernel
// release had written its L2 back).
__device__ __forceinline__ void publish(const GfkComm& c, int phase, int b, uint32_t e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  if (t < c.world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(c.flags[t] + ((size_t)phase * c.nblk + b) * CMAX + c.rank, e,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
}

// Wave 0 polls this workgroup's flag row until every rank reached epoch e.
__device__ __forceinline__ void await_all(const GfkComm& c, int phase, int b, uint32_t e) {
  const int t = threadIdx.x;
  if (t < 64) {
    const uint32_t* f = c.flags[c.rank] + ((size_t)phase * c.nblk + b) * CMAX;
    int spins = 0;
    for (;;) {
      uint32_t v = e;
      if (t < c.world) v = __hip_atomic_load(f + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (__all((int32_t)(v - e) >= 0)) break;
      if (++spins > c.spin_limit) {
        if (t == 0) __hip_atomic_store(c.err, 1 + phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

__device__ __forceinline__ void slice_range(const GfkComm& c, int ch, int b, int64_t& s0, int64_t& s1) {
  const int64_t c0 = (int64_t)ch * c.chunk, c1 = c0 + c.chunk < c.n ? c0 + c.chunk : c.n;
  s0 = c0 + (int64_t)b * c.slice;
  s1 = s0 + c.slice < c1 ? s0 + c.slice : c1;
}
}  // namespace

// No LDS at all (the epoch is read by every thread before thread 0 advances it): a kernel
// that waits on peers must not hold LDS a co-running kernel needs -- CombinedTM's ctx_bwd
// takes a whole CU's LDS, and a spinning all-reduce workgroup with even 4 bytes of it on
// every CU kept ctx_bwd from launching (a 2-rank one-GPU rehearsal waited out its bound).
extern "C" __global__ void __launch_bounds__(CT) gfk_xgmi_allreduce(GfkComm c, float* data) {
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t e = c.epoch[b] + 1;
  __syncthreads();
  if (t == 0) c.epoch[b] = e;
  const int buf = e & 1, R = c.rank, W = c.world;
  const int64_t sbytes = (int64_t)W * c.chunk * 4;
  const __amdgpu_buffer_rsrc_t mine = rsrc(c.stage[buf][R], sbytes);

  // (slices are float4-aligned; only the last one of the last chunk can end in a
  // partial float4, handled element-wise: nothing past n is ever touched)
  // ---- phase 0: publish slice b of every chunk (in-place: the data is the stage) ----
  if (!c.inplace) {
    for (int ch = 0; ch < W; ++ch) {
      int64_t s0, s1;
      slice_range(c, ch, b, s0, s1);
      const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
      for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT)
        st_sys(mine, i, *reinterpret_cast<const float4*>(data + i));
      if (s4 + t < s1) st_sys1(mine, s4 + t, data[s4 + t]);
    }
  }
  publish(c, 0, b, e);
  await_all(c, 0, b, e);

  // ---- phase 1: my chunk, slice b: sum over ranks in rank order ----
  {
    int64_t s0, s1;
    slice_range(c, R, b, s0, s1);
    __amdgpu_buffer_rsrc_t src[CMAX];
#pragma unroll
    for (int j = 0; j < CMAX; ++j) src[j] = rsrc(c.stage[buf][j < W ? j : 0], sbytes);
    const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
    // (in-place: mine IS the data, so the system-scope store is the data update)
    if (s4 + t < s1) {
      float acc = ld_sys1(src[0], s4 + t);
      for (int j = 1; j < W; ++j) acc += ld_sys1(src[j], s4 + t);
      st_sys1(mine, s4 + t, acc);
      if (!c.inplace) data[s4 + t] = acc;
    }
    for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT) {
      float4 v[CMAX];
#pragma unroll
      for (int j = 0; j < CMAX; ++j)
        if (j < W) v[j] = ld_sys(src[j], i);
      float4 acc = v[0];
#pragma unroll
      for (int j = 1; j < CMAX; ++j)
        if (j < W) acc = add4(acc, v[j]);
      st_sys(mine, i, acc);
      if (!c.inplace) *reinterpret_cast<float4*>(data + i) = acc;
    }
  }
  publish(c, 1, b, e);
  await_all(c, 1, b, e);

  // ---- phase 2: the other chunks' slice b from their owners ----
  for (int ch = 0; ch < W; ++ch) {
    if (ch == R) continue;
    int64_t s0, s1;
    slice_range(c, ch, b, s0, s1);
    const __amdgpu_buffer_rsrc_t src = rsrc(c.stage[buf][ch], sbytes);
    const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
    for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT)
      *reinterpret_cast<float4*>(data + i) = ld_sys(src, i);
    if (s4 + t < s1) data[s4 + t] = ld_sys1(src, s4 + t);
  }
  // ---- phase 3 (in-place): nobody leaves while a peer may still read its data ----
  if (c.inplace) {
    publish(c, 2, b, e);
    await_all(c, 2, b, e);
  }
}

// ---------------------------------------------------------------------------
// bf16-delta wire (opt-in, --fedavg_wire bf16delta): half the bytes of the fp32 sum.
// Every rank holds ref = the last averaged state (identical on all ranks) and sends its
// pre-scaled state's DEPARTURE from it, d_r = f_r - w_r ref (sum_r w_r = 1, so
// sum_r d_r = W_new - ref), rounded to bf16 (RNE); the owner of a chunk sums the peers'
// bf16 deltas in fp32 in rank order and publishes the sum rounded to bf16, S; every rank
// (the owner too) sets W_new = ref + S and ref = W_new.  So the replicas stay bit-identical
// and the rounding touches only the per-round change (~lr), never the weights themselves.
// Same phases, flags, epochs and bounded waits as the fp32 kernel; always staged (the
// peers read deltas, not the state).  Stage: [2][world * chunk] bf16.
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint32_t bf16_bits(float f) {
  const __bf16 h = (__bf16)f;                      // v_cvt_pk_bf16_f32: round to nearest even
  return (uint32_t)__builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float bf16_val(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ uint2 pack4(float4 f) {
  return make_uint2(bf16_bits(f.x) | (bf16_bits(f.y) << 16), bf16_bits(f.z) | (bf16_bits(f.w) << 16));
}
__device__ __forceinline__ float4 unpack4(uint2 u) {
  return make_float4(bf16_val(u.x & 0xFFFFu), bf16_val(u.x >> 16), bf16_val(u.y & 0xFFFFu),
                     bf16_val(u.y >> 16));
}
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// element i of a bf16 stage (byte offset 2 i)
__device__ __forceinline__ uint2 ld4h(__amdgpu_buffer_rsrc_t r, int64_t i) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 2), 0, AUX_SYS);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void st4h(__amdgpu_buffer_rsrc_t r, int64_t i, uint2 u) {
  u32x2 v;
  v.x = u.x; v.y = u.y;
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)(i * 2), 0, AUX_SYS);
}
__device__ __forceinline__ uint32_t ld1h(__amdgpu_buffer_rsrc_t r, int64_t i) {
  return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, (int)(i * 2), 0, AUX_SYS);
}
__device__ __forceinline__ void st1h(__amdgpu_buffer_rsrc_t r, int64_t i, uint32_t b) {
  __builtin_amdgcn_raw_buffer_store_b16((unsigned short)b, r, (int)(i * 2), 0, AUX_SYS);
}
__device__ __forceinline__ float4 ld4f(const float* p, int64_t i) { return *reinterpret_cast<const float4*>(p + i); }
__device__ __forceinline__ void st4f(float* p, int64_t i, float4 v) { *reinterpret_cast<float4*>(p + i) = v; }
}  // namespace

extern "C" __global__ void __launch_bounds__(CT) gfk_xgmi_allreduce_bf16d(GfkComm c, float* data) {
  // (every product and sum rounded on its own: XgmiAllReduce.expected_bf16delta restates it)
#pragma clang fp contract(off)
  const int b = blockIdx.x, t = threadIdx.x;
  const uint32_t e = c.epoch[b] + 1;
  __syncthreads();
  if (t == 0) c.epoch[b] = e;
  const int buf = e & 1, R = c.rank, W = c.world;
  const int64_t sbytes = (int64_t)W * c.chunk * 2;
  const __amdgpu_buffer_rsrc_t mine = rsrc(c.stage[buf][R], sbytes);
  float* ref = c.ref;
  const float w = c.wgt;
  // ---- phase 0: my bf16 deltas of slice b of every chunk ----
  for (int ch = 0; ch < W; ++ch) {
    int64_t s0, s1;
    slice_range(c, ch, b, s0, s1);
    const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
    for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT) {
      const float4 d = ld4f(data, i), r = ld4f(ref, i);
      st4h(mine, i, pack4(make_float4(d.x - w * r.x, d.y - w * r.y, d.z - w * r.z, d.w - w * r.w)));
    }
    if (s4 + t < s1) st1h(mine, s4 + t, bf16_bits(data[s4 + t] - w * ref[s4 + t]));
  }
  publish(c, 0, b, e);
  await_all(c, 0, b, e);
  // ---- phase 1: my chunk, slice b: fp32 sum of the ranks' deltas in rank order ----
  {
    int64_t s0, s1;
    slice_range(c, R, b, s0, s1);
    __amdgpu_buffer_rsrc_t src[CMAX];
#pragma unroll
    for (int j = 0; j < CMAX; ++j) src[j] = rsrc(c.stage[buf][j < W ? j : 0], sbytes);
    const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
    if (s4 + t < s1) {
      float acc = bf16_val(ld1h(src[0], s4 + t));
      for (int j = 1; j < W; ++j) acc += bf16_val(ld1h(src[j], s4 + t));
      const uint32_t sb = bf16_bits(acc);
      st1h(mine, s4 + t, sb);
      const float wn = ref[s4 + t] + bf16_val(sb);
      data[s4 + t] = wn;
      ref[s4 + t] = wn;
    }
    for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT) {
      uint2 v[CMAX];
#pragma unroll
      for (int j = 0; j < CMAX; ++j)
        if (j < W) v[j] = ld4h(src[j], i);
      float4 acc = unpack4(v[0]);
#pragma unroll
      for (int j = 1; j < CMAX; ++j)
        if (j < W) acc = add4(acc, unpack4(v[j]));
      const uint2 sb = pack4(acc);
      st4h(mine, i, sb);
      const float4 wn = add4(ld4f(ref, i), unpack4(sb));
      st4f(data, i, wn);
      st4f(ref, i, wn);
    }
  }
  publish(c, 1, b, e);
  await_all(c, 1, b, e);
  // ---- phase 2: the other chunks' summed deltas from their owners ----
  for (int ch = 0; ch < W; ++ch) {
    if (ch == R) continue;
    int64_t s0, s1;
    slice_range(c, ch, b, s0, s1);
    const __amdgpu_buffer_rsrc_t src = rsrc(c.stage[buf][ch], sbytes);
    const int64_t s4 = s0 + ((s1 - s0) & ~(int64_t)3);
    for (int64_t i = s0 + 4 * t; i < s4; i += 4 * CT) {
      const float4 wn = add4(ld4f(ref, i), unpack4(ld4h(src, i)));
      st4f(data, i, wn);
      st4f(ref, i, wn);
    }
    if (s4 + t < s1) {
      const float wn = ref[s4 + t] + bf16_val(ld1h(src, s4 + t));
      data[s4 + t] = wn;
      ref[s4 + t] = wn;
    }
  }
}

// ---------------------------------------------------------------------------
// In-process FedAvg of N simulated clients on one GPU (LocalFederation), and the
// in-rank half of the hierarchical FedAvg of a rank that hosts several clients
// (run_distributed with more clients than ranks).  Every client's pre-scaled shared
// state f_i is summed as a left fold per GROUP of consecutive clients, and the group
// sums as a left fold in group order:  sum = (f_0 + .. + f_{e0-1}) + (f_{e0} + ..) + ..
// With one group this is the plain client-order sum; with one group per rank it is
// exactly the order of "each rank folds its own clients, then the xGMI kernel folds
// the ranks' partial sums in rank order" -- so a one-GPU simulation and the multi-rank
// run agree bit for bit.  Modes:
//   0  the sum is written back to every client's buffer (LocalFederation round);
//   1  the sum is written to f_0 only (a rank's local partial, before the collective);
//   2  broadcast: f_0 is copied into f_1 .. f_{n-1} (after the collective).
// One launch replaces the 2N + 1 eager kernels of a zero / add / copy sequence and is
// captured into the round graphs.  The client buffers and the group ends come from small
// DEVICE tables (uploaded once per client set, before any capture), so the number of
// clients a rank folds is not bounded by the kernel's argument block.  [off, off + n) is
// the float range folded in every buffer (the whole shared state, or only beta's part
// when it is reduced ahead of the rest); off is a multiple of 4, the pointers 16-byte
// aligned, and a partial last float4 is handled element-wise.
// ---------------------------------------------------------------------------
struct GfkLocalAvg {
  const uint64_t* f;             // device table [n_clients]: float* of every client's buffer
  const int32_t* gend;           // device table [n_groups]: exclusive end of each group
  int64_t off;                   // first float of the folded range
  int64_t n;                     // floats in the range
  int32_t n_clients;
  int32_t mode;
  int32_t n_groups;
  int32_t pad;
};

namespace {
template <class T>
__device__ __forceinline__ T* lptr(const GfkLocalAvg& a, int j) {
  return reinterpret_cast<T*>(reinterpret_cast<float*>(a.f[j]) + a.off);
}

template <class T>
__device__ __forceinline__ T fold(const GfkLocalAvg& a, int64_t i) {
  T tot{};
  int j = 0;
  for (int g = 0; g < a.n_groups; ++g) {
    const int e = a.gend[g];
    T s = lptr<const T>(a, j)[i];
    for (++j; j < e; ++j) s = s + lptr<const T>(a, j)[i];
    tot = g == 0 ? s : tot + s;
  }
  return tot;
}
}  // namespace

// FV clients at a time: every client's float4 of a chunk is loaded before the first add (one
// round trip per 8 clients instead of a dependent load per client), then folded in the same
// group order as fold() -- the same bits.  (17 clients on one GPU: the per-client loop was a
// chain of 17 dependent round trips.)
constexpr int FV = 8;
__device__ __forceinline__ float4 fold_regs(const GfkLocalAvg& a, int64_t i) {
  const int n = a.n_clients;
  float4 tot = {0.f, 0.f, 0.f, 0.f}, s = tot;
  int g = 0, gs = 0, e = a.gend[0];
  for (int j0 = 0; j0 < n; j0 += FV) {
    float4 v[FV];
#pragma unroll
    for (int j = 0; j < FV; ++j) v[j] = lptr<const float4>(a, j0 + j < n ? j0 + j : 0)[i];
#pragma unroll
    for (int j = 0; j < FV; ++j) {
      const int jj = j0 + j;
      if (jj >= n) break;
      s = jj == gs ? v[j] : s + v[j];
      if (jj == e - 1) {
        tot = g == 0 ? s : tot + s;
        ++g;
        gs = e;
        if (g < a.n_groups) e = a.gend[g];
      }
    }
  }
  return tot;
}

extern "C" __global__ void __launch_bounds__(256) gfk_local_fedavg(GfkLocalAvg a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = a.n >> 2;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int w1 = a.mode == 1 ? 1 : a.n_clients;     // buffers written
  const int w0 = a.mode == 2 ? 1 : 0;
  for (int64_t i = g; i < n4; i += stride) {
    const float4 acc = a.mode == 2 ? lptr<const float4>(a, 0)[i] : fold_regs(a, i);
    for (int j = w0; j < w1; ++j) lptr<float4>(a, j)[i] = acc;
  }
  if (g < (a.n & 3)) {           // the partial float4 at the end: nothing past n is touched
    const int64_t i = (n4 << 2) + g;
    const float acc = a.mode == 2 ? lptr<const float>(a, 0)[i] : fold<float>(a, i);
    for (int j = w0; j < w1; ++j) lptr<float>(a, j)[i] = acc;
  }
}

extern "C" size_t gfk_local_avg_struct_size() { return sizeof(GfkLocalAvg); }

// the tables' contents (client count, group ends, pointer alignment) are checked by the
// caller when it builds them (parallel/aggregator.py _LocalTable)
extern "C" int gfk_local_fedavg_launch(const GfkLocalAvg* a, int grid, hipStream_t s) {
  if (a->n_clients < 1 || grid < 1 || a->mode < 0 || a->mode > 2 || a->n_groups < 1 ||
      a->n_groups > a->n_clients || !a->f || !a->gend || (a->off & 3) || a->off < 0 || a->n < 0)
    return -1;
  hipLaunchKernelGGL(gfk_local_fedavg, dim3(grid), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Cross-rank state digest (failure detection of the data plane, federation/runner.py).
// After a round's FedAvg every rank must hold the SAME shared state bit for bit (each
// chunk is summed by exactly one rank).  A stale peer line, a lost write-back or a
// broken IPC mapping would instead leave the replicas silently diverged; the ranks
// therefore compare a digest of their shared prefix every few hundred rounds and at
// every aligned round:
//     D = sum over i of mix(i << 32 | bits(x_i))   (mod 2^64, mix = splitmix64's finaliser)
// Position-sensitive, and a sum mod 2^64 is order-independent, so the per-workgroup
// partials and their fold give the same value however the grid is cut -- the numpy
// re-statement in parallel/digest.py computes it bit for bit (CPU ranks, tests).
// Two launches on the stream behind the round (partials, then a one-workgroup fold),
// no atomics; the 8-byte result is copied to pinned host memory asynchronously.
// ---------------------------------------------------------------------------
namespace {
__device__ __forceinline__ uint64_t dg_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t dg_word(int64_t i, uint32_t w) {
  return dg_mix(((uint64_t)i << 32) | w);
}

// block-wide sum of one uint64 per thread (256 threads), result in thread 0
__device__ __forceinline__ uint64_t dg_block_sum(uint64_t v, uint64_t* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  return red[0];
}
}  // namespace

extern "C" __global__ void __launch_bounds__(256)
gfk_digest_part(const uint32_t* __restrict__ w, int64_t n, uint64_t* __restrict__ part) {
  __shared__ uint64_t red[256];
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t n4 = n >> 2;
  uint64_t acc = 0;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < n4; q += stride) {
    const uint4 v = reinterpret_cast<const uint4*>(w)[q];
    const int64_t i = q << 2;
    acc += dg_word(i, v.x) + dg_word(i + 1, v.y) + dg_word(i + 2, v.z) + dg_word(i + 3, v.w);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    acc += dg_word(i, w[i]);
  }
  const uint64_t s = dg_block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

extern "C" __global__ void __launch_bounds__(256)
gfk_digest_fold(const uint64_t* __restrict__ part, int nblk, uint64_t* __restrict__ out) {
  __shared__ uint64_t red[256];
  uint64_t acc = 0;
  for (int b = threadIdx.x; b < nblk; b += 256) acc += part[b];
  const uint64_t s = dg_block_sum(acc, red);
  if (threadIdx.x == 0) out[0] = s;
}

// digest of n words at w (16-byte aligned) into out[0]; part: nblk uint64 of scratch;
// host (pinned, optional): the result copied there behind the two kernels
extern "C" int gfk_digest_launch(const void* w, int64_t n, void* part, int nblk, void* out,
                                 void* host, hipStream_t s) {
  if (!w || !part || !out || n < 0 || nblk < 1 || ((uintptr_t)w & 15)) return -1;
  hipLaunchKernelGGL(gfk_digest_part, dim3(nblk), dim3(256), 0, s,
                     static_cast<const uint32_t*>(w), n, static_cast<uint64_t*>(part));
  hipLaunchKernelGGL(gfk_digest_fold, dim3(1), dim3(256), 0, s,
                     static_cast<const uint64_t*>(part), nblk, static_cast<uint64_t*>(out));
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && host)
    e = hipMemcpyAsync(host, out, sizeof(uint64_t), hipMemcpyDeviceToHost, s);
  return (int)e;
}

// ---------------------------------------------------------------------------
// host API (ctypes)
// ---------------------------------------------------------------------------
extern "C" size_t gfk_comm_struct_size() { return sizeof(GfkComm); }

// The kernel addresses the stage (or, in place, the data) through buffer descriptors with
// 32-bit byte offsets: a state must stay below this many bytes (XgmiAllReduce refuses
// larger ones, and the caller keeps RCCL for them).
extern "C" int64_t gfk_comm_max_bytes() { return ((int64_t)1 << 31) - 64; }

// stage: 2 * stage_bytes (regular); flags: uncached, zeroed; state: epoch[nblk] + err, zeroed.
// *uncached = 1 if the flag array got uncached memory, 0 if it fell back to hipMalloc (the
// flags' L2 write-backs in publish() then carry the protocol alone; recorded by the caller).
extern "C" int gfk_comm_alloc(int64_t stage_bytes, int64_t flag_bytes, int64_t state_bytes,
                              void** stage, void** flags, void** state, int* uncached) {
  hipError_t e;
  if ((e = hipMalloc(stage, 2 * stage_bytes))) return (int)e;
  if ((e = hipMemset(*stage, 0, 2 * stage_bytes))) return (int)e;
  *uncached = 1;
  if (hipExtMallocWithFlags(flags, flag_bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    *uncached = 0;
    if ((e = hipMalloc(flags, flag_bytes))) return (int)e;
  }
  if ((e = hipMemset(*flags, 0, flag_bytes))) return (int)e;
  if ((e = hipMalloc(state, state_bytes))) return (int)e;
  if ((e = hipMemset(*state, 0, state_bytes))) return (int)e;
  return (int)hipDeviceSynchronize();
}

extern "C" int gfk_comm_free(void* stage, void* flags, void* state) {
  const hipError_t e0 = hipFree(stage), e1 = hipFree(flags), e2 = hipFree(state);
  return (int)(e0 ? e0 : e1 ? e1 : e2);
}

extern "C" int gfk_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

extern "C" int gfk_ipc_get(void* ptr, void* handle) {
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), ptr);
}

extern "C" int gfk_ipc_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int gfk_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// The IPC handle of the allocation holding ptr (a caching-allocator sub-block) and
// ptr's byte offset into it: peers open the handle and add the offset.
extern "C" int gfk_ipc_get_range(void* ptr, void* handle, int64_t* offset) {
  void* base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, ptr);
  if (e != hipSuccess) return (int)e;
  *offset = (int64_t)((char*)ptr - (char*)base);
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), base);
}

// The error word (0 = fine; 1 / 2 / 3 = a phase-0 / phase-1 / in-place phase-3 wait timed
// out: 1 + the phase's flag row); synchronous.
extern "C" int gfk_comm_error(const GfkComm* c) {
  int32_t v = 0;
  if (hipMemcpy(&v, c->err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return v;
}

// Diagnostics: this rank's per-workgroup epochs [nblk] and its own flag array
// [phases][nblk][CMAX] (what the peers published to it), copied to host; synchronous.
extern "C" int gfk_comm_dump(const GfkComm* c, uint32_t* epoch, uint32_t* flags, int phases) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(epoch, c->epoch, sizeof(uint32_t) * c->nblk, hipMemcpyDeviceToHost) != hipSuccess) return -2;
  const size_t fb = sizeof(uint32_t) * (size_t)phases * c->nblk * CMAX;
  if (hipMemcpy(flags, c->flags[c->rank], fb, hipMemcpyDeviceToHost) != hipSuccess) return -3;
  return 0;
}

// The error word copied to (pinned) host memory behind the stream's work: the runner polls
// it between rounds without synchronising the device.
extern "C" int gfk_comm_error_async(const GfkComm* c, int32_t* host, hipStream_t s) {
  return (int)hipMemcpyAsync(host, c->err, sizeof(int32_t), hipMemcpyDeviceToHost, s);
}

extern "C" int gfk_comm_launch(const GfkComm* c, float* data, hipStream_t s) {
  if (c->world < 1 || c->world > CMAX || c->nblk < 1 || (c->chunk & 3) || (c->slice & 3) ||
      (int64_t)c->slice * c->nblk < c->chunk || (int64_t)c->chunk * c->world < c->n ||
      ((uintptr_t)data & 15) || (int64_t)c->world * c->chunk * 4 > gfk_comm_max_bytes())
    return -1;
  if (c->wire == 1) {
    if (c->inplace || !c->ref || ((uintptr_t)c->ref & 15)) return -1;
    hipLaunchKernelGGL(gfk_xgmi_allreduce_bf16d, dim3(c->nblk), dim3(CT), 0, s, *c, data);
  } else {
    hipLaunchKernelGGL(gfk_xgmi_allreduce, dim3(c->nblk), dim3(CT), 0, s, *c, data);
  }
  return (int)hipGetLastError();
}
