// Peer-to-peer gradient all-reduce over xGMI (gfx950): one-shot and two-shot.
//
// on an 8x MI355X node every GPU has a direct xGMI link to
// every other GPU. A ring all-reduce (RCCL's default for a bucket) crosses ONE
// link per step and pays 2(s-1) latency hops. Both forms here use all s-1
// links of a group at once:
//
// one-shot (latency-bound buckets, 1-4 MB): one hop.
//   1. push: every rank writes its whole bucket straight into each peer's
//      receive slab (remote stores over xGMI through hipIpc mappings);
//   2. signal: release fence, then one flag per (source rank, block) in each
//      peer's flag array;
//   3. wait: poll the local flags of every peer (acquire), bounded in time;
//   4. reduce: sum the s contributions IN RANK ORDER (bitwise identical result
//      on every replica), scale by 1/s, write back into the gradient arena.
//   Each link carries the whole bucket.
// two-shot (bandwidth-bound buckets, s >= 3): two hops, each link carries
// 2/s of the bucket instead of all of it.
//   1. reduce-scatter: the bucket is cut into s chunks, chunk q owned by rank
//      q; every rank pushes chunk q to rank q only; the owner sums its chunk in
//      rank order (the same order and scale as one-shot: bitwise the same
//      values) and writes it back;
//   2. all-gather: the owner pushes its reduced chunk to every peer's gather
//      slab; each rank copies the s-1 foreign chunks into its arena.
// No grid-wide synchronisation: block g of rank r only waits for block g of
// its peers, so the kernel runs with any number of co-resident blocks and
// overlaps with backward kernels on other streams. Per-block epoch counters
// live in device memory, so the launch is hipGraph-capturable; the receive
// slabs are double-buffered by epoch parity (a peer can run at most one epoch
// ahead: its next push into the same parity needs this rank's next flag).
// Receive slabs and flags are uncached (hipDeviceMallocUncached) so polled
// flags and freshly pushed data never come from a stale cache line.
// A wait that exceeds `timeout_ticks` records the bucket in `status` and the
// block exits: a lost peer never hangs the GPU. Once `status` is set (or the
// host raised the abort word) later waits give up at their first unsuccessful
// poll, so the launches queued behind a failure drain at once.
#include "common.h"
#include "p2p_allreduce.h"

namespace mdt {

__device__ __forceinline__ long long p2p_stride(long long n) { return (n + 63) / 64 * 64; }

// dst[i] = src[i] for i in [0, n) into every peer p != me (dst_p = peer base + off)
__device__ __forceinline__ void p2p_push(const P2PArgs& a, const float* src, long long off, long long n) {
  const bool vec = ((((uintptr_t)src) & 15) == 0);
  const long long nv = vec ? n / 4 * 4 : 0;
  for (long long i = 4 * (long long)threadIdx.x; i < nv; i += 4 * (long long)blockDim.x) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(src + i);
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < a.s && p != a.me) *reinterpret_cast<f32x4*>(a.peer_recv[p] + off + i) = v;
  }
  for (long long i = nv + threadIdx.x; i < n; i += blockDim.x) {
    const float v = src[i];
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < a.s && p != a.me) a.peer_recv[p][off + i] = v;
  }
}

// every wave's remote stores complete and visible system-wide, then flag (phase, me, g) = e in every peer
__device__ __forceinline__ void p2p_signal(const P2PArgs& a, int phase, unsigned e) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  const int G = gridDim.x;
  if (threadIdx.x < a.s && (int)threadIdx.x != a.me) {
    unsigned* f = a.peer_flags[threadIdx.x] + a.flag_off + ((long long)phase * a.s + a.me) * G + blockIdx.x;
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// wait for flag (phase, p, g) >= e of every peer p (lane p polls peer p's flag in local memory);
// false after a timeout (the bucket is recorded in status)
__device__ __forceinline__ bool p2p_wait(const P2PArgs& a, int phase, unsigned e, int* s_ok) {
  const int G = gridDim.x;
  if (threadIdx.x < 64) {
    const int p = threadIdx.x;
    const bool mine = p < a.s && p != a.me;
    const unsigned* f = a.my_flags + a.flag_off + ((long long)phase * a.s + p) * G + blockIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int fail = 0;  // 1: timed out, 2: abandoned (earlier failure or host abort)
    for (unsigned it = 0;; ++it) {
      const bool ready = !mine || (int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) >= 0;
      if (__all(ready)) break;
      if ((it & 63u) == 0 && p2p_wait_abandoned(a.status, a.abort_flag, p)) {
        fail = 2;
        break;
      }
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (fail && p == 0) {
      atomicCAS(a.status, 0, fail == 1 ? 1 + a.bucket : kCommAborted);
      *s_ok = 0;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return *s_ok != 0;
}

// out[i] = scale * sum_p src[p][i] (rank order), i in [0, n)
__device__ __forceinline__ void p2p_reduce(const P2PArgs& a, const float* const* src, float* out, long long n,
                                           bool vec) {
  const long long nv = vec ? n / 4 * 4 : 0;
  for (long long i = 4 * (long long)threadIdx.x; i < nv; i += 4 * (long long)blockDim.x) {
    f32x4 acc = *reinterpret_cast<const f32x4*>(src[0] + i);
#pragma unroll
    for (int p = 1; p < kP2PMaxRanks; ++p)
      if (p < a.s) acc += *reinterpret_cast<const f32x4*>(src[p] + i);
    *reinterpret_cast<f32x4*>(out + i) = acc * a.scale;
  }
  for (long long i = nv + threadIdx.x; i < n; i += blockDim.x) {
    float acc = src[0][i];
#pragma unroll
    for (int p = 1; p < kP2PMaxRanks; ++p)
      if (p < a.s) acc += src[p][i];
    out[i] = acc * a.scale;
  }
}

__global__ void __launch_bounds__(256) p2p_allreduce_k(P2PArgs a) {
  __shared__ unsigned s_ep;
  __shared__ int s_ok;
  const int g = blockIdx.x, G = gridDim.x;
  if (threadIdx.x == 0) {
    s_ep = a.ep[g] + 1u;
    s_ok = 1;
  }
  __syncthreads();
  const unsigned e = s_ep;
  const int par = (int)(e & 1u);
  const bool vec = ((((uintptr_t)a.data) & 15) == 0);
  const float* src[kP2PMaxRanks];

  if (!a.two_shot) {
    const long long per = ((a.n + G - 1) / G + 3) / 4 * 4;
    const long long lo = (long long)g * per;
    const long long hi = lo + per < a.n ? lo + per : a.n;
    const long long len = hi > lo ? hi - lo : 0;
    const long long stride = p2p_stride(a.n);
    // 1-2. push this block's range into every peer's slab [par][me], signal
    p2p_push(a, a.data + lo, a.recv_off + ((long long)par * a.s + a.me) * stride + lo, len);
    p2p_signal(a, 0, e);
    // 3. wait for block g of every peer
    if (!p2p_wait(a, 0, e, &s_ok)) return;  // epoch not advanced: the host reports the timeout via status()
    // 4. reduce in rank order: identical bits on every replica
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      src[p] = ((p == a.me) ? a.data : a.my_recv + a.recv_off + ((long long)par * a.s + p) * stride) + lo;
    p2p_reduce(a, src, a.data + lo, len, vec);
  } else {
    // chunk q = [q*cs, min(n, (q+1)*cs)) is owned by rank q; block g covers [g*per, (g+1)*per) of every chunk
    const long long cs = ((a.n + a.s - 1) / a.s + 3) / 4 * 4;
    const long long per = ((cs + G - 1) / G + 3) / 4 * 4;
    const long long cstride = p2p_stride(cs);
    const long long lo = (long long)g * per;
    auto clen = [&](int q) -> long long {  // elements of chunk q in this block's range
      long long b = (long long)q * cs + lo, t = (long long)q * cs + (lo + per < cs ? lo + per : cs);
      if (t > a.n) t = a.n;
      return t > b ? t - b : 0;
    };
    const long long rs_off = a.recv_off;                               // [2][s][cstride]
    const long long ag_off = a.recv_off + 2LL * a.s * cstride;         // [2][s][cstride]
    // 1. reduce-scatter: chunk q of this rank goes to rank q's RS slab [par][me]
    {
      const long long dst = rs_off + ((long long)par * a.s + a.me) * cstride + lo;
      for (int q = 0; q < a.s; ++q) {
        if (q == a.me) continue;
        const long long n = clen(q);
        const float* sp = a.data + (long long)q * cs + lo;
        const bool v = ((((uintptr_t)sp) & 15) == 0);
        const long long nv = v ? n / 4 * 4 : 0;
        float* dp = a.peer_recv[q] + dst;
        for (long long i = 4 * (long long)threadIdx.x; i < nv; i += 4 * (long long)blockDim.x)
          *reinterpret_cast<f32x4*>(dp + i) = *reinterpret_cast<const f32x4*>(sp + i);
        for (long long i = nv + threadIdx.x; i < n; i += blockDim.x) dp[i] = sp[i];
      }
    }
    p2p_signal(a, 0, e);
    if (!p2p_wait(a, 0, e, &s_ok)) return;
    const long long mine = clen(a.me);
    float* out = a.data + (long long)a.me * cs + lo;
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      src[p] = (p == a.me) ? out : a.my_recv + rs_off + ((long long)par * a.s + p) * cstride + lo;
    p2p_reduce(a, src, out, mine, vec);
    __syncthreads();  // the block's reduced range is complete before it is pushed
    // 2. all-gather: the reduced range goes to every peer's AG slab [par][me]
    p2p_push(a, out, ag_off + ((long long)par * a.s + a.me) * cstride + lo, mine);
    p2p_signal(a, 1, e);
    if (!p2p_wait(a, 1, e, &s_ok)) return;
    for (int q = 0; q < a.s; ++q) {
      if (q == a.me) continue;
      const long long n = clen(q);
      const float* sp = a.my_recv + ag_off + ((long long)par * a.s + q) * cstride + lo;
      float* dp = a.data + (long long)q * cs + lo;
      const bool v = ((((uintptr_t)dp) & 15) == 0);
      const long long nv = v ? n / 4 * 4 : 0;
      for (long long i = 4 * (long long)threadIdx.x; i < nv; i += 4 * (long long)blockDim.x)
        *reinterpret_cast<f32x4*>(dp + i) = *reinterpret_cast<const f32x4*>(sp + i);
      for (long long i = nv + threadIdx.x; i < n; i += blockDim.x) dp[i] = sp[i];
    }
  }
  if (threadIdx.x == 0) a.ep[g] = e;
}

// Construction-time data-plane self-test (parallel/ddp.py::selftest_fused):
// the rank-coded pattern and the bitwise check of the reduced result, as
// kernels of this extension (no framework elementwise kernels, whose first
// use in a fresh process costs milliseconds of module loading each).
// pattern(q, i) = ((i * 40503 + q * 9973 + 7) mod 4093 - 2046) * 2^-6: any
// sum of <= 8 of them is exact in f32, so the expected value is the plain sum
// times the reducer's scale, bitwise, in any order.
__device__ __forceinline__ float selftest_pattern(long long i, int q) {
  return (float)((int)((i * 40503LL + (long long)q * 9973LL + 7LL) % 4093LL) - 2046) * 0.015625f;
}

__global__ void __launch_bounds__(256) selftest_fill_k(float* g, long long n, int q) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    g[i] = selftest_pattern(i, q);
}

__global__ void __launch_bounds__(256) selftest_check_k(const float* g, long long n, int s, float scale, int* bad) {
  int miss = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float acc = selftest_pattern(i, 0);
    for (int q = 1; q < s; ++q) acc += selftest_pattern(i, q);
    acc *= scale;
    miss += __float_as_uint(acc) != __float_as_uint(g[i]);
  }
  if (miss) atomicAdd(bad, miss);
}

}  // namespace mdt

extern "C" int mdt_selftest_fill(float* g, long long n, int q, hipStream_t stream) {
  if (n < 1) return 1;
  const long long b = (n + 255) / 256;
  hipLaunchKernelGGL(mdt::selftest_fill_k, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, stream, g, n, q);
  return (int)hipGetLastError();
}

extern "C" int mdt_selftest_check(const float* g, long long n, int s, float scale, int* bad, hipStream_t stream) {
  if (n < 1 || s < 1) return 1;
  const long long b = (n + 255) / 256;
  hipLaunchKernelGGL(mdt::selftest_check_k, dim3((unsigned)(b < 4096 ? b : 4096)), dim3(256), 0, stream, g, n, s, scale,
                     bad);
  return (int)hipGetLastError();
}

extern "C" int mdt_p2p_allreduce(const mdt::P2PArgs* a, int grid, hipStream_t stream) {
  if (grid < 1 || a->s < 1 || a->s > mdt::kP2PMaxRanks || a->me < 0 || a->me >= a->s || a->n < 1) return 1;
  hipLaunchKernelGGL(mdt::p2p_allreduce_k, dim3(grid), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}
