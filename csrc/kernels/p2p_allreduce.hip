// One-shot peer-to-peer gradient all-reduce over xGMI for small buckets (gfx950).
//
// on an 8x MI355X node every GPU has a direct xGMI link to
// every other GPU. A ring all-reduce (RCCL's default for a bucket) crosses ONE
// link per step and pays 2(s-1) latency hops; for the latency-bound buckets of
// the VAE models (1-4 MB) a one-shot exchange uses all s-1 links of a group at
// once and pays one hop:
//   1. push: every rank writes its bucket chunk straight into each peer's
//      receive slab (remote stores over xGMI through hipIpc mappings);
//   2. signal: release fence, then one flag per (source rank, block) in each
//      peer's flag array;
//   3. wait: poll the local flags of every peer (acquire), bounded in time;
//   4. reduce: sum the s contributions IN RANK ORDER (bitwise identical result
//      on every replica), scale by 1/s, write back into the gradient arena.
// No grid-wide synchronisation: block g of rank r only waits for block g of
// its peers, so the kernel runs with any number of co-resident blocks and
// overlaps with backward kernels on other streams. Per-block epoch counters
// live in device memory, so the launch is hipGraph-capturable; the receive
// slab is double-buffered by epoch parity (a peer can run at most one epoch
// ahead: its next push into the same parity needs this rank's next flag).
// Receive slabs and flags are uncached (hipDeviceMallocUncached) so polled
// flags and freshly pushed data never come from a stale cache line.
// A wait that exceeds `timeout_ticks` records the bucket in `status` and the
// block exits: a lost peer never hangs the GPU.
#include "common.h"
#include "p2p_allreduce.h"

namespace mdt {

__device__ __forceinline__ long long p2p_stride(long long n) { return (n + 63) / 64 * 64; }

__global__ void __launch_bounds__(256) p2p_allreduce_k(P2PArgs a) {
  __shared__ unsigned s_ep;
  __shared__ int s_ok;
  const int g = blockIdx.x, G = gridDim.x;
  const long long per = ((a.n + G - 1) / G + 3) / 4 * 4;
  const long long lo = (long long)g * per;
  const long long hi = lo + per < a.n ? lo + per : a.n;
  if (threadIdx.x == 0) {
    s_ep = a.ep[g] + 1u;
    s_ok = 1;
  }
  __syncthreads();
  const unsigned e = s_ep;
  const int par = (int)(e & 1u);
  const long long stride = p2p_stride(a.n);
  const bool vec = ((((uintptr_t)a.data) & 15) == 0);
  const long long vhi = vec ? lo + (hi > lo ? (hi - lo) / 4 * 4 : 0) : lo;

  // 1. push this rank's chunk into every peer's slab [par][me]
  const long long dst_off = a.recv_off + ((long long)par * a.s + a.me) * stride;
  for (long long i = lo + 4 * (long long)threadIdx.x; i < vhi; i += 4 * (long long)blockDim.x) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(a.data + i);
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < a.s && p != a.me) *reinterpret_cast<f32x4*>(a.peer_recv[p] + dst_off + i) = v;
  }
  for (long long i = vhi + threadIdx.x; i < hi; i += blockDim.x) {
    const float v = a.data[i];
#pragma unroll
    for (int p = 0; p < kP2PMaxRanks; ++p)
      if (p < a.s && p != a.me) a.peer_recv[p][dst_off + i] = v;
  }
  // 2. signal: every wave's remote stores complete and visible system-wide, then one flag per peer
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if (threadIdx.x < a.s && (int)threadIdx.x != a.me) {
    unsigned* f = a.peer_flags[threadIdx.x] + a.flag_off + (long long)a.me * G + g;
    __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. wait for block g of every peer (lane p polls peer p's flag in local memory)
  if (threadIdx.x < 64) {
    const int p = threadIdx.x;
    bool mine = p < a.s && p != a.me;
    const unsigned* f = a.my_flags + a.flag_off + (long long)p * G + g;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool timed_out = false;
    while (true) {
      const bool ready = !mine || (int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) >= 0;
      if (__all(ready)) break;
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        timed_out = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (timed_out && p == 0) {
      atomicCAS(a.status, 0, 1 + a.bucket);
      s_ok = 0;
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  if (!s_ok) return;  // epoch not advanced: the host reports the timeout via status()

  // 4. reduce in rank order: identical bits on every replica
  const float* src[kP2PMaxRanks];
#pragma unroll
  for (int p = 0; p < kP2PMaxRanks; ++p)
    src[p] = (p == a.me) ? a.data : a.my_recv + a.recv_off + ((long long)par * a.s + p) * stride;
  for (long long i = lo + 4 * (long long)threadIdx.x; i < vhi; i += 4 * (long long)blockDim.x) {
    f32x4 acc = *reinterpret_cast<const f32x4*>(src[0] + i);
#pragma unroll
    for (int p = 1; p < kP2PMaxRanks; ++p)
      if (p < a.s) acc += *reinterpret_cast<const f32x4*>(src[p] + i);
    *reinterpret_cast<f32x4*>(a.data + i) = acc * a.scale;
  }
  for (long long i = vhi + threadIdx.x; i < hi; i += blockDim.x) {
    float acc = src[0][i];
#pragma unroll
    for (int p = 1; p < kP2PMaxRanks; ++p)
      if (p < a.s) acc += src[p][i];
    a.data[i] = acc * a.scale;
  }
  if (threadIdx.x == 0) a.ep[g] = e;
}

}  // namespace mdt

extern "C" int mdt_p2p_allreduce(const mdt::P2PArgs* a, int grid, hipStream_t stream) {
  if (grid < 1 || a->s < 1 || a->s > mdt::kP2PMaxRanks || a->me < 0 || a->me >= a->s || a->n < 1) return 1;
  hipLaunchKernelGGL(mdt::p2p_allreduce_k, dim3(grid), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}
