// Shared device helpers for the MI355X (gfx950, CDNA4) kernels.
//
// Everything here is written for wave64 + MFMA; no CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mdt {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Exact-f32 MFMA: lane l holds A[l&15][l>>4] and B[l>>4][l&15];
// C/D: col = l&15, row = 4*(l>>4) + reg.
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Exact-f32 MFMA 32x32x2: lane l holds A[l&31][l>>5] and B[l>>5][l&31];
// C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*(l>>5), reg in [0,16).
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum (blockDim.x multiple of 64, <= 1024). `scratch` >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x < 64) {
    t = (threadIdx.x < nw) ? scratch[threadIdx.x] : 0.f;
    t = wave_sum(t);
  }
  return t;  // valid in wave 0
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG (Salmon et al., SC'11). Stateless: the
// reparameterisation noise for (seed, step, element) is a pure function, so
// graph replays, resumes and the CPU reference produce identical eps.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// Standard normal from two uint32 (Box-Muller, first output).
__device__ __forceinline__ float normal_from_bits(uint32_t a, uint32_t b) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
  const float u2 = (float)b * 2.3283064365386963e-10f;           // [0, 1)
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// Write-through stores for a kernel's large outputs that the NEXT launch
// reads. Plain stores leave their lines dirty in the XCD's L2 until the
// end-of-kernel release writes them back -- a tail of ~bytes / 6 TB/s after
// the last wave (~2 us behind a 17 MB bf16 activation, profiles/r5_wt_stores)
// that nothing overlaps. An agent-scope relaxed atomic store lowers to
// `global_store ... sc1`: the bytes go out while the rest of the grid still
// computes. Used where measured faster (the direct convs' bf16 outputs); the
// thin convs' outputs and f32 outputs measured no better (the consumer then
// reads from the Infinity Cache instead of L2).
__device__ __forceinline__ void st_wt8(void* p, unsigned long long v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Slow path of the xGMI all-reduce waits (p2p_allreduce.hip, comm_jobs.h),
// called by every lane of the polling wave after an unsuccessful poll: true
// (wave-uniform) when a wait already failed (`status` != 0, this or an earlier
// step) or the host raised the abort word (host-mapped, may be null). The
// caller records the abort in `status` (so later waits stop at the cheaper
// device-memory read); here lane 0 only reads, at system scope (the words are
// written by other workgroups / the host).
__device__ __forceinline__ bool p2p_wait_abandoned(const int* status, const int* abort_flag, int lane) {
  int bad = 0;
  if (lane == 0) {
    bad = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    if (!bad && abort_flag) bad = __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  }
  return __any(bad);
}

}  // namespace mdt
