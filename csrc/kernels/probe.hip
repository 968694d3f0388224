// Hardware probes used by the profiling tools (multidisttorch_amd/obs/probe.py):
// shader clock under load, dependent-load latency, empty-kernel cost.
#include "common.h"

namespace mdt {

// One wave: shader-clock cycles (s_memtime) vs 100 MHz wall ticks (s_memrealtime)
// around `iters` dependent FMAs -> effective SCLK in MHz.
__global__ void probe_clock(unsigned long long* out, int iters) {
  float x = (float)threadIdx.x;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) x = fmaf(x, 1.0000001f, 0.5f);
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = r1 - r0;
    out[2] = (unsigned long long)(x > 1e30f);  // keep x live
  }
}

// One lane: pointer chase over `idx` (n hops) -> cycles per dependent load.
__global__ void probe_latency(const int* idx, int hops, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  int j = 0;
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < hops; ++i) j = idx[j];
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  out[0] = c1 - c0;
  out[1] = (unsigned long long)j;
}

__global__ void probe_empty() {}

// Fill every CU's LDS (the whole 160 KB, one 1024-thread workgroup per CU at
// a time) with a pattern: an uninitialised-LDS read in a later kernel then
// shows up as a changed result (tests: the fused step under a poisoned LDS).
__global__ void __launch_bounds__(1024) probe_lds_poison(unsigned pattern) {
  extern __shared__ unsigned lds_all[];
  for (int i = threadIdx.x; i < 160 * 1024 / 4; i += blockDim.x) lds_all[i] = pattern;
  __syncthreads();
}

// Where each workgroup ran: (XCC id << 16) | HW_ID bits (CU, SH, SE) of wave 0.
// Rehearsal check of HSA_CU_MASK (runtime/env.py::apply_cu_split).
__global__ void probe_cu_ids(unsigned* out) {
  if (threadIdx.x != 0) return;
  unsigned hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  // HW_ID: cu_id [11:8], sh_id [12], se_id [15:13]
  out[blockIdx.x] = (xcc << 16) | (hw & 0xff00u);
  // keep the workgroup resident long enough that the grid spreads over every allowed CU
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000ull) __builtin_amdgcn_s_sleep(8);
}

}  // namespace mdt

extern "C" int mdt_probe_cu_ids(unsigned* out, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(mdt::probe_cu_ids, dim3(blocks), dim3(64), 0, s, out);
  return (int)hipGetLastError();
}

extern "C" int mdt_probe_clock(unsigned long long* out, int iters, hipStream_t s) {
  hipLaunchKernelGGL(mdt::probe_clock, dim3(1), dim3(64), 0, s, out, iters);
  return (int)hipGetLastError();
}

extern "C" int mdt_probe_latency(const int* idx, int hops, unsigned long long* out, hipStream_t s) {
  hipLaunchKernelGGL(mdt::probe_latency, dim3(1), dim3(64), 0, s, idx, hops, out);
  return (int)hipGetLastError();
}

extern "C" int mdt_probe_empty(int blocks, int threads, hipStream_t s) {
  hipLaunchKernelGGL(mdt::probe_empty, dim3(blocks), dim3(threads), 0, s);
  return (int)hipGetLastError();
}

extern "C" int mdt_probe_lds_poison(unsigned pattern, int blocks, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&mdt::probe_lds_poison),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return (int)attr;
  hipLaunchKernelGGL(mdt::probe_lds_poison, dim3(blocks), dim3(1024), 160 * 1024, s, pattern);
  return (int)hipGetLastError();
}
