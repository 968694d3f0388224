// Horizontally fused conv-VAE launches ("job kernels") for MI355X (gfx950).
//
// Why: at the conv-VAE's batch sizes most launches of a training step are
// latency-bound -- a 28x28 step was 29 launches of which a dozen do < 2 us
// of work, and a kernel boundary in a replayed hipGraph costs ~1.5 us plus
// the fill/drain of the grid. Independent pieces of work of the same step
// (the weight gradient and the backward-data GEMM of one layer, a bias column
// sum, the loss reduction) therefore share ONE launch: each job owns a
// contiguous range of workgroups and runs the same device body as its
// stand-alone kernel (conv_igemm_dev.h, conv_thin.h, conv_small.h), so results
// are bitwise identical to the unfused sequence. Two streams with graph
// branches were measured slower on this stack (cross-stream graph edges,
// models/conv_vae.py::_backward_overlap), which is why the fusion is done
// inside a launch instead.
//
// A launch of jobs (kinds k0 < k1 < k2 after sorting) needs an instantiated
// jobs_k<J0, J1, J2>; the table below lists the combinations the 28x28 and
// 128x128 models' backward sweeps use. Any other combination reports "not
// fused" and the caller launches the jobs' stand-alone kernels instead.
#include <string.h>

#include <algorithm>

#include "conv_direct.h"
#include "conv_dwgrad.h"
#include "conv_igemm_dev.h"
#include "comm_jobs.h"
#include "conv_small.h"
#include "conv_thin.h"
#include "conv_thin_wg.h"

namespace mdt {
using namespace tiles;

struct JobPack {
  JobBlob j[3];
  int start1, start2;  // first workgroup of job 1 / job 2
};

template <class T>
__device__ __forceinline__ const T& job_args(const JobBlob& j) {
  return *reinterpret_cast<const T*>(j.args);
}

struct JNone {
  static constexpr int ID = 0, LDS = 0;
  static __device__ __forceinline__ void run(const JobBlob&, uint8_t*, int) {}
};

// forward-type GEMM (bf16, vector gathers); aux = {tiles per plane, k-splits}
template <int MODE, int CFG, class TC>
struct JIg {
  static constexpr int ID = kJobIgemm + MODE * 100 + CFG, LDS = igemm_lds_bytes<TC>();
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    const int ntb = j.aux[0], ks = j.aux[1];
    const int r = b / ntb, t = b - r * ntb;
    const int cls = r / ks, kz = r - cls * ks;
    igemm_body<MODE, __bf16, true, TC>(job_args<IgArgs>(j), lds, t, ntb, kz, cls);
  }
};

template <int CFG, class TC>
struct JWg {
  static constexpr int ID = kJobWgrad + CFG, LDS = wgrad_lds_bytes<TC>();
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    wgrad_body<__bf16, true, TC>(job_args<WgArgs>(j), lds, b, j.nblk);
  }
};

template <typename XT, int CFG, class TC>
struct JWgThin {
  static constexpr int ID = kJobWgradThin + (sizeof(XT) == 4 ? 20 : 0) + CFG, LDS = wgrad_lds_bytes<TC>();
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    wgrad_body<XT, false, TC>(job_args<WgArgs>(j), lds, b, j.nblk);
  }
};

template <typename XT>
struct JThinWg {
  static constexpr int ID = kJobThinWgM + (sizeof(XT) == 4 ? 1 : 0), LDS = thin_wgrad_mfma_lds_bytes();
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    thin_wgrad_mfma_body<XT>(job_args<WgArgs>(j), lds, b);
  }
};

template <int CO, typename TIN>
struct JThinConv {
  static constexpr int ID = kJobThinConv + CO + (sizeof(TIN) == 4 ? 100 : 0), LDS = thin_conv_lds_bytes<CO, 4>();
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    thin_conv_body<CO, 4, TIN>(job_args<ThinConvArgs>(j), lds, b);
  }
};

// patch-resident direct conv (the backward-data of the 64x64 / 32x32 layers):
// shares a launch with the layer's weight gradient
template <int CFG, class CF>
struct JDc {
  static constexpr int ID = kJobDconv + CFG, LDS = CF::LDS;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    dconv_body<CF>(job_args<DcArgs>(j), lds, xcd_remap(b, j.nblk));
  }
};

struct JColsum {
  static constexpr int ID = kJobColsum, LDS = 0;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t*, int b) { colsum_body(job_args<ColsumArgs>(j), b); }
};

struct JLoss {
  static constexpr int ID = kJobLoss, LDS = 64;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int) {
    loss_finalize_body(job_args<LossArgs>(j), reinterpret_cast<float*>(lds));
  }
};

struct JFinalize {
  static constexpr int ID = kJobFinalize, LDS = kFinalizeThreads * 4 + 64;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    grad_finalize_body(job_args<FinalizeArgs>(j), reinterpret_cast<float*>(lds),
                       reinterpret_cast<AdamC*>(lds + kFinalizeThreads * 4), b);
  }
};

struct JWtrans {
  static constexpr int ID = kJobWtrans, LDS = kWtransLds;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    wtrans_body(job_args<WtransArgs>(j), lds, b);
  }
};

// gradient all-reduce push / reduce+Adam over finalize units (comm_jobs.h)
struct JComm {
  static constexpr int ID = kJobComm, LDS = kCommLds;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int b) {
    comm_unit_body(job_args<CommJobArgs>(j), lds, b);
  }
};

// next-batch gather of the fused 28x28 step after the loss job of the same
// launch (conv_small.h batch_gather_dep_body)
struct JGather {
  static constexpr int ID = kJobGather, LDS = 0;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t*, int b) {
    batch_gather_dep_body(job_args<BatchGather>(j), b);
  }
};

struct JLossStep {
  static constexpr int ID = kJobLossStep, LDS = 64;
  static __device__ __forceinline__ void run(const JobBlob& j, uint8_t* lds, int) {
    loss_step_body(job_args<LossArgs>(j), reinterpret_cast<float*>(lds));
  }
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

// ------------------------------------------------------------ multi-job ----
// Up to 8 independent jobs (kMaxMultiJobs = 16 with dependencies, below) of
// any supported kind in ONE launch, dispatched per workgroup by a runtime switch (the fused 28x28 step's six
// weight gradients + its loss/step job). Unlike jobs_k it needs no
// instantiation per combination; its register allocation is the maximum over
// the bodies, which is what those bodies use anyway.
//
// Dependencies between the jobs of ONE launch (jobs_multi_k<true>). A job whose
// `wait` mask is set runs each of its workgroups only after every workgroup
// of the masked jobs has finished; those count themselves done:
//   producer: every wave `s_waitcnt vmcnt(0)` -> workgroup barrier -> one lane
//     (signal 2 only: agent release, for plain stores) -> relaxed agent add
//     to its job's counter (signal 1: the job's handed-off bytes all leave
//     through sc1 stores, nothing dirty in this XCD's L2 to write back);
//   consumer: one lane polls the counters with relaxed agent (sc1) loads and
//     s_sleep -> workgroup barrier -> EVERY load of handed-off bytes is an sc1
//     vector load (FinalizeArgs.dep, batch_gather_dep_body): no L1 line and no
//     scalar-cache line can serve an old copy.
// Deadlock-free by construction of the tables: waiting jobs come after their
// producers in the grid and producers never wait, so a spinning workgroup
// only ever waits for workgroups dispatched before it. A poll that sees no
// progress for kDepTimeoutTicks records the job in ctr[err] and goes on (the
// host checks that word: dep_error); the last waiting workgroup to pass its
// wait re-zeroes the counters for the next launch.
#ifndef MDT_DEP_SLEEP
#define MDT_DEP_SLEEP 2
#endif
constexpr int kDepStride = 32;  // words between counters (one 128-B line each)
constexpr int kDepDone = kMaxMultiJobs, kDepErr = kMaxMultiJobs + 1, kDepWords = (kMaxMultiJobs + 2) * kDepStride;
constexpr unsigned long long kDepTimeoutTicks = 5000000ull;  // 50 ms of the 100 MHz s_memrealtime

struct JobPackN {
  JobBlob j[kMaxMultiJobs];
  int start[kMaxMultiJobs + 1];
  int n;
  unsigned long long* stamps;  // profiling (null = off): per workgroup {start, end} s_memrealtime
  unsigned* ctr;               // dependency counters [kDepWords] (null = independent jobs)
  unsigned wait[kMaxMultiJobs];          // bit k: wait for job k
  unsigned char signal[kMaxMultiJobs];   // 0 none, 1 sc1 stores, 2 plain stores (release first)
  int nwait_blocks;                      // workgroups of all waiting jobs
};

constexpr int kMultiLds = cmax(cmax(cmax(wgrad_lds_bytes<W0>(), wgrad_lds_bytes<W1>()),
                                    cmax(wgrad_lds_bytes<W3>(), wgrad_lds_bytes<W4>())),
                               cmax(cmax(wgrad_lds_bytes<W2>(), wgrad_lds_bytes<W5>()),
                                    cmax(cmax(JFinalize::LDS, JComm::LDS), JColsum::LDS + 64)));

template <int CFG, class TC>
__device__ __forceinline__ bool run_wg_cfg(const JobBlob& j, uint8_t* lds, int b) {
  if (j.kind == kJobWgrad + CFG) {
    wgrad_body<__bf16, true, TC>(job_args<WgArgs>(j), lds, b, j.nblk);
    return true;
  }
  if (j.kind == kJobWgradThin + CFG) {
    wgrad_body<__bf16, false, TC>(job_args<WgArgs>(j), lds, b, j.nblk);
    return true;
  }
  if (j.kind == kJobWgradThin + 20 + CFG) {
    wgrad_body<float, false, TC>(job_args<WgArgs>(j), lds, b, j.nblk);
    return true;
  }
  return false;
}

__device__ __forceinline__ void run_multi_job(const JobBlob& j, uint8_t* lds, int lb) {
  if (run_wg_cfg<0, W0>(j, lds, lb) || run_wg_cfg<1, W1>(j, lds, lb) || run_wg_cfg<2, W2>(j, lds, lb) ||
      run_wg_cfg<3, W3>(j, lds, lb) || run_wg_cfg<4, W4>(j, lds, lb) || run_wg_cfg<5, W5>(j, lds, lb))
    return;
  switch (j.kind) {
    case kJobLossStep: JLossStep::run(j, lds, lb); break;
    case kJobLoss: JLoss::run(j, lds, lb); break;
    case kJobFinalize:
      if (job_args<FinalizeArgs>(j).dep)  // a dependent launch: slabs and step state written in it
        grad_finalize_body_t<true>(job_args<FinalizeArgs>(j), reinterpret_cast<float*>(lds),
                                   reinterpret_cast<AdamC*>(lds + kFinalizeThreads * 4), lb);
      else
        JFinalize::run(j, lds, lb);
      break;
    case kJobComm: JComm::run(j, lds, lb); break;
    case kJobColsum: JColsum::run(j, lds, lb); break;
    case kJobGather: JGather::run(j, lds, lb); break;
    default: break;
  }
}

// every counter access is a GLOBAL agent-scope access (never flat)
using gu32 = __attribute__((address_space(1))) unsigned;
__device__ __forceinline__ gu32* dep_word(unsigned* ctr, int i) { return (gu32*)(ctr + i * kDepStride); }

__device__ __forceinline__ void dep_wait(const JobPackN* __restrict__ p, unsigned* ctr, unsigned mask, int n) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < n; ++k) {
      if (!((mask >> k) & 1u)) continue;
      const unsigned need = (unsigned)(p->start[k + 1] - p->start[k]);
      while (__hip_atomic_load(dep_word(ctr, k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > kDepTimeoutTicks) {
          __hip_atomic_store(dep_word(ctr, kDepErr), 1u + (unsigned)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(MDT_DEP_SLEEP);
      }
    }
  }
  __syncthreads();
}

// After a waiting workgroup's work (off its critical path): the last one of
// the launch re-zeroes the counters. Every waiting workgroup has passed its
// wait by then, and every producer has counted itself (each is waited on in
// full), so nothing reads or adds to them any more in this launch.
__device__ __forceinline__ void dep_done(const JobPackN* __restrict__ p, unsigned* ctr, int n) {
  if (threadIdx.x == 0) {
    const unsigned done = __hip_atomic_fetch_add(dep_word(ctr, kDepDone), 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (done + 1 == (unsigned)p->nwait_blocks) {
      for (int k = 0; k < n; ++k) __hip_atomic_store(dep_word(ctr, k), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dep_word(ctr, kDepDone), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ void dep_signal(unsigned* ctr, int job, int mode) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left
  __syncthreads();                                  // ... every wave's
  if (threadIdx.x == 0) {
    if (mode == 2) {  // plain stores: write this XCD's dirty L2 lines back first
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(dep_word(ctr, job), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The job table lives in DEVICE memory (packed once per plan by the host,
// static across graph replays): a runtime index into a kernel-argument struct
// makes the compiler copy the whole 2.4 KB pack into per-lane scratch
// (measured 2368 B/lane, the launch ~10x slower), and selecting it with
// constant indices inlines every body eight times (1100+ SGPR spills).
// DEP = false: independent jobs, at most kPlainMultiJobs (the default path,
// code unchanged by the dependency support); DEP = true: a table packed with
// mdt_pack_jobs_multi_deps (up to kMaxMultiJobs jobs, counters in p->ctr).
constexpr int kPlainMultiJobs = 8;

template <bool DEP>
__global__ void __launch_bounds__(256) jobs_multi_k(const JobPackN* __restrict__ p) {
  constexpr int NJ = DEP ? kMaxMultiJobs : kPlainMultiJobs;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kMultiLds];
  const int b = blockIdx.x;
  // every start in ONE batch of scalar loads, then count the jobs this block
  // is past (starts ascend over [0, n)): a while loop over p->start was one
  // dependent load per job in front of the table's later (longest) jobs
  int st[NJ];
#pragma unroll
  for (int k = 0; k < NJ; ++k) st[k] = p->start[k];
  const int n = p->n;
  int i = 0, s0 = st[0];
#pragma unroll
  for (int k = 1; k < NJ; ++k)
    if (k < n && b >= st[k]) {
      i = k;
      s0 = st[k];
    }
  unsigned long long* stamps = p->stamps;
  unsigned long long t0 = 0;
  if (stamps) t0 = __builtin_amdgcn_s_memrealtime();
  if constexpr (DEP) {
    unsigned* ctr = p->ctr;
    const unsigned wmask = p->wait[i];
    if (wmask) dep_wait(p, ctr, wmask, n);
    run_multi_job(p->j[i], lds, b - s0);
    const int sig = p->signal[i];
    if (sig) dep_signal(ctr, i, sig);
    if (wmask) dep_done(p, ctr, n);
  } else {
    run_multi_job(p->j[i], lds, b - s0);
  }
  if (stamps) {  // which job ran where and when: overlap of jobs inside one launch (bench/ddp_structure.py)
    __syncthreads();
    if (threadIdx.x == 0) {
      stamps[2 * b] = t0;
      stamps[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

__host__ inline bool multi_kind_ok(int k) {
  if (k >= kJobWgrad && k <= kJobWgrad + 5) return true;
  if (k >= kJobWgradThin && k <= kJobWgradThin + 5) return true;
  if (k >= kJobWgradThin + 20 && k <= kJobWgradThin + 25) return true;
  return k == kJobLossStep || k == kJobLoss || k == kJobFinalize || k == kJobColsum || k == kJobComm ||
         k == kJobGather;
}

template <class A, class B, class C>
__global__ void __launch_bounds__(256) jobs_k(JobPack p) {
  // 1 KB aligned: the direct-conv bodies land LDS-DMA pieces at 1 KB offsets
  __shared__ __attribute__((aligned(1024))) uint8_t lds[cmax(cmax(A::LDS, B::LDS), cmax(C::LDS, 16))];
  const int b = blockIdx.x;
  if (b < p.start1) A::run(p.j[0], lds, b);
  else if (b < p.start2) B::run(p.j[1], lds, b - p.start1);
  else C::run(p.j[2], lds, b - p.start2);
}

}  // namespace mdt

using namespace mdt;

namespace {

typedef void (*PackLaunch)(const JobPack&, int, hipStream_t);

template <class A, class B, class C>
void launch_pack(const JobPack& p, int grid, hipStream_t s) {
  hipLaunchKernelGGL((jobs_k<A, B, C>), dim3(grid), dim3(256), 0, s, p);
}

struct Combo {
  int k0, k1, k2;
  PackLaunch fn;
};

#define COMBO3(A, B, C) {A::ID, B::ID, C::ID, &launch_pack<A, B, C>}
#define COMBO2(A, B) {A::ID, B::ID, 0, &launch_pack<A, B, JNone>}

using WgT5 = JWgThin<__bf16, 5, W5>;
using WgT5f = JWgThin<float, 5, W5>;
using ThinC32 = JThinConv<32, __bf16>;
using ThinC32f = JThinConv<32, float>;
using TwB = JThinWg<__bf16>;
using TwF = JThinWg<float>;
using Wg0 = JWg<0, W0>;
using Wg1 = JWg<1, W1>;
using IgC1 = JIg<kModeConv, 1, F1>;
using IgC4 = JIg<kModeConv, 4, F4>;
using IgC5 = JIg<kModeConv, 5, F5>;
using IgC6 = JIg<kModeConv, 6, F6>;
using IgT1 = JIg<kModeTconv, 1, F1>;
using IgT2 = JIg<kModeTconv, 2, F2>;
using IgT4 = JIg<kModeTconv, 4, F4>;
using IgT5 = JIg<kModeTconv, 5, F5>;
using IgT6 = JIg<kModeTconv, 6, F6>;
using DcJS2 = JDc<1, DcS2>;
using DcJT2 = JDc<2, DcT2>;

// kinds sorted ascending within each entry
const Combo kCombos[] = {
    // last layer: thin weight gradient || thin backward-data || loss reduction
    COMBO3(WgT5, ThinC32, JLoss),
    COMBO2(WgT5, ThinC32),
    COMBO3(TwB, ThinC32, JLoss),
    COMBO2(TwB, ThinC32),
    COMBO2(TwF, JFinalize),
    // transposed-conv layers: conv-mode backward-data || weight gradient
    COMBO2(IgC5, Wg0),
    COMBO2(IgC1, Wg0),
    COMBO2(IgC4, Wg0),
    COMBO2(IgC6, Wg0),  // 128x128: narrow column tiles of deep layers (BN split)
    COMBO3(IgC6, Wg0, JColsum),
    // decoder Linear (split-K backward-data) || weight gradient || its bias column sums
    COMBO3(IgT6, Wg1, JColsum),
    COMBO3(IgT5, Wg0, JColsum),
    COMBO3(IgT6, Wg0, JColsum),
    // encoder head || weight gradient || head bias column sums
    COMBO3(IgT4, Wg0, JColsum),
    // conv layers: parity-mode backward-data || weight gradient
    COMBO2(IgT6, Wg0),
    COMBO2(IgT4, Wg0),
    COMBO2(IgT1, Wg0),
    COMBO2(IgT2, Wg0),
    COMBO2(IgT5, Wg0),
    // backward-data || weight gradient || finalize+Adam of the layers whose
    // gradients the previous launches completed (spread optimizer)
    COMBO3(IgC1, Wg0, JFinalize),
    COMBO3(IgC4, Wg0, JFinalize),
    COMBO3(IgC5, Wg0, JFinalize),
    COMBO3(IgC6, Wg0, JFinalize),
    COMBO3(IgT1, Wg0, JFinalize),
    COMBO3(IgT2, Wg0, JFinalize),
    COMBO3(IgT4, Wg0, JFinalize),
    COMBO3(IgT6, Wg0, JFinalize),
    // optimizer tail: first-layer weight gradient || finalize+Adam of every
    // other layer; then first-layer finalize || transposed weight copies
    COMBO2(WgT5f, JFinalize),
    COMBO2(JFinalize, JWtrans),
    // step's first launch (batch gather + step begin + first layer) || the
    // transposed weight copies of the previous step's update (MDT_CONV_DEFER_WT=1)
    COMBO2(ThinC32f, JWtrans),
    // ... or the first decoder GEMM (MDT_CONV_DEFER_WT=2)
    COMBO2(IgC1, JWtrans),
    COMBO2(IgC4, JWtrans),
    COMBO2(IgC5, JWtrans),
    COMBO2(IgC6, JWtrans),
    // 128x128 32x32 <-> 16x16 layers: direct backward-data || im2col weight
    // gradient (the 64x64 <-> 32x32 pair's direct weight gradient runs 8-wave
    // workgroups in its own launch: 15.9 -> 14.2 us, profiles/r3_dconv2)
    COMBO2(Wg0, DcJS2),
    COMBO2(Wg0, DcJT2),
    // intra-group DDP with the fused xGMI all-reduce (comm_jobs.h): a backward
    // launch also pushes the gradients the previous launches completed; the
    // tail reduces + applies Adam (two comm jobs) after the first layer's
    // weight gradient pushed the rest
    COMBO3(IgC1, Wg0, JComm),
    COMBO3(IgC4, Wg0, JComm),
    COMBO3(IgC5, Wg0, JComm),
    COMBO3(IgC6, Wg0, JComm),
    COMBO3(IgT1, Wg0, JComm),
    COMBO3(IgT2, Wg0, JComm),
    COMBO3(IgT4, Wg0, JComm),
    COMBO3(IgT5, Wg0, JComm),
    COMBO3(IgT6, Wg0, JComm),
    COMBO3(Wg0, JComm, DcJS2),
    COMBO3(Wg0, JComm, DcJT2),
    COMBO2(TwF, JComm),
    COMBO2(WgT5f, JComm),
    COMBO2(JComm, JComm),
};

#undef COMBO3
#undef COMBO2

inline int cdivj(long long a, long long b) { return (int)((a + b - 1) / b); }

// workgroups of a direct-conv launch (conv_igemm.hip launch_dc)
template <class CF>
constexpr int dc_grid(int n) { return n * CF::RB * CF::NBB; }
inline int direct_grid(int dc, int n) {
  switch (dc) {
    case 0: return dc_grid<DcS1>(n);
    case 1: return dc_grid<DcS2>(n);
    case 2: return dc_grid<DcT2>(n);
    case 3: return dc_grid<DcT3>(n);
    default: return 0;
  }
}

template <class T>
void put_args(JobBlob* j, const T& a) {
  static_assert(sizeof(T) <= kJobArgBytes, "job arguments exceed the blob");
  memset(j->args, 0, sizeof(j->args));
  memcpy(j->args, &a, sizeof(T));
}

}  // namespace

extern "C" {

// Forward-type GEMM as a job (`g`); with split-K the combine pass is a second
// job (`c`, kind kJobCombine, to run after `g`), else c->kind = 0. g->kind = 0
// when the GEMM has no job form (f32 / per-element gathers, LDS-DMA path).
int mdt_job_igemm(JobBlob* g, JobBlob* c, int mode, const void* A, int a_is_f32, const void* B16, ConvDesc d,
                  const float* bias, int relu, void* y16, float* y32, const void* omask, float* colsum, float* ws,
                  int skip_combine) {
  IgArgs a;
  FwdPlan q;
  CombineArgs cb;
  int nc = 0;
  if (build_igemm(mode, A, B16, d, bias, relu, y16, y32, omask, colsum, ws, &a, &q, &cb, &nc)) return 1;
  memset(g, 0, sizeof(*g));
  memset(c, 0, sizeof(*c));
  // direct-kernel geometries: the direct body as a job (backward-data calls;
  // the 16x16 <-> 8x8 forward-only tiles have no job form)
  const int dc = direct_cfg(mode, d, false);
  if (dc >= 0) {
    if (a_is_f32 || dc > 3) return 0;  // kind 0: the caller launches it alone
    DcArgs da{};
    da.A = reinterpret_cast<const __bf16*>(A);
    da.B = reinterpret_cast<const __bf16*>(B16);
    da.y16 = reinterpret_cast<__bf16*>(y16);
    da.y32 = y32;
    da.bias = bias;
    da.omask = reinterpret_cast<const __bf16*>(omask);
    da.colsum = colsum;
    da.relu = relu;
    da.nimg = d.N;
    g->kind = kJobDconv + dc;
    g->nblk = direct_grid(dc, d.N);
    put_args(g, da);
    return 0;
  }
  const bool ok = !a_is_f32 && !q.thin;
  g->kind = ok ? kJobIgemm + mode * 100 + q.cfg : 0;
  g->nblk = q.mtiles * q.ntiles * q.ksplit * q.classes;
  g->aux[0] = q.mtiles * q.ntiles;
  g->aux[1] = q.ksplit;
  put_args(g, a);
  if (nc > 0 && !skip_combine) {
    c->kind = kJobCombine;
    c->nblk = nc;
    put_args(c, cb);
  }
  return 0;
}

int mdt_job_wgrad(JobBlob* j, const void* G16, const void* X, int x_is_f32, ConvDesc d, float* out) {
  WgArgs a;
  WgradPlan q;
  if (build_wgrad(G16, X, d, out, &a, &q)) return 1;
  memset(j, 0, sizeof(*j));
  if (q.cfg == 110) j->kind = kJobThinWgM + (x_is_f32 ? 1 : 0);  // MFMA thin weight gradient
  else if (q.cfg >= 100) {  // direct weight gradient (conv_dwgrad.h): 512-thread workgroups, its own launch
    return 0;
  }
  else if (!q.thin) j->kind = x_is_f32 ? 0 : kJobWgrad + q.cfg;
  else j->kind = kJobWgradThin + (x_is_f32 ? 20 : 0) + q.cfg;
  j->nblk = q.cotiles * q.ktiles * q.nsplit;
  put_args(j, a);
  return 0;
}

int mdt_job_thin_conv(JobBlob* j, const void* X, int x_is_f32, const float* Wf, ConvDesc d, const float* bias,
                      int relu, void* y16, const void* omask, float* colsum, const int* idx, void* st,
                      const void* hp, int B, float* xb) {
  if (d.C != 1 || d.KH != 4 || d.KW != 4) return 1;
  if ((idx || xb || hp) && (!st || !x_is_f32 || (d.H * d.W) % 4)) return 1;
  memset(j, 0, sizeof(*j));
  const bool ok = d.CO == 16 || d.CO == 32 || d.CO == 64;
  j->kind = ok ? kJobThinConv + d.CO + (x_is_f32 ? 100 : 0) : 0;
  j->nblk = cdivj((long long)d.N * d.OH * d.OW, 256);
  const ThinConvArgs ta{X, Wf, d, bias, relu, reinterpret_cast<__bf16*>(y16), reinterpret_cast<const __bf16*>(omask),
                        colsum, idx, reinterpret_cast<TrainState*>(st), reinterpret_cast<const HParams*>(hp), B, xb,
                        j->nblk, thin_conv_mfma_ok(d, x_is_f32)};
  put_args(j, ta);
  return 0;
}

int mdt_job_colsum(JobBlob* j, const void* G16, int M, int N, int rows_per, float* slab) {
  if (N % 8 || rows_per < 1) return 1;
  memset(j, 0, sizeof(*j));
  const int gx = cdivj(N / 8, 256);
  j->kind = kJobColsum;
  j->nblk = gx * cdivj(M, rows_per);
  put_args(j, ColsumArgs{reinterpret_cast<const __bf16*>(G16), M, N, rows_per, gx, slab});
  return 0;
}

int mdt_job_loss(JobBlob* j, const float* bce_part, int nb, const float* kld_part, int nk, void* st, const void* hp,
                 int advance_cursor) {
  memset(j, 0, sizeof(*j));
  // bit 0: advance the batch cursor; bit 1: also advance the step (loss_step_body)
  j->kind = (advance_cursor & 2) ? kJobLossStep : kJobLoss;
  advance_cursor &= 1;
  j->nblk = 1;
  put_args(j, LossArgs{bce_part, nb, kld_part, nk, reinterpret_cast<TrainState*>(st),
                       reinterpret_cast<const HParams*>(hp), advance_cursor});
  return 0;
}

int mdt_job_finalize(JobBlob* j, float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs,
                     const void* units, int nunits, const void* st, const void* hp, int do_adam, int dep) {
  memset(j, 0, sizeof(*j));
  if (nunits <= 0) return 1;
  j->kind = kJobFinalize;
  j->nblk = nunits;
  put_args(j, FinalizeArgs{P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16), reinterpret_cast<const GradSeg*>(segs),
                           reinterpret_cast<const GradUnit*>(units), reinterpret_cast<const TrainState*>(st),
                           reinterpret_cast<const HParams*>(hp), do_adam, dep ? 1 : 0});
  return 0;
}

int mdt_job_comm(JobBlob* j, float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs, const void* units,
                 int nunits, const void* st, const void* hp, int do_adam, const void* ctx, int mode) {
  memset(j, 0, sizeof(*j));
  if (nunits <= 0 || !ctx || mode < kCommPush || mode > kCommPushReduce) return 1;
  j->kind = kJobComm;
  j->nblk = nunits;
  CommJobArgs a{};
  a.fa = FinalizeArgs{P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16), reinterpret_cast<const GradSeg*>(segs),
                      reinterpret_cast<const GradUnit*>(units), reinterpret_cast<const TrainState*>(st),
                      reinterpret_cast<const HParams*>(hp), do_adam};
  a.ctx = reinterpret_cast<const CommCtx*>(ctx);
  a.mode = mode;
  put_args(j, a);
  return 0;
}

int mdt_job_wtrans(JobBlob* j, const void* w16, void* w16t, const void* segs, const void* units, int nunits) {
  memset(j, 0, sizeof(*j));
  if (nunits <= 0) return 1;
  j->kind = kJobWtrans;
  j->nblk = nunits;
  put_args(j, WtransArgs{reinterpret_cast<const __bf16*>(w16), reinterpret_cast<__bf16*>(w16t),
                         reinterpret_cast<const GradSeg*>(segs), reinterpret_cast<const TrUnit*>(units)});
  return 0;
}

// Launch 2-3 jobs as ONE kernel. Returns 0 when launched, 1 when no fused
// kernel exists for this combination of kinds (nothing launched: the caller
// falls back to the stand-alone kernels), 2 on bad input.
int mdt_launch_jobs(const JobBlob* jobs, int n, hipStream_t s) {
  if (n < 2 || n > 3) return 2;
  const JobBlob* v[3] = {&jobs[0], &jobs[1], n > 2 ? &jobs[2] : nullptr};
  for (int i = 0; i < n; ++i)
    if (v[i]->kind <= 0 || v[i]->nblk <= 0) return 1;
  std::sort(v, v + n, [](const JobBlob* a, const JobBlob* b) { return a->kind < b->kind; });
  const int k2 = n > 2 ? v[2]->kind : 0;
  for (const Combo& c : kCombos) {
    if (c.k0 != v[0]->kind || c.k1 != v[1]->kind || c.k2 != k2) continue;
    JobPack p;
    memset(&p, 0, sizeof(p));
    p.j[0] = *v[0];
    p.j[1] = *v[1];
    if (n > 2) p.j[2] = *v[2];
    p.start1 = v[0]->nblk;
    p.start2 = v[0]->nblk + v[1]->nblk;
    const int grid = p.start2 + (n > 2 ? v[2]->nblk : 0);
    c.fn(p, grid, s);
    return (int)hipGetLastError() ? -1 : 0;
  }
  return 1;
}

// Pack 1..kMaxMultiJobs jobs of any supported kinds into a JobPackN image at
// `dst` (host memory, mdt_jobs_multi_bytes() bytes; the caller uploads it once).
// Returns the grid size, 0 for an unsupported kind, -1 for bad input.
int mdt_jobs_multi_bytes() { return (int)sizeof(JobPackN); }

int mdt_pack_jobs_multi_stamps(void* img, void* stamps) {
  reinterpret_cast<JobPackN*>(img)->stamps = reinterpret_cast<unsigned long long*>(stamps);
  return 0;
}

int mdt_pack_jobs_multi(const JobBlob* jobs, int n, void* dst) {
  if (n < 1 || n > kMaxMultiJobs) return -1;
  JobPackN p;
  memset(&p, 0, sizeof(p));
  int grid = 0;
  for (int i = 0; i < n; ++i) {
    if (jobs[i].nblk <= 0) return -1;
    if (!multi_kind_ok(jobs[i].kind)) return 0;
    p.j[i] = jobs[i];
    p.start[i] = grid;
    grid += jobs[i].nblk;
  }
  p.start[n] = grid;
  p.n = n;
  memcpy(dst, &p, sizeof(p));
  return grid;
}

// Dependencies for a packed table (see JobDeps above JobPackN): wait[i] is
// the bit mask of the jobs job i waits for; ctr the zeroed device counter
// block (mdt_jobs_dep_words() words). Producers must precede their waiters
// and must not wait themselves. Returns 0, or -1 for a bad table.
int mdt_jobs_dep_words() { return kDepWords; }
int mdt_jobs_dep_err() { return kDepErr * kDepStride; }

static int dep_signal_mode(const JobBlob& j) {
  const int k = j.kind;
  if (k == kJobThinWgM || k == kJobThinWgM + 1) {  // sc1 row stores when the slab is 16-B aligned
    const WgArgs& a = *reinterpret_cast<const WgArgs*>(j.args);
    return ((uintptr_t)a.out & 15) == 0 ? 1 : 2;
  }
  if ((k >= kJobWgrad && k <= kJobWgrad + 5) || (k >= kJobWgradThin && k <= kJobWgradThin + 25)) {
    const WgArgs& a = *reinterpret_cast<const WgArgs*>(j.args);  // wgrad_epilogue: sc1 slabs when K2 % 4 == 0
    return (a.K2 & 3) == 0 ? 1 : 2;
  }
  return 2;  // loss / step state and anything else: plain stores, release first
}

int mdt_pack_jobs_multi_deps(void* img, void* ctr, const unsigned* wait, int n) {
  JobPackN* p = reinterpret_cast<JobPackN*>(img);
  if (!ctr || n != p->n) return -1;
  unsigned producers = 0;
  int nwait = 0;
  for (int i = 0; i < n; ++i) {
    const unsigned w = wait[i];
    if (w >> i) return -1;  // a job may only wait for jobs before it (and never for itself)
    producers |= w;
    if (w) nwait += p->start[i + 1] - p->start[i];
  }
  for (int i = 0; i < n; ++i) {
    if (((producers >> i) & 1u) && wait[i]) return -1;  // no chains: producers never wait
    p->wait[i] = wait[i];
    p->signal[i] = ((producers >> i) & 1u) ? (unsigned char)dep_signal_mode(p->j[i]) : 0;
  }
  if (!nwait) return -1;
  p->nwait_blocks = nwait;
  p->ctr = reinterpret_cast<unsigned*>(ctr);
  return 0;
}

int mdt_job_gather(JobBlob* j, const float* X, const int* idx, const void* st, float* xn, unsigned* xtag, int B) {
  memset(j, 0, sizeof(*j));
  if (!X || !idx || !st || !xn || !xtag || B <= 0) return 1;
  j->kind = kJobGather;
  j->nblk = gather_blocks(B);
  put_args(j, BatchGather{X, idx, reinterpret_cast<const TrainState*>(st), xn, xtag, B, 0});
  return 0;
}

// ONE jobs_multi_k launch over a packed table already in device memory.
int mdt_launch_jobs_multi(const void* dev_pack, int grid, int dep, hipStream_t s) {
  if (!dev_pack || grid <= 0) return 2;
  if (dep)
    hipLaunchKernelGGL(jobs_multi_k<true>, dim3(grid), dim3(256), 0, s, reinterpret_cast<const JobPackN*>(dev_pack));
  else
    hipLaunchKernelGGL(jobs_multi_k<false>, dim3(grid), dim3(256), 0, s, reinterpret_cast<const JobPackN*>(dev_pack));
  return (int)hipGetLastError() ? -1 : 0;
}

// Launch one job with its stand-alone kernel form (combine / colsum / loss).
int mdt_launch_job1(const JobBlob* j, hipStream_t s) {
  if (j->kind == kJobCombine) return launch_splitk_combine(*reinterpret_cast<const CombineArgs*>(j->args), j->nblk, s);
  return 1;
}

}  // extern "C"
