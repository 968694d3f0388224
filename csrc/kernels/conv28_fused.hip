// Fused 28x28 conv-VAE step kernels (gfx950) and their launchers.
//
//   f28_fwd_k   one workgroup per sample: forward (train or eval)
//   f28_bwd_k   one workgroup per sample: backward-data (two-launch form)
//   f28_step_k  forward + backward in one launch: grid 2M with two workgroups
//               per sample (conv28_pair.h; a leader whose partner is not
//               resident in time runs the solo body), or grid M solo
//
// Bodies: conv28_fused.h (solo), conv28_pair.h (pairs).
#include <stdlib.h>

#include "conv28_pair.h"

namespace mdt {
namespace f28 {

__global__ void __launch_bounds__(kThreads) f28_fwd_k(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[FwdLayout::LDS];
  fwd_body<FwdLayout>(a, lds, blockIdx.x);
}

__global__ void __launch_bounds__(kThreads) f28_bwd_k(BwdArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[BwdLayout::LDS];
  bwd_body<BwdLayout, false>(a, lds, blockIdx.x);
}

__global__ void __launch_bounds__(kThreads) f28_step_k(FwdArgs fa, BwdArgs ba, PairCtl pc) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[StepLayout::LDS];
  if (pc.acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (!pc.pair) {
    const int n = blockIdx.x;
    fwd_body<StepLayout>(fa, lds, n);
    if (!fa.train) return;  // eval: forward only
    lds_barrier();
    bwd_body<StepLayout, true>(ba, lds, n);
    return;
  }
  // pairing (see conv28_pair.h): ticket at entry, the leader's solo claim
  // after P0 (its result is needed only after P1, which both forms share)
  const int n = (int)blockIdx.x % pc.M;
  g32i* word = (g32i*)(pc.pairw + n);
  int ticket = 0, seen = 1;
  if (pc.delay_us > 0 && (int)blockIdx.x >= pc.M && threadIdx.x == 0) {  // tests: a partner that comes late
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * (unsigned)pc.delay_us) __builtin_amdgcn_s_sleep(8);
  }
  if (threadIdx.x == 0) ticket = __hip_atomic_fetch_add(word, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  fill_ptab<StepLayout>(lds, fa, ba, pc, n);  // read by the paired body after P0's barrier
  fwd_p01<StepLayout>(fa, lds, n, [&] {
    if (threadIdx.x == 0 && ticket == 0)
      __hip_atomic_compare_exchange_strong(word, &seen, 3, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
  });
  int* mode_w = reinterpret_cast<int*>(lds + StepLayout::Scr + 124);  // Scr[31]: unused before P4
  if (threadIdx.x == 0) {
    int mode;
    if (ticket == 0) {
      mode = seen == 1 ? kModeSolo : kModeRole0;  // CAS 1 -> 3 won: solo; saw 2: the partner is in
      if (mode == kModeRole0) __hip_atomic_store(word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (ticket == 1) {
      mode = kModeRole1;
    } else {  // the leader went solo before this workgroup arrived: last to touch the word
      mode = kModeExit;
      __hip_atomic_store(word, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *mode_w = mode;
    if (fa.stamps) fa.stamps[blockIdx.x * 16 + 15] = (unsigned long long)mode;
  }
  lds_barrier();
  const int mode = __builtin_amdgcn_readfirstlane(*mode_w);
  if (mode == kModeExit) return;
  if (mode == kModeSolo) {
    fwd_rest<StepLayout>(fa, lds, n);
    if (!fa.train) return;  // eval: forward only
    lds_barrier();
    bwd_body<StepLayout, true>(ba, lds, n);
    return;
  }
  if (pc.delay_us < 0 && mode == kModeRole1 && n == 0) {  // tests: a paired half that stalls (sweep timeout)
    if (threadIdx.x == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * (unsigned)(-pc.delay_us)) __builtin_amdgcn_s_sleep(64);
    }
    lds_barrier();
  }
  pair_rest<StepLayout>(lds, n, mode == kModeRole1 ? 1 : 0);
}

}  // namespace f28
}  // namespace mdt

using namespace mdt;

namespace {

template <class T>
T* P(const long long* p, int i) {
  return reinterpret_cast<T*>((intptr_t)p[i]);
}

void fill_weights(f28::Weights& w, const long long* p) {
  w.W1f = P<const float>(p, 0);
  w.b1 = P<const float>(p, 1);
  w.W2 = P<const __bf16>(p, 2);
  w.b2 = P<const float>(p, 3);
  w.Wh = P<const __bf16>(p, 4);
  w.bh = P<const float>(p, 5);
  w.Wd = P<const __bf16>(p, 6);
  w.bd = P<const float>(p, 7);
  w.W3 = P<const __bf16>(p, 8);
  w.b3 = P<const float>(p, 9);
  w.W4f = P<const float>(p, 10);
  w.b4 = P<const float>(p, 11);
}

void fill_fwd(f28::FwdArgs& a, const long long* p, int B, unsigned stream, int train) {
  fill_weights(a.w, p);
  a.X = P<const float>(p, 12);
  a.idx = P<const int>(p, 13);
  a.st = P<const TrainState>(p, 14);
  a.hp = P<const HParams>(p, 15);
  a.B = B;
  a.stream = stream;
  a.train = train;
  a.xb = P<float>(p, 16);
  a.a1 = P<__bf16>(p, 17);
  a.a2 = P<__bf16>(p, 18);
  a.mulv = P<float>(p, 19);
  a.eps = P<float>(p, 20);
  a.z16 = P<__bf16>(p, 21);
  a.d0 = P<__bf16>(p, 22);
  a.d1 = P<__bf16>(p, 23);
  a.dlog = P<float>(p, 24);
  a.recon = P<float>(p, 25);
  a.bce_part = P<float>(p, 26);
  a.kld_part = P<float>(p, 27);
  a.db4_part = P<float>(p, 28);
  a.stamps = P<unsigned long long>(p, 29);
  a.pf_slices = 16;
  a.xn = P<const float>(p, 30);
  a.xtag = P<const unsigned>(p, 31);
}

void fill_bwd(f28::BwdArgs& a, const long long* p, int M) {
  fill_weights(a.w, p);
  a.hp = P<const HParams>(p, 12);
  a.mulv = P<const float>(p, 13);
  a.eps = P<const float>(p, 14);
  a.a1 = P<const __bf16>(p, 15);
  a.a2 = P<const __bf16>(p, 16);
  a.d0 = P<const __bf16>(p, 17);
  a.d1 = P<const __bf16>(p, 18);
  a.dlog = P<const float>(p, 19);
  a.gd1 = P<__bf16>(p, 20);
  a.gd0 = P<__bf16>(p, 21);
  a.dbd_part = P<float>(p, 22);
  a.dmulv = P<float>(p, 23);
  a.dmulv16 = P<__bf16>(p, 24);
  a.ga2 = P<__bf16>(p, 25);
  a.ga1 = P<__bf16>(p, 26);
  a.db3_part = P<float>(p, 27);
  a.db2_part = P<float>(p, 28);
  a.db1_part = P<float>(p, 29);
  a.stamps = P<unsigned long long>(p, 30);
  a.db2_m2 = M;  // db2_part is always [2][M][64] (second row: the paired step's role-1 half)
}

}  // namespace

extern "C" {

// Pointer tables (validated by the caller, csrc/runtime/conv_ops.cpp):
// forward  [0..11] weights (W1f b1 W2 b2 Wh bh Wd bd W3 b3 W4f b4), 12 X, 13 idx,
//          14 state, 15 hparams, 16 xb, 17 a1, 18 a2, 19 mulv, 20 eps, 21 z16,
//          22 d0, 23 d1, 24 dlog, 25 recon, 26 bce_part, 27 kld_part, 28 db4_part,
//          29 stamps (optional)
// backward [0..11] weights, 12 hparams, 13 mulv, 14 eps, 15 a1, 16 a2, 17 d0,
//          18 d1, 19 dlog, 20 gd1, 21 gd0, 22 dbd_part, 23 dmulv, 24 dmulv16,
//          25 ga2, 26 ga1, 27 db3_part, 28 db2_part ([2][M][64]), 29 db1_part,
//          30 stamps (optional)
// pair     0 exchange granules [M][2][f28_pair_words], 1 pairing words [M] int32,
//          2 error word (uint32); all zero before the first launch
int mdt_f28_forward(const long long* p, int B, int M, unsigned stream, int train, hipStream_t s) {
  if (M <= 0 || M > B) return 1;
  f28::FwdArgs a{};
  fill_fwd(a, p, B, stream, train);
  hipLaunchKernelGGL(f28::f28_fwd_k, dim3(M), dim3(f28::kThreads), 0, s, a);
  return (int)hipGetLastError();
}

int mdt_f28_pair_words() { return f28::kXW; }

// Forward only (eval: train = 0) through the step kernel's paired form: two
// workgroups per sample, so an eval batch of M samples fills 2M CUs instead of
// the solo f28_fwd_k's M. Same arithmetic as the solo forward (the paired and
// solo forms are bitwise equal); the backward half of the kernel is skipped.
int mdt_f28_forward_pair(const long long* p, const long long* pp, int B, int M, unsigned stream, hipStream_t s) {
  if (M <= 0 || M > B) return 1;
  if (!pp || !pp[0] || !pp[1] || !pp[2]) return 2;
  f28::FwdArgs fa{};
  fill_fwd(fa, p, B, stream, 0);
  fa.pf_slices = 0;
  f28::BwdArgs ba{};
  f28::PairCtl pc{};
  pc.M = M;
  pc.pair = 1;
  pc.xg = P<unsigned long long>(pp, 0);
  pc.pairw = P<int>(pp, 1);
  pc.err = P<unsigned>(pp, 2);
  hipLaunchKernelGGL(f28::f28_step_k, dim3(2 * M), dim3(f28::kThreads), 0, s, fa, ba, pc);
  return (int)hipGetLastError();
}

// One launch per training step: forward then backward, two workgroups per
// sample when `pair` (pp = pair table), else one.
int mdt_f28_step(const long long* pf, const long long* pb, const long long* pp, int B, int M, unsigned stream,
                 int pair, int delay_us, hipStream_t s) {
  if (M <= 0 || M > B) return 1;
  f28::FwdArgs fa{};
  fill_fwd(fa, pf, B, stream, 1);
  f28::BwdArgs ba{};
  fill_bwd(ba, pb, M);
  f28::PairCtl pc{};
  pc.M = M;
  pc.pair = pair ? 1 : 0;
  pc.delay_us = delay_us;
  static const int acq = [] {
    const char* e = getenv("MDT_F28_ACQ");
    return e && e[0] == '1' ? 1 : 0;
  }();
  pc.acquire = acq;
  if (pair) {
    if (!pp || !pp[0] || !pp[1] || !pp[2]) return 2;
    pc.xg = P<unsigned long long>(pp, 0);
    pc.pairw = P<int>(pp, 1);
    pc.err = P<unsigned>(pp, 2);
    // no P0 L2 prefetch in the paired form: measured 0.0636-0.0639 vs
    // 0.0638-0.0644 ms/step on the driver command with 32 slices, 200/20
    // 0.0608-0.0613 vs 0.0616-0.0622 (profiles/r4_end, gpurun_out r4af/r4ag)
    fa.pf_slices = 0;
  }
  static const int pf_env = [] {  // A/B: MDT_F28_PF = L2-prefetch slices per XCD (0 = no prefetch)
    const char* e = getenv("MDT_F28_PF");
    return e ? atoi(e) : -1;
  }();
  if (pf_env >= 0) fa.pf_slices = pf_env;
  hipLaunchKernelGGL(f28::f28_step_k, dim3(pair ? 2 * M : M), dim3(f28::kThreads), 0, s, fa, ba, pc);
  return (int)hipGetLastError();
}

int mdt_f28_backward(const long long* p, int M, hipStream_t s) {
  if (M <= 0) return 1;
  f28::BwdArgs a{};
  fill_bwd(a, p, M);
  hipLaunchKernelGGL(f28::f28_bwd_k, dim3(M), dim3(f28::kThreads), 0, s, a);
  return (int)hipGetLastError();
}

}  // extern "C"
