// Two workgroups per sample for the fused 28x28 conv-VAE step (gfx950).
//
// Why: the solo step (conv28_fused.h) runs one 512-thread workgroup per
// sample, so a B = 128 trial -- the headline config -- keeps 128 of the 256
// CUs busy, and its per-sample Linear GEMVs re-stream 600 KB of weights per
// CU per direction. Here a launch of 2M workgroups gives every sample a PAIR
// (blocks n and n + M: with M % 8 == 0 round-robin dispatch puts both on one
// XCD, which buys L2 sharing of the weight slices -- speed only, never
// correctness). Each half does half of every heavy phase:
//
//   7x7 maps (enc2 out, dec_fc out, their gradients): split by PIXEL --
//     role 0 owns pixels 0..23, role 1 pixels 24..48, i.e. the contiguous
//     ranges [0, 1536) / [1536, 3136) of the flattened 3136-vectors, so the
//     Linear weight streams (head rows, dec_fc rows) are contiguous slices;
//   14x14 maps (dec1 out, enc1 grad): split by CHANNEL -- 16 of 32 each;
//   enc1, reparam, BCE/dlogits (cheap, and needed whole): both, redundantly
//     and bitwise identically (fixed (role 0 + role 1) summation order).
//
// Six hand-offs per step, each a data-tagged 8-byte granule sweep
// (MI355X_MICROARCH.md "handoff-1to1"; cdna_hip_programming.md Guideline 16
// R2: {tag, payload} in ONE agent-scope store, so the data is its own flag and
// no release/acquire fence is needed):
//   X1 head partial sums (64 f32, K split)    X4 gd1 channel half (3 KB bf16)
//   X2 d0 pixel half (~3 KB bf16)             X5 dz partial sums (32 f32)
//   X3 dec2 partial logits (784 f32)          X6 ga2 pixel half (~3 KB bf16)
// The consumer clears every granule it read, so the slabs are all-zero
// between launches (graph replays need no memset node); tags also carry the
// step so a stale granule can never match.
//
// Pairing never assumes co-residency. Each workgroup takes a ticket on its
// sample's word at entry; the first arriver (leader) claims the sample SOLO
// with a CAS after P0 unless the partner has already taken the second ticket.
// A solo leader runs the one-workgroup body; a partner that arrives after the
// claim exits. So a launch that cannot hold all 2M workgroups at once (trial
// packing, a busy device) degrades to the solo step instead of deadlocking.
// Every sweep is bounded (s_memrealtime) and reports a timeout in `err`.
//
// Bias-gradient partials: per-channel sums over the 7x7 pixels (enc2 bias)
// come out per half, so db2_part is [2][M][64] and the finalize sums 2M rows;
// everything else each half writes into its own part of the solo layout.
#pragma once
#include "conv28_fused.h"

namespace mdt {
namespace f28 {

struct PairCtl {
  unsigned long long* xg;  // [M][2][kXW] exchange granules (all zero between launches)
  int* pairw;              // [M] pairing words (0 between launches)
  unsigned* err;           // [1] bit 0: an exchange sweep timed out
  int M;
  int pair;                // 1: grid = 2M (pairs), 0: grid = M (solo)
  int delay_us;            // tests: > 0 workgroups >= M wait this long before their ticket (forces solo);
                           //        < 0 sample 0's role-1 half stalls -delay_us after pairing (forces a
                           //        sweep timeout of its partner: `err` bit 0)
  int acquire;             // diagnostic (MDT_F28_ACQ=1): agent-scope acquire fence at kernel entry
};

// granule offsets inside one (sample, role) slab
constexpr int kX1 = 0, kX2 = 72, kX3 = kX2 + 800, kX4 = kX3 + 784, kX5 = kX4 + 1568, kX6 = kX5 + 32;
constexpr int kXW = kX6 + 800;
constexpr unsigned long long kSpinTicks = 25000000ull;  // 0.25 s of s_memrealtime (100 MHz)

enum : int { kModeSolo = 0, kModeRole0 = 1, kModeRole1 = 2, kModeExit = 3 };

// Pointer table in LDS (StepLayout::PTab): the paired body takes every buffer
// pointer from here, already offset to its sample, instead of from the kernel
// arguments. Kept as arguments, the ~60 pointers of FwdArgs + BwdArgs did not
// fit the 102 SGPRs: the compiler spilled them to VGPR lanes and reloaded a
// 16-SGPR block (16 v_readlane) around every global store of an epilogue. A
// table read costs one ds_read_b64 + two readfirstlane per pointer per phase.
enum : int {
  kTWh, kTWd, kTW3, kTW2, kTSt, kTHp, kTA2, kTMulv, kTEps, kTZ16, kTD0, kTD1, kTDlog, kTRecon, kTBce, kTKld,
  kTDb4, kTStamp, kTGd1, kTDb3, kTGd0, kTDbd, kTDmulv, kTDmulv16, kTGa2, kTDb2, kTGa1, kTDb1, kTXg, kTErr,
  kTInts, kTNum  // kTInts: M | stream << 16 ... packed below
};

using g64 = __attribute__((address_space(1))) unsigned long long;
using g32i = __attribute__((address_space(1))) int;

// `near`: both workgroups of the pair run on ONE XCD (their HW_REG_XCC_ID
// match, exchanged in X1), so they share one L2: the granule goes out as a
// plain (workgroup-scope) store that stays in that L2 instead of an sc1
// write-through to memory, and the partner's sc1 (L1-bypassing, agent-scope)
// polls hit it there. Read from the hardware at run time, not assumed from
// dispatch order: with different XCDs every store stays agent scope.
// Why this is sound on gfx950 although the HIP scoped model gives a
// workgroup-scope store no visibility to another workgroup: the vector L1 is
// write-through -- a plain store leaves the CU for the XCD's L2 and keeps the
// line there (MI355X_MICROARCH.md, "stores of each flavour") -- the consumer
// never reads its own L1 (sc1 loads), and {tag, payload} is ONE 8-byte store,
// so there is no payload/flag ordering to lose. Measured (profiles/r4_near_scope):
// agent scope on the near path costs +1.1-1.3 us per 64 us step (driver
// command 0.0652-0.0653 vs 0.0640-0.0642 ms). Stress coverage: pairs run under
// a concurrent GEMM stream and a packed second trial, near pairs counted from
// the stamps, results bitwise run to run (tests/gpu/test_conv28_fused.py,
// scripts/diag/diag_determinism.py). MDT_HIP_EXTRA_FLAGS=-DMDT_F28_NEAR_WG=0 builds
// the agent-scope form.
#ifndef MDT_F28_NEAR_WG  // 0: agent scope on the near path too (A/B build, profiles/r4_near_scope)
#define MDT_F28_NEAR_WG 1
#endif
__device__ __forceinline__ void xput(unsigned long long* g, uint32_t tag, uint32_t v, bool near) {
  const unsigned long long x = ((unsigned long long)tag << 32) | v;
  if (near && MDT_F28_NEAR_WG)
    __hip_atomic_store((g64*)g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    __hip_atomic_store((g64*)g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Each lane waits for its N granules gi[k] (< 0: none) of slab `base` to
// carry `tag`, returns their payloads in v and clears them. Wave-uniform loop.
template <int N>
__device__ __forceinline__ void xget(unsigned long long* base, const int (&gi)[N], uint32_t tag, uint32_t (&v)[N],
                                     unsigned* err, bool near) {
  uint32_t pend = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    v[k] = 0;
    if (gi[k] >= 0) pend |= 1u << k;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned spin = 0;; ++spin) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (pend & (1u << k)) {
        const unsigned long long x = __hip_atomic_load((g64*)(base + gi[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(x >> 32) == tag) {
          v[k] = (uint32_t)x;
          pend &= ~(1u << k);
        }
      }
    }
    if (!__any(pend != 0)) break;
    if ((spin & 15) == 15 && __builtin_amdgcn_s_memrealtime() - t0 > kSpinTicks) {
      if (pend) atomicOr(err, 1u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (gi[k] >= 0) {
      if (near && MDT_F28_NEAR_WG)
        __hip_atomic_store((g64*)(base + gi[k]), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        __hip_atomic_store((g64*)(base + gi[k]), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <class L, class T>
__device__ __forceinline__ T* tab(const uint8_t* lds, int i) {
  const unsigned long long v = reinterpret_cast<const unsigned long long*>(lds + L::PTab)[i];
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  // through a global-address-space pointer, so the accesses stay global_* (a
  // generic pointer would make them flat_*, which also count in lgkmcnt and
  // so hold every later LDS wait until the global access completes)
  auto* g = (__attribute__((address_space(1))) T*)(((unsigned long long)hi << 32) | lo);
  return (T*)g;
}

// Thread 0 writes the table for sample n (visible after P0's barrier).
template <class L>
__device__ __forceinline__ void fill_ptab(uint8_t* lds, const FwdArgs& a, const BwdArgs& b, const PairCtl& pc, int n) {
  if (threadIdx.x != 0) return;
  unsigned long long* t = reinterpret_cast<unsigned long long*>(lds + L::PTab);
  auto at = [](const void* p, size_t bytes) {
    return p ? (unsigned long long)(reinterpret_cast<const char*>(p) + bytes) : 0ull;
  };
  const size_t N = (size_t)n;
  t[kTWh] = at(a.w.Wh, 0);
  t[kTWd] = at(a.w.Wd, 0);
  t[kTW3] = at(a.w.W3, 0);
  t[kTW2] = at(a.w.W2, 0);
  t[kTSt] = at(a.st, 0);
  t[kTHp] = at(a.hp, 0);
  t[kTA2] = at(a.a2, N * kFlat * 2);
  t[kTMulv] = at(a.mulv, N * 64 * 4);
  t[kTEps] = at(a.eps, N * 32 * 4);
  t[kTZ16] = at(a.z16, N * 32 * 2);
  t[kTD0] = at(a.d0, N * kFlat * 2);
  t[kTD1] = at(a.d1, N * 6272 * 2);
  t[kTDlog] = at(a.dlog, N * 784 * 4);
  t[kTRecon] = at(a.recon, N * 784 * 4);
  t[kTBce] = at(a.bce_part, N * 4);
  t[kTKld] = at(a.kld_part, N * 4);
  t[kTDb4] = at(a.db4_part, N * 4);
  t[kTStamp] = at(a.stamps, (size_t)blockIdx.x * 16 * 8);
  t[kTGd1] = at(b.gd1, N * 6272 * 2);
  t[kTDb3] = at(b.db3_part, N * 32 * 4);
  t[kTGd0] = at(b.gd0, N * kFlat * 2);
  t[kTDbd] = at(b.dbd_part, N * kFlat * 4);
  t[kTDmulv] = at(b.dmulv, N * 64 * 4);
  t[kTDmulv16] = at(b.dmulv16, N * 64 * 2);
  t[kTGa2] = at(b.ga2, N * kFlat * 2);
  t[kTDb2] = at(b.db2_part, N * 64 * 4);
  t[kTGa1] = at(b.ga1, N * 6272 * 2);
  t[kTDb1] = at(b.db1_part, N * 32 * 4);
  t[kTXg] = at(pc.xg, N * 2 * kXW * 8);
  t[kTErr] = at(pc.err, 0);
  t[kTInts] = (unsigned long long)(pc.M & 0xffff) | ((unsigned long long)(a.train ? 1 : 0) << 16) |
              ((unsigned long long)a.stream << 32);
}

__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t bf16bits(__bf16 h) { return (uint32_t)__builtin_bit_cast(uint16_t, h); }

// conv14to7 restricted to output pixels [p0, p1) (<= 32 of them): 2 m-tiles
// x 4 n-tiles, one item per wave.
// Out-of-image taps read the 16-B zero chunk `zero` (a select, not a branch
// around the load), and all 16 A and B fragments are read before the first
// MFMA: the gathers are issued back to back and only the MFMA chain waits.
template <class BFrag, class Pre, class Epi>
__device__ __forceinline__ void conv14to7_rows(const uint8_t* in_img, const uint8_t* zero, int p0, int p1,
                                               BFrag bfrag, Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = w & 3, mt = w >> 2;
  float pv[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int p = p0 + mt * 16 + 4 * (lane >> 4) + rr;
    pv[rr] = pre(p < p1 ? p : p1 - 1, 16 * j + (lane & 15));
  }
  const int r0 = p0 + mt * 16 + (lane & 15);
  const int r = r0 < 49 ? r0 : 48;  // padding rows (>= p1) compute garbage that is never stored
  const int oy = r / 7, ox = r - 7 * (r / 7), ch = lane >> 4;
  const uint32_t zoff = (uint32_t)(zero - in_img);
  bf16x8 av[16], bv[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int iy = 2 * oy - 1 + (t >> 2), ix = 2 * ox - 1 + (t & 3);
    const bool ok = (unsigned)iy < 14u && (unsigned)ix < 14u;
    const int pix = ok ? iy * 14 + ix : 0;
    const uint32_t off = ok ? (uint32_t)img14(pix, ch) : zoff;
    av[t] = *reinterpret_cast<const bf16x8*>(in_img + off);
    bv[t] = bfrag(j, t);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 16; ++t) acc = mfma_bf16(av[t], bv[t], acc);
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int p = p0 + mt * 16 + 4 * (lane >> 4) + rr;
    if (p < p1) epi(p, 16 * j + (lane & 15), acc[rr], pv[rr]);
  }
}

// tconv7to14 restricted to output channels [16 nj, 16 nj + 16): 4 classes x
// 4 m-tiles, two items per wave (classes w >> 2 and (w >> 2) + 2, m-tile
// w & 3). Returns this lane's column (16 nj + (lane & 15)) sum of epi's values
// over the wave's items.
template <class Pre, class Epi>
__device__ __forceinline__ float tconv7to14_half(const uint8_t* in, const uint8_t* zero, const uint8_t* wimg, int nj,
                                                 Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int mt = w & 3;
  float pv[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = (w >> 2) + 2 * i;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r2 = mt * 16 + 4 * (lane >> 4) + rr;
      const int rc = r2 < 49 ? r2 : 48;
      const int jy2 = rc / 7, jx2 = rc - 7 * (rc / 7);
      pv[i][rr] = pre((2 * jy2 + (q >> 1)) * 14 + 2 * jx2 + (q & 1), 16 * nj + (lane & 15));
    }
  }
  const uint32_t zoff = (uint32_t)(zero - in);
  const int r0 = mt * 16 + (lane & 15);
  const int r = r0 < 49 ? r0 : 48;  // rows >= 49: garbage, never stored
  const int jy = r / 7, jx = r - 7 * (r / 7);
  float cs = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = (w >> 2) + 2 * i;
    const int a = q >> 1, b = q & 1;
    bf16x8 av[8], bv[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {  // every fragment of the item first, then the MFMA chain
      const int ty = ks >> 2, tx = (ks >> 1) & 1, hh = ks & 1;
      const int iy = jy + a - ty, ix = jx + b - tx;
      const bool ok = (unsigned)iy < 7u && (unsigned)ix < 7u;
      const uint32_t off = ok ? (uint32_t)img49(iy * 7 + ix, 4 * hh + (lane >> 4)) : zoff;
      av[ks] = *reinterpret_cast<const bf16x8*>(in + off);
      const int tap = ((1 - a) + 2 * ty) * 4 + (1 - b) + 2 * tx;
      bv[ks] = tr_frag<32>(wimg + tap * 4096, 16 * nj, 32 * hh, lane);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) acc = mfma_bf16(av[ks], bv[ks], acc);
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r2 = mt * 16 + 4 * (lane >> 4) + rr;
      if (r2 < 49) {
        const int jy2 = r2 / 7, jx2 = r2 - 7 * (r2 / 7);
        s += epi((2 * jy2 + a) * 14 + 2 * jx2 + b, 16 * nj + (lane & 15), acc[rr], pv[i][rr]);
      }
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    cs += s;
  }
  return cs;
}

// P2 .. Q6 of one sample, role r (0/1) of its pair. LDS map: StepLayout (the
// solo merged step's), every region used for the same thing.
template <class L>
__device__ __forceinline__ void pair_rest(uint8_t* lds, int n, int r) {
  float* Xs = reinterpret_cast<float*>(lds + L::X);
  float* W4s = reinterpret_cast<float*>(lds + L::W4);
  uint8_t* A1s = lds + L::A1;
  __bf16* A2s = reinterpret_cast<__bf16*>(lds + L::A2);
  uint8_t* D0u = lds + L::D0;  // img49
  float* Hs = reinterpret_cast<float*>(lds + L::H);
  __bf16* Zs = reinterpret_cast<__bf16*>(lds + L::Z);
  float* Eps = reinterpret_cast<float*>(lds + L::Red);
  float* Scr = reinterpret_cast<float*>(lds + L::Scr);
  uint8_t* IMG = lds + L::IMG;
  __bf16* D1s = reinterpret_cast<__bf16*>(lds + L::D1);
  float* Gs = reinterpret_cast<float*>(lds + L::G);
  const float* Bds = reinterpret_cast<const float*>(lds + L::Bd);
  uint8_t* GD1s = lds + L::GD1;                                  // aliases Bd (dead after P5)
  __bf16* GD0s = reinterpret_cast<__bf16*>(lds + L::GD0);        // aliases the DMA landing zone
  float* DMs = reinterpret_cast<float*>(lds + L::DM);            // aliases X (dead after P7)
  float* DZR = reinterpret_cast<float*>(lds + L::DZR);
  uint8_t* GA2u = lds + L::GA2;                                  // img49, aliases D0 (dead after Q2)
  float* GA2F = reinterpret_cast<float*>(lds + L::GA2F);         // aliases D1 (dead after Q1)
  float* CS = reinterpret_cast<float*>(lds + L::CS);
  float* CSB = reinterpret_cast<float*>(lds + L::CSB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto TB = [&](int i) { return tab<L, __bf16>(lds, i); };
  auto TF = [&](int i) { return tab<L, float>(lds, i); };
  const unsigned long long ints = reinterpret_cast<const unsigned long long*>(lds + L::PTab)[kTInts];
  const int M = __builtin_amdgcn_readfirstlane((int)(ints & 0xffff));
  const bool train = ((ints >> 16) & 1) != 0;
  const uint32_t stream = __builtin_amdgcn_readfirstlane((uint32_t)(ints >> 32));
  auto pstamp = [&](int k) {
    if (tid == 0) {
      unsigned long long* st = tab<L, unsigned long long>(lds, kTStamp);
      if (st) st[k] = __builtin_amdgcn_s_memrealtime();
    }
  };
  const int p0 = r ? 24 : 0, p1 = r ? 49 : 24;  // own pixels of the 7x7 maps
  const int q0 = r ? 0 : 24, q1 = r ? 24 : 49;  // the partner's
  const int k0 = 64 * p0, klen = 64 * (p1 - p0);
  const uint32_t tg = (uint32_t)tab<L, const TrainState>(lds, kTSt)->step * 8u;  // tags tg+1 .. tg+6 (never 0)
  unsigned long long* xo = tab<L, unsigned long long>(lds, kTXg) + r * kXW;        // own slab (written)
  unsigned long long* xi = tab<L, unsigned long long>(lds, kTXg) + (r ^ 1) * kXW;  // partner's (read, cleared)
  unsigned* err = tab<L, unsigned>(lds, kTErr);
  const float* Bias = reinterpret_cast<const float*>(lds + L::Bias);
  const uint8_t* Zero = lds + L::Bias + 4 * kZero;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  if (tid == 0) xput(xo + kX1 + 64, tg + 1, xcc, false);  // X1 also carries this XCD's id

  pstamp(2);
  // P3's first two own-K weight rows per wave, in flight under P2
  auto ld_rows = [&](int c2, bf16x8 (&v)[8]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = w + 16 * c2 + 8 * h, k = 512 * i + 8 * lane;
        v[4 * h + i] = k < klen ? *reinterpret_cast<const bf16x8*>(TB(kTWh) + (size_t)o * kFlat + k0 + k) : zero8();
      }
  };
  bf16x8 wh0[8];
  ld_rows(0, wh0);
  // ---- P2: enc2 on own pixels, ReLU
  __bf16* const a2p = TB(kTA2);  // table reads hoisted above the epilogue's LDS stores (which may alias them)
  conv14to7_rows(A1s, Zero, p0, p1, [&](int j, int t) { return conv_bfrag(IMG, j, t, lane); },
                 [&](int, int col) { return Bias[kB2 + col]; }, [&](int p, int col, float v, float bias) {
    const __bf16 o = (__bf16)fmaxf(v + bias, 0.f);
    A2s[p * 64 + col] = o;
    if (train) a2p[p * 64 + col] = o;
  });
  lds_barrier();

  pstamp(3);
  // ---- P3: head partial sums over own K (= own pixels). Wave w: rows
  // w + 16 c2 + 8 h (c2 < 4, h < 2). All eight rows' loads are in flight at
  // once (the first two since P2): the phase is L2-latency bound, so one
  // round trip instead of four.
  {
    bf16x8 av[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 512 * i + 8 * lane;
      av[i] = k < klen ? *reinterpret_cast<const bf16x8*>(A2s + k0 + k) : zero8();
    }
    bf16x8 wr[4][8];
#pragma unroll
    for (int i = 0; i < 8; ++i) wr[0][i] = wh0[i];
    ld_rows(1, wr[1]);
#ifdef MDT_F28_HALFW_EXP  // timing experiment only (wrong results): half the P3 / Q5 weight bytes
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      wr[2][i] = wr[0][i];
      wr[3][i] = wr[1][i];
    }
#else
    ld_rows(2, wr[2]);
    ld_rows(3, wr[3]);
#endif
    float d[8];
#pragma unroll
    for (int c2 = 0; c2 < 4; ++c2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float dq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x8& wv = wr[c2][4 * h + i];
          if (512 * i + 8 * lane < klen) {
            dq[0] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 0, 1),
                                                    __builtin_shufflevector(wv, wv, 0, 1), dq[0], false);
            dq[1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 2, 3),
                                                    __builtin_shufflevector(wv, wv, 2, 3), dq[1], false);
            dq[2] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 4, 5),
                                                    __builtin_shufflevector(wv, wv, 4, 5), dq[2], false);
            dq[3] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 6, 7),
                                                    __builtin_shufflevector(wv, wv, 6, 7), dq[3], false);
          }
        }
        d[2 * c2 + h] = (dq[0] + dq[1]) + (dq[2] + dq[3]);
      }
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = wave_sum(d[i]);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int o = w + 16 * (i >> 1) + 8 * (i & 1);
        Hs[o] = d[i];
        xput(xo + kX1 + o, tg + 1, fbits(d[i]), false);
      }
    }
  }
  TapImageRegs w3r;
  w3r.load(TB(kTW3));  // dec1 tap images: in flight during P4-P5
  // P5's first dec_fc weight loads (own n-tiles t = 4 p0 + w + 8 i), in flight across P4
  const int t0 = 4 * p0, t1 = 4 * p1;
  const __bf16* wp5 = TB(kTWd) + (size_t)(lane & 15) * 32 + 8 * (lane >> 4);
  auto wd5_ld = [&](int i) {
    const int t = t0 + w + 8 * i;
    return *reinterpret_cast<const bf16x8*>(wp5 + (size_t)(t < t1 ? t : t0) * 512);
  };
  bf16x8 wd5[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) wd5[i] = wd5_ld(i);
  lds_barrier();

  pstamp(4);
  // ---- X1 + P4: mu | logvar = (role-0 part + role-1 part) + bias; reparam + KLD (both halves)
  if (tid < 64) {
    float kl = 0.f;
    if (tid < 32) {
      const int c = tid;
      // eps first: it needs nothing from the partner, so it overlaps the X1 wait
      const unsigned long long stp = (unsigned long long)tab<L, const TrainState>(lds, kTSt)->step;
      const HParams* hp = tab<L, const HParams>(lds, kTHp);
      const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(n * 32 + c), stream, (uint32_t)(stp & 0xffffffffu),
                                             (uint32_t)(stp >> 32)},
                                       hp->seed_lo, hp->seed_hi);
      const float ep = normal_from_bits(bits.x, bits.y);
      const int gi[2] = {kX1 + c, kX1 + 32 + c};
      uint32_t pv[2];
      xget<2>(xi, gi, tg + 1, pv, err, false);
      const float m0 = Hs[c], l0 = Hs[32 + c], mp = bitsf(pv[0]), lp = bitsf(pv[1]);
      const float mu = (r ? mp + m0 : m0 + mp) + Bias[kBh + c];
      const float lv = (r ? lp + l0 : l0 + lp) + Bias[kBh + 32 + c];
      Hs[c] = mu;
      Hs[32 + c] = lv;
      const float sd = expf(0.5f * lv);
      const float zz = fmaf(ep, sd, mu);
      kl = fmaf(-sd, sd, fmaf(-mu, mu, 1.f + lv));  // explicit: one rounding sequence in both bodies
      Zs[c] = (__bf16)zz;
      Eps[c] = ep;
      if (train && r == 0) {
        TF(kTMulv)[c] = mu;
        TF(kTMulv)[32 + c] = lv;
        TF(kTEps)[c] = ep;
        TB(kTZ16)[c] = (__bf16)zz;
      }
    }
    if (tid == 32) {
      const int gi[1] = {kX1 + 64};
      uint32_t pv[1];
      xget<1>(xi, gi, tg + 1, pv, err, false);
      reinterpret_cast<int*>(Scr)[30] = pv[0] == xcc;
    }
    kl = wave_sum(kl);
    if (tid == 0) Scr[0] = -0.5f * kl;
  }
  lds_barrier();
  const bool near = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(Scr)[30]) != 0;
  if (tid == 0) {  // slot 15: mode | near << 4
    unsigned long long* st = tab<L, unsigned long long>(lds, kTStamp);
    if (st) st[15] |= (unsigned long long)near << 4;
  }

  pstamp(5);
  // ---- P5: dec_fc on own pixels (n-tiles [t0, t1)), ReLU; X2 publishes them
  {
    __bf16* const d0p = TB(kTD0);
    const bf16x8 av = (lane & 15) == 0 ? *reinterpret_cast<const bf16x8*>(Zs + 8 * (lane >> 4)) : zero8();
    stream2_pre<13, 1>(wd5, wd5_ld, [&](int i, const bf16x8& bw) {
      const int t = t0 + w + 8 * i;
      if (t < t1) {
        const f32x4 acc = mfma_bf16(av, bw, f32x4{0.f, 0.f, 0.f, 0.f});
        const int jj = 16 * t + (lane & 15);
        const __bf16 o = (__bf16)fmaxf(acc[0] + Bds[jj], 0.f);
        const uint32_t ob = bf16bits(o), nb = (uint32_t)__shfl_xor((int)ob, 1, 64);
        if (lane < 16) {
          *reinterpret_cast<__bf16*>(D0u + img49e(jj >> 6, jj & 63)) = o;
          if (train) d0p[jj] = o;
          if ((lane & 1) == 0) xput(xo + kX2 + ((jj - k0) >> 1), tg + 2, ob | (nb << 16), near);
        }
      }
    });
  }
  w3r.store(IMG);
  {  // X2: the partner's d0 pixels into the img49 image
    const int cnt = 32 * (q1 - q0);
    const int gi[2] = {tid < cnt ? kX2 + tid : -1, tid + 512 < cnt ? kX2 + tid + 512 : -1};
    uint32_t pv[2];
    xget<2>(xi, gi, tg + 2, pv, err, near);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (gi[k] >= 0) {
        const int jj = 64 * q0 + 2 * (gi[k] - kX2);
        *reinterpret_cast<uint32_t*>(D0u + img49e(jj >> 6, jj & 63)) = pv[k];
      }
    }
  }
  lds_barrier();

  pstamp(6);
  // ---- P6: dec1 (convT 64 -> 32) on own channels [16 r, 16 r + 16), ReLU
  __bf16* const d1p = TB(kTD1);
  tconv7to14_half(D0u, Zero, IMG, r, [&](int, int co) { return Bias[kB3 + co]; }, [&](int pix, int co, float v, float bias) {
    const __bf16 o = (__bf16)fmaxf(v + bias, 0.f);
    D1s[pix * 32 + co] = o;
    if (train) d1p[pix * 32 + co] = o;
    return 0.f;
  });
  lds_barrier();

  pstamp(7);
  // ---- P7: dec2 partial logits over own channels, X3, then BCE + dlogits (both)
  float loss = 0.f, gsum = 0.f;
  {
    float* const dlp = TF(kTDlog);
    float* const rcp = TF(kTRecon);
    float tp[2] = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pix = tid + 512 * k;
      if (pix < 784) {
        const int oy = pix / 28, ox = pix - 28 * (pix / 28);
        const int ca = oy & 1, cb = ox & 1, jy = oy >> 1, jx = ox >> 1;
        float t = 0.f;
#pragma unroll
        for (int ty = 0; ty < 2; ++ty)
#pragma unroll
          for (int tx = 0; tx < 2; ++tx) {
            const int iy = jy + ca - ty, ix = jx + cb - tx;
            if ((unsigned)iy < 14u && (unsigned)ix < 14u) {
              const int tap = ((1 - ca) + 2 * ty) * 4 + (1 - cb) + 2 * tx;
              const bf16x8* dp = reinterpret_cast<const bf16x8*>(D1s + (iy * 14 + ix) * 32 + 16 * r);
              const float4* wp = reinterpret_cast<const float4*>(W4s + tap * 32 + 16 * r);
#pragma unroll
              for (int ch = 0; ch < 2; ++ch) {
                const bf16x8 dv = dp[ch];
                const float4 w0 = wp[2 * ch], w1 = wp[2 * ch + 1];
                t = fmaf((float)dv[0], w0.x, t); t = fmaf((float)dv[1], w0.y, t);
                t = fmaf((float)dv[2], w0.z, t); t = fmaf((float)dv[3], w0.w, t);
                t = fmaf((float)dv[4], w1.x, t); t = fmaf((float)dv[5], w1.y, t);
                t = fmaf((float)dv[6], w1.z, t); t = fmaf((float)dv[7], w1.w, t);
              }
            }
          }
        tp[k] = t;
        xput(xo + kX3 + pix, tg + 3, fbits(t), near);
      }
    }
    const int gi[2] = {tid < 784 ? kX3 + tid : -1, tid + 512 < 784 ? kX3 + tid + 512 : -1};
    uint32_t pv[2];
    xget<2>(xi, gi, tg + 3, pv, err, near);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int pix = tid + 512 * k;
      if (pix < 784) {
        const float pp = bitsf(pv[k]);
        const float t = Bias[kB4] + (r ? pp + tp[k] : tp[k] + pp);
        const float x = Xs[pix];
        const float p = 1.f / (1.f + expf(-t));
        const float g = p - x;
        const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
        loss += fmaf(x, fminf(sp_pos - t, 100.f), (1.f - x) * fminf(sp_pos, 100.f));  // explicit fma (see kl)
        gsum += g;
        Gs[pix] = g;
        if (train && (pix >= 392) == (r == 1)) dlp[pix] = g;
        if (rcp && (pix >= 392) == (r == 1)) rcp[pix] = p;
      }
    }
  }
  loss = wave_sum(loss);
  gsum = wave_sum(gsum);
  if (lane == 0) {
    Scr[8 + w] = loss;
    Scr[16 + w] = gsum;
  }
  lds_barrier();
  if (tid == 0 && r == 0) {
    float sl = 0.f, sg = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sl += Scr[8 + i];
      sg += Scr[16 + i];
    }
    TF(kTBce)[0] = sl;
    TF(kTKld)[0] = Scr[0];
    if (float* d4 = TF(kTDb4)) d4[0] = sg;
  }
  // eval (forward only): both halves end here; X1-X3 are consumed (cleared),
  // X4-X6 never written, so the granules are zero for the next launch
  if (!train) return;

  pstamp(8);
  // ---- Q1: dec2 backward-data on own channels x dec1 ReLU mask; X4 publishes gd1.
  // Exact-f32 MFMA (v_mfma_f32_16x16x4_f32, as enc1 in P1): D[own channel]
  // [pixel] = W4[channel][tap] x im2col(dlogits)[tap][pixel], 13 pixel tiles x
  // 4 tap steps, wave w takes pixel tiles w and w + 8; a lane ends with four
  // consecutive own channels of one pixel.
  __bf16* const gd1p = TB(kTGd1);
  {
    const int col = lane & 15, kq = lane >> 4;
    float wa[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) wa[ks] = W4s[(4 * ks + kq) * 32 + 16 * r + col];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 8 * j;
      if (nt < 13) {
        const int pix = 16 * nt + col;
        const bool live = pix < 196;
        const int oy = pix / 14, ox = pix - 14 * (pix / 14);
        float gb[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int t = 4 * ks + kq;
          const int iy = 2 * oy - 1 + (t >> 2), ix = 2 * ox - 1 + (t & 3);
          gb[ks] = live && (unsigned)iy < 28u && (unsigned)ix < 28u ? Gs[iy * 28 + ix] : 0.f;
        }
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma16x16x4(wa[ks], gb[ks], acc);
        if (live) {
          const int cl = 4 * kq, c0 = 16 * r + cl;  // own-local / global first channel of the four
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
          const bf16x4 m = *reinterpret_cast<const bf16x4*>(lds + L::D1 + pix * 64 + c0 * 2);
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = (float)m[e] > 0.f ? acc[e] : 0.f;
            o[e] = (__bf16)v;
            CSB[(cl + e) * 197 + pix] = v;  // dec1 bias partials (own channel cl + e)
          }
          *reinterpret_cast<bf16x4*>(GD1s + img14(pix, c0 >> 3) + ((c0 & 7) << 1)) = o;
          *reinterpret_cast<bf16x4*>(gd1p + pix * 32 + c0) = o;
          // granule layout [4][392] (unchanged): channel pair (e, e + 1) of own
          // chunk h at [(e >> 1)][2 pix + h]
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int c = cl + 2 * q, h = c >> 3, e = c & 7;
            xput(xo + kX4 + (e >> 1) * 392 + 2 * pix + h, tg + 4,
                 bf16bits(o[2 * q]) | (bf16bits(o[2 * q + 1]) << 16), near);
          }
        }
      }
    }
  }
  // Q3's first dec_fc weight loads (own rows), in flight during X4 and Q2
  const int jr = lane >> 2;
  auto wd_ld = [&](int it) {
    const int jj = k0 + it * 128 + w * 16 + jr;
    return *reinterpret_cast<const bf16x8*>(TB(kTWd) + (size_t)(jj < k0 + klen ? jj : k0) * 32 + 8 * (lane & 3));
  };
  bf16x8 wd0[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) wd0[i] = wd_ld(i);
  lds_barrier();
  if (tid < 128) {  // dec1 bias partials of own channels: 8 lanes per channel, fixed order
    const int c = tid >> 3, part = tid & 7;
    float s = 0.f;
    for (int p = part; p < 196; p += 8) s += CSB[c * 197 + p];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (part == 0) TF(kTDb3)[16 * r + c] = s;
  }
  {  // X4: the partner's gd1 channels into the img14 image
    int gi[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) gi[k] = tid + 512 * k < 1568 ? kX4 + tid + 512 * k : -1;
    uint32_t pv[4];
    xget<4>(xi, gi, tg + 4, pv, err, near);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (gi[k] >= 0) {
        const int g = gi[k] - kX4, e2 = g / 392, t = g - 392 * e2;
        const int pix = t >> 1, ch = 16 * (r ^ 1) + 8 * (t & 1) + 2 * e2;
        *reinterpret_cast<uint32_t*>(GD1s + img14(pix, ch >> 3) + ((ch & 7) << 1)) = pv[k];
      }
    }
  }
  lds_barrier();

  pstamp(9);
  // ---- Q2: dec1 backward-data (conv 32 -> 64, B from dec1's tap images) on own pixels x dec_fc mask
  __bf16* const gd0p = TB(kTGd0);
  float* const dbdp = TF(kTDbd);
  conv14to7_rows(GD1s, Zero, p0, p1,
                 [&](int j, int t) {
                   return *reinterpret_cast<const bf16x8*>(IMG + t * 4096 + timg<32>(16 * j + (lane & 15), lane >> 4));
                 },
                 [&](int p, int col) { return (float)*reinterpret_cast<const __bf16*>(D0u + img49e(p, col)); },
                 [&](int p, int col, float v, float mask) {
    const int e = p * 64 + col;
    const float g = mask > 0.f ? v : 0.f;
    const __bf16 o = (__bf16)g;
    GD0s[p * 64 + col] = o;
    gd0p[e] = o;
    dbdp[e] = g;
  });
  lds_barrier();

  TapImageRegs w2r;  // enc2 tap images (loaded in Q5, written before Q6)
  pstamp(10);
  // ---- Q3: dz partial over own dec_fc rows
  {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    stream2_pre<13, 1>(wd0, wd_ld, [&](int it, const bf16x8& wv) {
      const int jj = k0 + it * 128 + w * 16 + jr;
      if (jj < k0 + klen) {
        const float g = (float)GD0s[jj];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(g, (float)wv[e], acc[e]);
      }
    });
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[e];
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      acc[e] = v;
    }
    if (lane < 4) {
#pragma unroll
      for (int e = 0; e < 8; ++e) DZR[w * 32 + 8 * lane + e] = acc[e];
    }
  }
  // Q5's first 16 head-weight loads: row group grp = tid >> 8 (rows 32 grp ..), own 8-chunk ck
  const int nck = klen >> 3, grp = tid >> 8, ck = tid & 255;
  const int kk = k0 + 8 * (ck < nck ? ck : 0);
  auto wh_ld = [&](int i) { return *reinterpret_cast<const bf16x8*>(TB(kTWh) + (size_t)(32 * grp + i) * kFlat + kk); };
  bf16x8 wh5[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) wh5[i] = wh_ld(i);
  lds_barrier();

  pstamp(11);
  // ---- X5 + Q4: dz = role-0 part + role-1 part; reparam backward (both halves)
  if (tid < 32) {
    const int c = tid;
    float mine = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) mine += DZR[i * 32 + c];
    xput(xo + kX5 + c, tg + 5, fbits(mine), near);
    const int gi[1] = {kX5 + c};
    uint32_t pv[1];
    xget<1>(xi, gi, tg + 5, pv, err, near);
    const float dz = r ? bitsf(pv[0]) + mine : mine + bitsf(pv[0]);
    const float beta = tab<L, const HParams>(lds, kTHp)->kl_beta;
    const float mu = Hs[c], lv = Hs[32 + c], ep = Eps[c];
    const float sd = expf(0.5f * lv);
    const float dm = dz + beta * mu;
    const float dl = 0.5f * dz * ep * sd + 0.5f * beta * (sd * sd - 1.f);
    DMs[c] = dm;
    DMs[32 + c] = dl;
    if (r == 0) {
      TF(kTDmulv)[c] = dm;
      TF(kTDmulv)[32 + c] = dl;
      TB(kTDmulv16)[c] = (__bf16)dm;
      TB(kTDmulv16)[32 + c] = (__bf16)dl;
    }
  }
  lds_barrier();

  pstamp(12);
  // ---- Q5: head backward-data on own K: two row groups of 32 per 8-chunk, combined in a fixed order
  {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    bf16x8 wh6[16];  // rows 16..31 of the group: with wh5, all 32 in flight at once
#ifdef MDT_F28_HALFW_EXP
#pragma unroll
    for (int i = 0; i < 16; ++i) wh6[i] = wh5[i];
#else
#pragma unroll
    for (int i = 0; i < 16; ++i) wh6[i] = wh_ld(16 + i);
#endif
    w2r.load(TB(kTW2));  // enc2 tap images: in flight during Q5
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const bf16x8& wv = i < 16 ? wh5[i] : wh6[i - 16];
      const float dm = DMs[32 * grp + i];
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaf(dm, (float)wv[e], acc[e]);
    }
    if (grp == 1 && ck < nck) {
#pragma unroll
      for (int e = 0; e < 8; ++e) CSB[ck * 8 + e] = acc[e];
    }
    lds_barrier();
    __bf16* const ga2p = TB(kTGa2);
    if (grp == 0 && ck < nck) {
      const bf16x8 mk = *reinterpret_cast<const bf16x8*>(A2s + kk);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v0 = acc[e] + CSB[ck * 8 + e];
        const float v = (float)mk[e] > 0.f ? v0 : 0.f;
        o[e] = (__bf16)v;
        GA2F[kk + e] = v;
      }
      *reinterpret_cast<bf16x8*>(GA2u + img49(kk >> 6, (kk >> 3) & 7)) = o;
      *reinterpret_cast<bf16x8*>(ga2p + kk) = o;
#pragma unroll
      for (int e = 0; e < 8; e += 2)  // granule layout [4][200] (8-chunk ck of the own range)
        xput(xo + kX6 + (e >> 1) * 200 + ck, tg + 6, bf16bits(o[e]) | (bf16bits(o[e + 1]) << 16), near);
    }
  }
  w2r.store(IMG);
  {  // X6: the partner's ga2 pixels into the img49 image
    const int nckp = 8 * (q1 - q0);  // the partner's 8-chunks
    int gi[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int g = tid + 512 * k, e2 = g / 200, c = g - 200 * e2;
      gi[k] = g < 800 && c < nckp ? kX6 + g : -1;
    }
    uint32_t pv[2];
    xget<2>(xi, gi, tg + 6, pv, err, near);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (gi[k] >= 0) {
        const int g = gi[k] - kX6, e2 = g / 200, c = g - 200 * e2;
        const int jj = 64 * q0 + 8 * c + 2 * e2;
        *reinterpret_cast<uint32_t*>(GA2u + img49e(jj >> 6, jj & 63)) = pv[k];
      }
    }
  }
  lds_barrier();
  if (tid < 64) {  // enc2 bias partials over own pixels, in order: row r of [2][M][64]
    float s = 0.f;
    for (int p = p0; p < p1; ++p) s += GA2F[p * 64 + tid];
    TF(kTDb2)[(size_t)r * M * 64 + tid] = s;
  }

  pstamp(13);
  // ---- Q6: enc2 backward-data (convT 64 -> 32 with the conv weights) on own channels x enc1 mask
  {
    __bf16* const ga1p = TB(kTGa1);
    const float cs = tconv7to14_half(GA2u, Zero, IMG, r,
                                     [&](int pix, int co) {
                                       return (float)*reinterpret_cast<const __bf16*>(A1s + img14(pix, co >> 3) +
                                                                                      ((co & 7) << 1));
                                     },
                                     [&](int pix, int co, float v, float mask) {
      const float g = mask > 0.f ? v : 0.f;
      ga1p[pix * 32 + co] = (__bf16)g;
      return g;
    });
    if (lane < 16) CS[w * 16 + lane] = cs;
  }
  lds_barrier();
  if (tid < 16) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += CS[i * 16 + tid];
    TF(kTDb1)[16 * r + tid] = s;
  }
  pstamp(14);
}

}  // namespace f28
}  // namespace mdt
