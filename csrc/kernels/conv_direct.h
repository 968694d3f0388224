// Patch-resident direct convolution GEMMs for the stride-2, 4x4, pad-1
// layers of the 128x128 conv-VAE on CDNA4 (gfx950).
//
// Why not the im2col implicit GEMM (conv_igemm_dev.h) for these layers: every
// input pixel of a stride-2 4x4 conv is read by 4 output pixels, so the
// im2col A stream is 4x the activation, gathered through the TA in 64-128 B
// pieces, and one k-tile in flight per block left those kernels at 6-10 %
// MFMA busy (profiles/r1_pmc/conv128_pmc.md). Here a workgroup owns
//   conv  (MODE 0): image n, R output rows x all OW columns, NB output channels
//   tconv (MODE 1): image n, R rows of the low-resolution grid, all four
//                   stride-parity classes (the 2x2 taps that reach each output
//                   parity), NB output channels
// and keeps the input halo patch those need -- (2R+2 or R+2) rows x (W+2)
// columns x all input channels, zero padding materialised -- resident in LDS
// for the whole k loop: the activation is fetched once per tile (plus the
// 2-row halo), as whole contiguous NHWC rows, by LDS-DMA (global_load_lds,
// 16 B per lane, no staging registers). The weight operand streams through an
// S-stage LDS-DMA ring of 64-deep k stages while the patch is multiplied.
//
// MFMA: v_mfma_f32_32x32x16_bf16 (half the LDS operand bytes per MAC of the
// 16x16x32 form). A fragment = 32 consecutive tile pixels x 16 channels of one
// tap, read straight out of the patch (ds_read_b128); B fragment = 32 output
// channels x 16 k from the ring. Conv mode stores each patch row with its even
// and odd columns split, so the stride-2 pixels of one tap are consecutive
// slots. Every patch pixel's 16-B chunks are XOR-swizzled by
// ((x + AL*y) >> BE) & MK of its slot (x, y); the per-configuration constants
// were searched so that every tap's fragment read is conflict-free under the
// ds_read_b128 lane grouping (4 LDS cycles per wave-instruction).
//
// Epilogue (same semantics as igemm_epilogue): bias, ReLU, the ReLU-backward
// mask of the produced gradient, bf16/f32 stores and one row of per-workgroup
// column sums (the next layer's bias-gradient partials, fixed order). The bf16
// activation leaves through write-through (sc1) stores: plain ones sat dirty in
// L2 until the end-of-kernel write-back, a tail nothing overlapped.
#pragma once

#include "conv_igemm_dev.h"

namespace mdt {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

struct DcArgs {
  const __bf16* A;      // NHWC [nimg][WA][WA][CA]
  const __bf16* B;      // [classes][NCOLS][K], K = taps x CA (k = (tap, ci))
  __bf16* y16;          // output NHWC, or null
  float* y32;           // output NHWC f32, or null
  const float* bias;    // [NCOLS] or null
  const __bf16* omask;  // output-shaped: zero where the value is dropped, or null
  float* colsum;        // [nimg * RB][NCOLS] column-sum partials, or null
  unsigned long long* stamps;  // optional [grid][8] s_memrealtime (profiling)
  int relu;
  int nimg;
};

// KS_ = 2: two groups of four waves split every weight stage's k-steps (group
// g multiplies k-steps 2g and 2g + 1 of each 64-deep stage; group 1's
// accumulators are added into group 0's before the epilogue). For the
// deep-K layers with one output tile per CU: two waves per SIMD, so one
// wave's LDS fragment latency hides behind the other's MFMAs.
// HS_: weight stages per ring hand-off (wait + barrier + refill): 2 halves the
// hand-offs and doubles the MFMAs between them (needs S >= 2 HS).
template <int MODE_, int CA_, int WA_, int NCOLS_, int NB_, int R_, int WM_, int S_, int AL_, int BE_, int MK_,
          int KS_ = 1, int HS_ = 1>
struct DcCfg {
  static constexpr int MODE = MODE_, CA = CA_, WA = WA_, NCOLS = NCOLS_, NB = NB_, R = R_, S = S_;
  static constexpr int AL = AL_, BE = BE_, MK = MK_;
  static constexpr int KS = KS_, HS = HS_, WAVES = 4 * KS_, THREADS = 64 * WAVES;
  static constexpr bool CONV = MODE == 0;
  static constexpr int OW = CONV ? WA / 2 : WA;      // tile row width (output / class-grid pixels)
  static constexpr int OH = OW;
  static constexpr int MT = R * OW;                  // pixels per tile (per class in tconv mode)
  static constexpr int PR = CONV ? 2 * R + 2 : R + 2;
  static constexpr int PC = WA + 2;
  static constexpr int P = 2 * CA;                   // bytes per patch pixel
  static constexpr int NCH = CA / 8;                 // 16-B chunks per patch pixel
  static constexpr int PATCH = PR * PC * P;
  static constexpr int NPI = (PATCH + 1023) / 1024;  // 1-KB DMA instructions
  static constexpr int NPW = (NPI + WAVES - 1) / WAVES;
  static constexpr int PATCH_LDS = NPW * WAVES * 1024;
  static constexpr int K = CONV ? 16 * CA : 4 * CA;  // per class
  static constexpr int NSTAGE = K / 64;
  static constexpr int BROWS = CONV ? NB : 4 * NB;
  static constexpr int STAGE = BROWS * 128;
  static constexpr int NBI = BROWS / 8;              // DMA instructions per stage
  static constexpr int NBW = NBI / WAVES;
  static constexpr int WM = CONV ? WM_ : 1;
  static constexpr int WN = CONV ? 4 / WM_ : 1;  // per k-group of four waves
  static constexpr int TM = CONV ? MT / WM : MT;     // wave tile
  static constexpr int TN = CONV ? NB / WN : NB;
  static constexpr int FM = TM / 32, FN = TN / 32;
  static constexpr int RB = OH / R;                  // row blocks per image
  static constexpr int NBB = NCOLS / NB;             // column blocks
  static constexpr int CS_OFF = PATCH_LDS + S * STAGE;
  static constexpr int LDS = CS_OFF + WAVES * TN * 4;
  // epilogue staging: per wave one 32-row slice of its tile, f32, rows padded
  // to TN + 8 floats (the fragment-order writes of a half-wave pair land on
  // disjoint banks)
  static constexpr int SPITCH = TN + 8;
  static constexpr int STG = 32 * SPITCH * 4;
  static_assert(WAVES * STG <= CS_OFF, "dconv epilogue staging");
  static_assert(CA % 16 == 0 && NBI % WAVES == 0 && FM >= 1 && FN >= 1, "dconv tile");
  static_assert(TM % 32 == 0 && TN % 32 == 0 && OH % R == 0 && NCOLS % NB == 0, "dconv tile");
  static_assert(K % 64 == 0 && S >= 2 * HS && NSTAGE >= S && NSTAGE % HS == 0 && NBW * (S - 1) <= 63,
                "dconv pipeline");
  static_assert(MK < NCH && LDS <= 160 * 1024, "dconv LDS");
  static_assert(KS == 1 || (KS == 2 && 4 * STG + 4 * FM * FN * 64 * 64 <= CS_OFF), "dconv k-group exchange");
};

// vmcnt wait leaving `n` (<= MAXN) newer DMA stages of NBW instructions in flight.
template <int NBW, int MAXN>
__device__ __forceinline__ void dc_wait_stages(int n) {
  if constexpr (MAXN > 0) {
    if (n >= MAXN) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MAXN * NBW) : "memory");
      return;
    }
    dc_wait_stages<NBW, MAXN - 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__device__ __forceinline__ void dc_stamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0) st[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

template <class CF>
__device__ __forceinline__ int dc_swz(int y, int x) {
  return ((x + CF::AL * y) >> CF::BE) & CF::MK;
}

// Workgroup body; `tile` is the (XCD-remapped) tile index.
template <class CF>
__device__ __forceinline__ void dconv_body(const DcArgs& a, uint8_t* lds, int tile) {
  constexpr int WA = CF::WA, CA = CF::CA, OW = CF::OW, PC = CF::PC, P = CF::P, K = CF::K;
  constexpr int FM = CF::FM, FN = CF::FN, S = CF::S, NSTAGE = CF::NSTAGE, NBW = CF::NBW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = tile % CF::NBB;
  const int t2 = tile / CF::NBB;
  const int rb = t2 % CF::RB, n = t2 / CF::RB;
  const int r0 = rb * CF::R;  // first output row (conv) / class-grid row (tconv)
  dc_stamp(a.stamps, 0);

  uint8_t* patch = lds;
  uint8_t* ring = lds + CF::PATCH_LDS;
  const __bf16* An = a.A + (size_t)n * WA * WA * CA;

  // ---- patch: NPW 1-KB LDS-DMA instructions per wave (pad slots read zeros)
#pragma unroll 1
  for (int i = 0; i < CF::NPW; ++i) {
    const int j = i * CF::WAVES + w;
    const int pos = j * 1024 + 16 * lane;
    const int pix = pos / P;
    const int pc = (pos % P) >> 4;
    const int y = pix / PC, x = pix - (pix / PC) * PC;
    const int c = pc ^ dc_swz<CF>(y, x);
    int iy, ix;
    if constexpr (CF::CONV) {
      iy = 2 * r0 - 1 + y;
      ix = (x <= OW ? 2 * x : 2 * (x - OW - 1) + 1) - 1;
    } else {
      iy = r0 - 1 + y;
      ix = x - 1;
    }
    const bool ok = pix < CF::PR * PC && (unsigned)iy < (unsigned)WA && (unsigned)ix < (unsigned)WA;
    glds16(ok ? (const void*)(An + ((size_t)iy * WA + ix) * CA + 8 * c) : (const void*)g_zero16, patch + j * 1024);
  }
  // ---- weight ring: stage st = k range [64 st, 64 st + 64) of BROWS rows
  auto issue_stage = [&](int st) {
    uint8_t* dst = ring + (st % S) * CF::STAGE;
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int j = i * CF::WAVES + w;
      const int pos = j * 1024 + 16 * lane;
      const int r = pos >> 7;
      const int c = ((pos >> 4) & 7) ^ ((r >> 1) & 7);
      size_t row;
      if constexpr (CF::CONV) row = (size_t)nb * CF::NB + r;
      else row = (size_t)(r / CF::NB) * CF::NCOLS + nb * CF::NB + (r % CF::NB);
      glds16(a.B + row * K + 64 * st + 8 * c, dst + j * 1024);
    }
  };
#pragma unroll
  for (int s = 0; s < S; ++s) issue_stage(s);  // the whole ring in flight

  // ---- per-lane fragment coordinates (wl: wave within its k-group, kg0: the group's first k-step)
  const int wl = w & 3, kg0 = CF::KS == 2 ? 2 * (w >> 2) : 0;
  const int wm = CF::CONV ? wl / CF::WN : 0, wn = CF::CONV ? wl % CF::WN : 0;
  const int cls = CF::CONV ? 0 : wl;
  int ea = 0, eb = 0, oa = 0, ob = 0;
  if constexpr (!CF::CONV) {
    // class (ca, cb): output parity (oa, ob); taps (t0, t1) read A rows a + ea - t0
    const int ca = cls >> 1, cb = cls & 1;
    oa = (ca + 1) & 1;
    ob = (cb + 1) & 1;
    ea = (oa + 1 - ca) >> 1;
    eb = (ob + 1 - cb) >> 1;
  }
  int py[FM], px[FM];  // patch row / slot of tap (0, 0) (conv) or of (t0, t1) = (0, 0) (tconv)
#pragma unroll
  for (int fm = 0; fm < FM; ++fm) {
    const int q = wm * CF::TM + 32 * fm + (lane & 31);
    const int rr = q / OW, cc = q % OW;
    if constexpr (CF::CONV) {
      py[fm] = 2 * rr;
      px[fm] = cc;
    } else {
      py[fm] = rr + 1 + ea;
      px[fm] = cc + 1 + eb;
    }
  }
  const int half = lane >> 5;
  int brow[FN], bsw[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) {
    const int r = (CF::CONV ? wn * CF::TN : cls * CF::NB) + 32 * fn + (lane & 31);
    brow[fn] = r * 128;
    bsw[fn] = half ^ ((r >> 1) & 7);
  }

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // fragment loads of (stage, kk) from the patch and the ring slot
  auto load_frags = [&](int st, int kk, bf16x8(&af)[FM], bf16x8(&bfr)[FN]) {
    const int kg = 64 * st + 16 * kk;
    const int tap = kg / CA;
    const int ci8 = (kg % CA) >> 3;  // even
    int dy, dx;
    if constexpr (CF::CONV) {
      const int ky = tap >> 2, kx = tap & 3;
      dy = ky;
      dx = (kx & 1) ? OW + 1 + (kx >> 1) : (kx >> 1);
    } else {
      dy = -(tap >> 1);
      dx = -(tap & 1);
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      const int y = py[fm] + dy, x = px[fm] + dx;
      const int c = (ci8 | half) ^ dc_swz<CF>(y, x);
      af[fm] = *reinterpret_cast<const bf16x8*>(patch + (y * PC + x) * P + 16 * c);
    }
    const uint8_t* Bs = ring + (st % S) * CF::STAGE;
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) bfr[fn] = *reinterpret_cast<const bf16x8*>(Bs + brow[fn] + 16 * (bsw[fn] ^ (2 * kk)));
  };
  auto mma = [&](const bf16x8(&af)[FM], const bf16x8(&bfr)[FN]) {
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = mfma32(af[fm], bfr[fn], acc[fm][fn]);
  };

  dc_wait_stages<NBW, S - 1>(S - CF::HS);  // the patch and stages 0 .. HS-1 have landed (this wave's part)
  stage_barrier();
  dc_stamp(a.stamps, 1);

#ifdef MDT_DC_STAGE_STAMPS  // per-stage timeline of the workgroup-leader wave (bench/dconv_stage_stamps.py)
#define DC_SS(k)                                                                                          \
  if (a.stamps && threadIdx.x == 0)                                                                        \
    a.stamps[(size_t)gridDim.x * 8 + ((size_t)blockIdx.x * NSTAGE + st) * 4 + (k)] = __builtin_amdgcn_s_memrealtime();
#else
#define DC_SS(k)
#endif
#ifndef MDT_DC_STEP_AHEAD
  // Fragments of a whole hand-off group (HS stages) are loaded one group
  // ahead: each wave holds its NF = HS x KPW k-steps of group g in registers
  // (set `cur`) while it reads those of group g + 1 (set `nxt`). Per group:
  // the first half of cur's MFMAs, then the ring hand-off (wait for group
  // g + 1, barrier, refill group g's slots with stages + S: every wave's reads
  // of group g completed at the previous hand-off), then nxt's LDS reads, then
  // cur's second half, under which their latency hides. sched_barrier(0) pins
  // the order.
  constexpr int HS = CF::HS, KPW = 4 / CF::KS, NF = HS * KPW, KH = NF / 2, NG = NSTAGE / HS;
  bf16x8 fa0[NF][FM], fb0[NF][FN], fa1[NF][FM], fb1[NF][FN];
  auto load_group = [&](int g, bf16x8(&fa)[NF][FM], bf16x8(&fb)[NF][FN]) {
#pragma unroll
    for (int h = 0; h < HS; ++h)
#pragma unroll
      for (int i = 0; i < KPW; ++i) load_frags(g * HS + h, kg0 + i, fa[h * KPW + i], fb[h * KPW + i]);
  };
  auto step = [&](int g, const bf16x8(&ca)[NF][FM], const bf16x8(&cb)[NF][FN], bf16x8(&na)[NF][FM],
                  bf16x8(&nb_)[NF][FN]) {
    const int st = g * HS;
    DC_SS(0);
#pragma unroll
    for (int i = 0; i < KH; ++i) mma(ca[i], cb[i]);
    __builtin_amdgcn_sched_barrier(0);
    DC_SS(1);
    if (g + 1 < NG) {
      // issued: stages < min(NSTAGE, st + S); needed: stages < st + 2 HS
      const int ahead = (st + S < NSTAGE ? st + S : NSTAGE) - st - 2 * HS;
      dc_wait_stages<NBW, S - 1>(ahead);
      DC_SS(2);
      stage_barrier();
      DC_SS(3);
#pragma unroll
      for (int h = 0; h < HS; ++h)
        if (st + h + S < NSTAGE) issue_stage(st + h + S);
      load_group(g + 1, na, nb_);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = KH; i < NF; ++i) mma(ca[i], cb[i]);
    __builtin_amdgcn_sched_barrier(0);
  };
  load_group(0, fa0, fb0);
#pragma unroll 1
  for (int g = 0; g < NG; g += 2) {
    step(g, fa0, fb0, fa1, fb1);
    if (g + 1 < NG) step(g + 1, fa1, fb1, fa0, fb0);
  }
#else
  // Fragments are loaded one k-step ahead of the MFMAs that use them, so LDS
  // latency hides under the previous step's MFMAs; the ring hand-off (wait for
  // stage st+1, barrier, refill slot st % S with stage st+S) sits at the last
  // k-step of a stage, after its fragments are already in registers.
  // sched_barrier(0) pins that order: left alone, the scheduler sinks each
  // fragment load next to its MFMA and every k-step waits out the full LDS
  // latency (s_waitcnt lgkmcnt(0) right before each MFMA).
  bf16x8 afA[FM], bfA[FN], afB[FM], bfB[FN];
  if constexpr (CF::KS == 2) {
    // group g: k-steps kg0, kg0 + 1 of every stage (two MFMA steps per stage and wave)
    load_frags(0, kg0, afA, bfA);
#pragma unroll 1
    for (int st = 0; st < NSTAGE; ++st) {
      load_frags(st, kg0 + 1, afB, bfB);
      __builtin_amdgcn_sched_barrier(0);
      mma(afA, bfA);
      __builtin_amdgcn_sched_barrier(0);
      if (st + 1 < NSTAGE) {
        const int ahead = NSTAGE - 2 - st;
        dc_wait_stages<NBW, S - 1>(ahead < S - 2 ? ahead : S - 2);
        stage_barrier();
        if (st + S < NSTAGE) issue_stage(st + S);
        load_frags(st + 1, kg0, afA, bfA);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(afB, bfB);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
  load_frags(0, 0, afA, bfA);
#pragma unroll 1
  for (int st = 0; st < NSTAGE; ++st) {
    DC_SS(0);
    load_frags(st, 1, afB, bfB);
    __builtin_amdgcn_sched_barrier(0);
    mma(afA, bfA);
    __builtin_amdgcn_sched_barrier(0);
    load_frags(st, 2, afA, bfA);
    __builtin_amdgcn_sched_barrier(0);
    mma(afB, bfB);
    __builtin_amdgcn_sched_barrier(0);
    load_frags(st, 3, afB, bfB);
    __builtin_amdgcn_sched_barrier(0);
    mma(afA, bfA);
    __builtin_amdgcn_sched_barrier(0);
    DC_SS(1);
    if (st + 1 < NSTAGE) {
      const int ahead = NSTAGE - 2 - st;
      dc_wait_stages<NBW, S - 1>(ahead < S - 2 ? ahead : S - 2);
      DC_SS(2);
      stage_barrier();
      DC_SS(3);
      if (st + S < NSTAGE) issue_stage(st + S);
      load_frags(st + 1, 0, afA, bfA);
    }
    __builtin_amdgcn_sched_barrier(0);
    mma(afB, bfB);
    __builtin_amdgcn_sched_barrier(0);
  }
  }
#endif
#undef DC_SS
  dc_stamp(a.stamps, 2);

  // ---- epilogue, per 32-row slice: fragments -> wave-private LDS staging ->
  // row-contiguous 4-column pieces per lane: bias, ReLU, mask (8-B loads),
  // column sums, 8-B bf16 / 16-B f32 stores
  stage_barrier();  // every wave is done with the patch / ring
  const bool store_wave = CF::KS == 1 || w < 4;
  if constexpr (CF::KS == 2) {  // group 1's accumulators into group 0's (fragment order, past the staging slices)
    float* xg = reinterpret_cast<float*>(lds + 4 * CF::STG) + (size_t)wl * FM * FN * 16 * 64;
    if (w >= 4) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) xg[((i * FN + j) * 16 + v) * 64 + lane] = acc[i][j][v];
    }
    __syncthreads();
    if (w < 4) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) acc[i][j][v] += xg[((i * FN + j) * 16 + v) * 64 + lane];
    }
  }
  constexpr int TN = CF::TN, SP = CF::SPITCH;
  constexpr int LPR = TN / 4;       // lanes per row
  constexpr int RPI = 64 / LPR;     // rows per pass
  float* stg = reinterpret_cast<float*>(lds + w * CF::STG);
  const int cq = lane % LPR, rl = lane / LPR;
  const int col0 = nb * CF::NB + (CF::CONV ? wn * TN : 0) + 4 * cq;
  float4 bv = {0.f, 0.f, 0.f, 0.f};
  if (a.bias) bv = *reinterpret_cast<const float4*>(a.bias + col0);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int fm = 0; fm < (store_wave ? FM : 0); ++fm) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
      for (int v = 0; v < 16; ++v)
        stg[((v & 3) + 8 * (v >> 2) + 4 * half) * SP + 32 * fn + (lane & 31)] = acc[fm][fn][v];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 32 / RPI; ++i) {
      const int r = rl + RPI * i;
      const int q = wm * CF::TM + 32 * fm + r;
      size_t grow;
      if constexpr (CF::CONV) {
        grow = ((size_t)n * CF::OH + r0) * OW + q;
      } else {
        const int y = 2 * (r0 + q / WA) + oa, x = 2 * (q % WA) + ob;
        grow = ((size_t)n * (2 * WA) + y) * (2 * WA) + x;
      }
      const size_t o = grow * CF::NCOLS + col0;
      const float4 t = *reinterpret_cast<const float4*>(stg + r * SP + 4 * cq);
      float x[4] = {t.x + bv.x, t.y + bv.y, t.z + bv.z, t.w + bv.w};
      if (a.omask) {
        // bf16 > 0 <=> positive as a signed 16-bit integer (sign clear, nonzero)
        const uint2 m = *reinterpret_cast<const uint2*>(a.omask + o);
        const short e[4] = {(short)(m.x & 0xffffu), (short)(m.x >> 16), (short)(m.y & 0xffffu), (short)(m.y >> 16)};
#pragma unroll
        for (int j = 0; j < 4; ++j) x[j] = e[j] > 0 ? x[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (a.relu) x[j] = fmaxf(x[j], 0.f);
        cs[j] += x[j];
      }
      if (a.y16) {
        s16x4 h;
#pragma unroll
        for (int j = 0; j < 4; ++j) h[j] = __builtin_bit_cast(short, (__bf16)x[j]);
        // write-through (common.h): 0.4-1.9 us per direct-conv launch at
        // 128x128 B=64, conv128 0.3584 -> 0.3531 ms/step (profiles/r5_wt_stores)
        st_wt8(a.y16 + o, __builtin_bit_cast(unsigned long long, h));
      }
      if (a.y32) *reinterpret_cast<float4*>(a.y32 + o) = float4{x[0], x[1], x[2], x[3]};
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (a.colsum) {
    float* sc = reinterpret_cast<float*>(lds + CF::CS_OFF);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int sh = LPR; sh < 64; sh <<= 1) cs[j] += __shfl_xor(cs[j], sh, 64);
    if (lane < LPR && store_wave) *reinterpret_cast<float4*>(sc + w * TN + 4 * cq) = float4{cs[0], cs[1], cs[2], cs[3]};
    __syncthreads();
    if (tid < CF::NB) {
      float t = 0.f;
      if constexpr (CF::CONV) {
        const int wn2 = tid / TN, j = tid % TN;
#pragma unroll
        for (int q = 0; q < CF::WM; ++q) t += sc[(q * CF::WN + wn2) * TN + j];
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) t += sc[q * TN + tid];
      }
      a.colsum[((size_t)n * CF::RB + rb) * CF::NCOLS + nb * CF::NB + tid] = t;
    }
  }
  dc_stamp(a.stamps, 3);
}

template <class CF>
__global__ void __launch_bounds__(CF::THREADS) dconv_k(DcArgs a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[CF::LDS];
  dconv_body<CF>(a, lds, xcd_remap(blockIdx.x, gridDim.x));
}

// The configurations (swizzles searched for conflict-free fragment reads of
// every tap: scripts/dconv_banks.py).
// R = 4 rows per workgroup (two workgroups per CU, <= 80 KB LDS): measured
// 15-18 % faster than R = 8 (one per CU) and 3-4 % faster than R = 2 (three
// per CU, shallower weight rings) at B = 64 and 128 (profiles/r2_dconv).
// The convs take two stages per hand-off (HS = 2): 11.5 -> 11.0 us (64x64)
// and 12.3 -> 10.6 us (32x32) at B = 64 (profiles/r3_dconv2); two k-groups
// there were slower (14.2 / 13.5 us: two 512-thread workgroups per CU).
//                mode CA  WA NCOLS NB  R  WM S  AL BE MK KS HS
using DcS1 = DcCfg<0, 32, 64, 64, 64, 4, 2, 4, 0, 2, 3, 1, 2>;     // conv 64x64x32 -> 32x32x64
using DcS2 = DcCfg<0, 64, 32, 128, 64, 4, 2, 4, 0, 1, 7, 1, 2>;    // conv 32x32x64 -> 16x16x128
using DcT2 = DcCfg<1, 128, 16, 64, 32, 4, 1, 3, 0, 0, 15>;   // tconv 16x16x128 -> 32x32x64
using DcT3 = DcCfg<1, 64, 32, 32, 32, 4, 1, 3, 0, 1, 7>;     // tconv 32x32x64 -> 64x64x32
// 16x16 <-> 8x8 layers: one image (conv, M = 64) / the whole 8x8 class grid
// (tconv, 4 x 64 rows) per workgroup, 64 / 32 output channels; one workgroup
// per CU, so two k-groups of four waves (two waves per SIMD) and two stages
// per hand-off over a ring of 6: enc4 forward 16.4 -> 13.0 us, dec1 12.6 ->
// 11.4 us at B = 64 against one k-group / one stage per hand-off
// (profiles/r3_dconv)
//                mode CA  WA NCOLS NB  R  WM S  AL BE MK KS HS
using DcS3 = DcCfg<0, 128, 16, 256, 64, 8, 2, 6, 4, 0, 15, 2, 2>;  // conv 16x16x128 -> 8x8x256
using DcT1 = DcCfg<1, 256, 8, 128, 32, 8, 1, 6, 8, 0, 15, 2, 2>;   // tconv 8x8x256 -> 16x16x128

}  // namespace mdt
