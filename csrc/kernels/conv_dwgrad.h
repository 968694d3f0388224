// Direct (row-streamed) weight gradients of the stride-2, 4x4, pad-1 layers of
// the 128x128 conv-VAE on CDNA4 (gfx950), conv view:
//   dW[co][ky][kx][ci] = sum_{n, oy, ox} G[n][oy][ox][co] * X[n][2oy-1+ky][2ox-1+kx][ci]
//
// Why not the im2col weight gradient (wgrad_body): its B operand is the im2col
// of X, gathered 16 B at a time through the TA -- every X element 4 times, G
// once per 64-column k' tile -- ~128 MB of L2/Infinity-Cache reads for the
// 4.3 GFLOP of the 64x64x32 layer. Run beside the direct backward-data kernel
// on a second stream, the two took as long as back to back (profiles/
// r2_dwgrad): both were bound by that traffic, not by latency.
//
// Here a workgroup owns image n and kernel row ky: it streams the image's
// output rows oy (G rows, all CO) and the matching input rows iy = 2oy-1+ky
// (all C, both column parities) through an S-stage LDS-DMA ring and multiplies
// with v_mfma_f32_32x32x16_bf16, k = 16 output pixels of one row. Wave w owns
// kx = w: its tile is all CO x all C of tap (ky, kx). Both operands are read
// transposed (pixels are the reduction dimension) with ds_read_b64_tr_b16:
//   A = G^T  (32 co x 16 px): G row image [px][co];
//   B = X    (16 px x 32 ci): input row split into even / odd columns (slot
//            ox + (kx >> 1) [+ OH + 1 for even kx] holds column 2ox-1+kx), so
//            the 16 pixels of a k-step are 16 consecutive slots;
// both XOR-swizzled per 16-B chunk (dw_gswz / dw_xswz) so that every
// transposed read is conflict-free.
// Each workgroup writes its f32 partial [CO][4 taps][C] into partial row n of
// the [N][CO][16 C] slab (the finalize sums the N rows in order): the same
// 8 MB as the im2col kernel's 64 m-splits at 64x64x32, deterministic.
#pragma once

#include "conv_direct.h"

namespace mdt {

struct DwArgs {
  const __bf16* X;  // NHWC [N][H][H][C] (conv input)
  const __bf16* G;  // NHWC [N][OH][OH][CO] (gradient of the conv output)
  float* out;       // [N][CO][16 C] partial rows
  int nimg;
  unsigned long long* stamps;  // optional [grid][8] s_memrealtime (profiling, mdt_dconv_stamps)
};

// KS_ = 2: two groups of four waves (one wave per kernel column kx each); group
// g multiplies the stage rows r with r % 2 == g, and group 1's accumulators are
// added into group 0's before the store (two waves per SIMD).
template <int C_, int H_, int CO_, int RPS_, int S_, int KS_ = 1>
struct DwCfg {
  static constexpr int C = C_, H = H_, OH = H_ / 2, CO = CO_, RPS = RPS_, S = S_;
  static constexpr int KS = KS_, WAVES = 4 * KS_, THREADS = 64 * WAVES;
  static constexpr int K2 = 16 * C;
  static constexpr int FM = CO / 32, FN = C / 32;
  static constexpr int KPR = OH / 16;                   // k-steps per output row
  static constexpr int NST = OH / RPS;                  // ring stages per workgroup
  static constexpr int SLOTS = 2 * (OH + 1);            // even + odd column slots of an input row
  static constexpr int XROW = SLOTS * 2 * C;            // bytes
  static constexpr int GROW = OH * 2 * CO;
  static constexpr int XINS = (RPS * XROW + 1023) / 1024;
  static constexpr int GINS = (RPS * GROW) / 1024;
  static constexpr int NI = (XINS + GINS + WAVES - 1) / WAVES * WAVES;  // 1-KB DMA instructions per stage
  static constexpr int NIW = NI / WAVES;
  static constexpr int STAGE = NI * 1024;
  static constexpr int GOFF = XINS * 1024;              // G rows inside a stage
  static constexpr int LDS = S * STAGE;
  static_assert((C == 32 || C == 64) && (CO == 64 || CO == 128) && OH % 16 == 0 && OH % RPS == 0, "dwgrad tile");
  static_assert((RPS * GROW) % 1024 == 0 && NST >= S && NIW * (S - 1) <= 63 && LDS <= 160 * 1024, "dwgrad ring");
  static_assert(KS == 1 || (KS == 2 && RPS % 2 == 0 && 4 * FM * FN * 64 * 64 <= LDS), "dwgrad k-groups");
};

// 16-B chunk XOR swizzles (chunk index bits 2-3): the four pixel rows / slots
// that one transposed read of a half-wave touches start on four different
// 64-B bank groups. G rows of 128 B (CO = 64): rows q and q+2 coincide, so
// flip 64 B for (px >> 1) & 1; rows of 256 B (CO = 128) all start on bank 0,
// so shift by px & 3. X slots of 128 B (C = 64) like the 128-B G rows; 64-B
// slots (C = 32) are conflict-free as they are.
template <class CF>
__device__ __forceinline__ int dw_gswz(int px) {
  return (CF::CO == 64 ? ((px >> 1) & 1) : (px & 3)) << 2;
}
template <class CF>
__device__ __forceinline__ int dw_xswz(int slot) {
  return CF::C == 64 ? ((slot >> 1) & 1) << 2 : 0;
}

template <class CF>
__device__ __forceinline__ void dwgrad_body(const DwArgs& a, uint8_t* lds, int b) {
  constexpr int C = CF::C, H = CF::H, OH = CF::OH, CO = CF::CO, RPS = CF::RPS, S = CF::S, NST = CF::NST;
  constexpr int FM = CF::FM, FN = CF::FN, NIW = CF::NIW;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kx = w & 3, grp = w >> 2;
  // the four kernel rows of an image on one XCD (block ids 8 apart): its G rows
  // are fetched into that XCD's L2 once
  int n, ky;
  if ((a.nimg & 7) == 0) {
    const int r = b >> 3;
    ky = r & 3;
    n = (r >> 2) * 8 + (b & 7);
  } else {
    ky = b & 3;
    n = b >> 2;
  }
  const __bf16* Xn = a.X + (size_t)n * H * H * C;
  const __bf16* Gn = a.G + (size_t)n * OH * OH * CO;

  auto issue = [&](int st) {
    uint8_t* dst = lds + (st % S) * CF::STAGE;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int j = i * CF::WAVES + w;
      const int off = j * 1024 + 16 * lane;
      const void* src = g_zero16;
      if (off < RPS * CF::XROW) {
        const int r = off / CF::XROW, rem = off - r * CF::XROW;
        const int slot = rem / (2 * C), ch = (rem - slot * 2 * C) >> 4;
        const int ix = slot <= OH ? 2 * slot : 2 * (slot - OH - 1) - 1;
        const int iy = 2 * (st * RPS + r) - 1 + ky;
        const int lch = ch ^ dw_xswz<CF>(slot);
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)H) src = Xn + ((size_t)iy * H + ix) * C + 8 * lch;
      } else if (off >= CF::GOFF && off < CF::GOFF + RPS * CF::GROW) {
        const int goff = off - CF::GOFF;
        const int r = goff / CF::GROW, rem = goff - r * CF::GROW;
        const int px = rem / (2 * CO), pch = (rem - px * 2 * CO) >> 4;
        const int lch = pch ^ dw_gswz<CF>(px);  // physical chunk pch holds logical chunk lch
        src = Gn + ((size_t)(st * RPS + r) * OH + px) * CO + 8 * lch;
      }
      glds16(src, dst + j * 1024);
    }
  };
  dc_stamp(a.stamps, 0);
#pragma unroll
  for (int s = 0; s < S; ++s) issue(s);

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  // per-lane transposed-read coordinates: group g16 = 16-lane column block,
  // lane 4q + p of it supplies row q, columns 4p .. 4p+3
  const int half = lane >> 5, g16 = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
  const int slot_base = (kx >> 1) + ((kx & 1) ? 0 : OH + 1);  // slot of ox = 0 for this kx

  auto tr = [](const uint8_t* addr) -> s16x4 {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)addr);
  };
  auto kstep = [&](const uint8_t* Xs, const uint8_t* Gs, int px0) {
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
      s16x4 t[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int px = px0 + 8 * half + 4 * u + q;
        const int byte = 2 * (fm * 32 + 16 * g16 + 4 * p);
        t[u] = tr(Gs + px * (2 * CO) + (((byte >> 4) ^ dw_gswz<CF>(px)) << 4) + (byte & 15));
      }
      af[fm] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(t[0], t[1], 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      s16x4 t[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int slot = slot_base + px0 + 8 * half + 4 * u + q;
        const int byte = 2 * (fn * 32 + 16 * g16 + 4 * p);
        t[u] = tr(Xs + slot * (2 * C) + (((byte >> 4) ^ dw_xswz<CF>(slot)) << 4) + (byte & 15));
      }
      bfr[fn] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(t[0], t[1], 0, 1, 2, 3, 4, 5, 6, 7));
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = mfma32(af[fm], bfr[fn], acc[fm][fn]);
  };

#pragma unroll 1
  for (int st = 0; st < NST; ++st) {
    const int ahead = NST - 1 - st;
    dc_wait_stages<NIW, S - 2>(ahead < S - 2 ? ahead : S - 2);  // stage st has landed (this wave's part)
    stage_barrier();  // ... every wave's, and every wave is done with stage st-1's slot
    if (st == 0) dc_stamp(a.stamps, 1);
    if (st == NST / 2) dc_stamp(a.stamps, 2);
    if (st >= 1 && st - 1 + S < NST) issue(st - 1 + S);
    const uint8_t* base = lds + (st % S) * CF::STAGE;
#pragma unroll
    for (int r = 0; r < RPS; r += CF::KS)
#pragma unroll
      for (int k = 0; k < CF::KPR; ++k)
        kstep(base + (r + grp) * CF::XROW, base + CF::GOFF + (r + grp) * CF::GROW, 16 * k);
  }

  if constexpr (CF::KS == 2) {  // group 1's accumulators into group 0's, through the drained ring
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    stage_barrier();
    float* xg = reinterpret_cast<float*>(lds) + (size_t)kx * FM * FN * 16 * 64;
    if (grp == 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int v = 0; v < 16; ++v) xg[((i * FN + j) * 16 + v) * 64 + lane] = acc[i][j][v];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[i][j][v] += xg[((i * FN + j) * 16 + v) * 64 + lane];
  }
  dc_stamp(a.stamps, 3);
  // partial row n: [CO][ky*4 + kx][C]. It leaves through 16-B write-through
  // (sc1) buffer stores, like the im2col weight-gradient slabs
  // (conv_igemm_dev.h wgrad_epilogue): each 32x32 fragment is transposed
  // through a wave-private LDS tile (row pitch 40 floats: the two half-waves'
  // rows land on different banks) so a lane holds 4 consecutive columns.
  // KS == 2 stages in this wave's own exchange slot (it has just read it);
  // KS == 1 waits for every wave to leave the ring first.
  if constexpr (CF::KS == 1) __syncthreads();
  constexpr int PITCH = 40;
  static_assert(4 * 32 * PITCH * 4 <= CF::LDS && (CF::KS == 1 || 32 * PITCH <= FM * FN * 16 * 64), "dwgrad staging");
  float* stg = reinterpret_cast<float*>(lds) + (size_t)kx * (CF::KS == 2 ? FM * FN * 16 * 64 : 32 * PITCH);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(a.out + (size_t)n * CO * CF::K2, 0, CO * CF::K2 * 4, 0x00020000);
  typedef unsigned uvec4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int fm = 0; fm < FM; ++fm)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
#pragma unroll
      for (int v = 0; v < 16; ++v) stg[((v & 3) + 8 * (v >> 2) + 4 * half) * PITCH + (lane & 31)] = acc[fm][fn][v];
      __builtin_amdgcn_wave_barrier();  // one wave's LDS ops run in order; keep the compiler's too
      f32x4 t[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r * 64 + lane;
        t[r] = *reinterpret_cast<const f32x4*>(stg + (i >> 3) * PITCH + 4 * (i & 7));
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = r * 64 + lane;
        const int co = fm * 32 + (i >> 3);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uvec4, t[r]), rs,
                                               (co * CF::K2 + (ky * 4 + kx) * C + fn * 32 + 4 * (i & 7)) * 4, 0,
                                               16 /* sc1 */);
      }
    }
  dc_stamp(a.stamps, 4);
}

template <class CF>
__global__ void __launch_bounds__(CF::THREADS) dwgrad_k(DwArgs a) {
  __shared__ __attribute__((aligned(1024))) uint8_t lds[CF::LDS];
  dwgrad_body<CF>(a, lds, blockIdx.x);
}

//               C   H  CO RPS S KS
#ifndef MDT_DW1_RPS  // A/B builds (ring depth / rows per stage of DwL1)
#define MDT_DW1_RPS 4
#endif
#ifndef MDT_DW1_S
#define MDT_DW1_S 3
#endif
// 64x64x32 -> 32x32x64 (enc2 / dec3): 15.9 -> 14.2 us with two k-groups, 13.4 -> 11.5
// us with 4 rows per stage (profiles/r5_dw_ring)
using DwL1 = DwCfg<32, 64, 64, MDT_DW1_RPS, MDT_DW1_S, 2>;
using DwL2 = DwCfg<64, 32, 128, 4, 3>;   // 32x32x64 -> 16x16x128 (enc3 / dec2)

}  // namespace mdt
