// MFMA weight gradient of the 128x128 conv-VAE's single-channel edge layers
// (gfx950): enc1 (conv 1 -> 32, X = the f32 input batch) and the last layer
// in its conv view (X = bf16 dlogits, G = the previous layer's activations).
// Included by conv_igemm.hip (stand-alone kernel) and conv_jobs.hip (fused
// job kind kJobThinWgM).
//
// Why: the generic weight-gradient GEMM (wgrad_body, per-element gathers
// because C = 1) spent ~4-5 M VALU instructions per call on fast-division
// index math and single-value gathers (profiles/r2_thin PMC). Here
//   dW[co][tap] = sum over pixels of G[px][co] * X[2 oy - 1 + ky][2 ox - 1 + kx]
// is an MFMA reduction over pixels: a workgroup = one image's 4 output rows
// (wave w = row oy0 + w, the same 64-pixel row for all 16 taps), A = G^T read
// with ds_read_b64_tr_b16 from a per-wave [64 px][32 co] LDS image (tr_frag),
// B = the 16 tap views of the input rows, stored de-interleaved by column
// parity (and pre-shifted) so each lane's 8 consecutive pixels of one tap are
// one aligned 32-B LDS read. f32 input is split x = x_hi + x_lo + x_lo2
// (three bf16 MFMAs, the product to ~2^-24 of |g x|). One partial row [32][16] per
// workgroup (the finalize sums N * OH / 4 rows in order, deterministic).
#pragma once
#include "conv_igemm_dev.h"
#include "conv_thin.h"

namespace mdt {

// Geometry of the MFMA thin weight gradient (conv view): C = 1, CO = 32,
// k4 s2 p1, 64-wide output rows, W = 128. MDT_THIN_MFMA without bit 4 keeps wgrad_body.
__host__ inline int thin_wgrad_mfma_ok(const ConvDesc& d) { return (thin_mfma_mask() & 4) && thin_mfma_geom(d); }

constexpr int kTwImg = 64 * 32 * 2;         // per wave: G row image [64 px][32 co] bf16
// per wave: 4 input rows x {O0, E0, O1, E1} x 64 f32, arrays padded to 68
// floats: the 16 taps of one B read (row ky, array kx) start at dword offset
// 16 ky + 4 kx (mod 64), i.e. on 16 distinct 16-B bank groups
constexpr int kTwAS = 68, kTwRS = 4 * kTwAS;
constexpr int kTwX = 4 * kTwRS * 4;
constexpr int kTwWave = kTwImg + kTwX;      // 8.25 KB
constexpr int thin_wgrad_mfma_lds_bytes() { return 4 * kTwWave; }

template <typename XT>
__device__ __forceinline__ void thin_wgrad_mfma_body(const WgArgs& a, uint8_t* lds, int bid) {
  const ConvDesc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rbn = d.OH / 4;
  const int n = bid / rbn, oy = (bid - n * rbn) * 4 + w;
  uint8_t* img = lds + w * kTwWave;
  float* xs = reinterpret_cast<float*>(img + kTwImg);  // [ky][arr][68]: arr 0 = O'[px], 1 = E[px], 2 = O'[px+1], 3 = E[px+1]
  const XT* X = reinterpret_cast<const XT*>(a.X) + (size_t)n * d.H * 128;  // W = 128 (thin_mfma_geom)
  // ---- loads (all issued before the first LDS store): the G row (lane =
  // pixel, 64 B) and the four input rows (lane = column pair 2l, 2l + 1)
  const __bf16* Grow = a.G + (((size_t)n * d.OH + oy) * 64 + lane) * 32;
  bf16x8 gv[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) gv[c] = *reinterpret_cast<const bf16x8*>(Grow + 8 * c);
  float xe[4], xo[4];
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    const int iy = 2 * oy - 1 + ky;
    const bool ok = (unsigned)iy < (unsigned)d.H;
    const XT* p = X + (ok ? iy : 0) * 128 + 2 * lane;
    const float e = (float)p[0], o = (float)p[1];
    xe[ky] = ok ? e : 0.f;
    xo[ky] = ok ? o : 0.f;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) *reinterpret_cast<bf16x8*>(img + timg<32>(lane, c)) = gv[c];
  // column 2l -> E[l] (arr 1 at l, arr 3 at l - 1); column 2l + 1 -> O'[l + 1]
  // (arr 0 at l + 1, arr 2 at l); O'[0] = column -1 and E[64] = column 128 are 0
#pragma unroll
  for (int ky = 0; ky < 4; ++ky) {
    float* r = xs + ky * kTwRS;
    r[kTwAS + lane] = xe[ky];
    if (lane > 0) r[3 * kTwAS + lane - 1] = xe[ky];
    else r[3 * kTwAS + 63] = 0.f;
    if (lane < 63) r[lane + 1] = xo[ky];
    else r[0] = 0.f;
    r[2 * kTwAS + lane] = xo[ky];
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  // ---- MFMA: D[co][tap] += G^T[co][px] X[px][tap], two 32-pixel k-steps
  const int tap = lane & 15, ky = tap >> 2, kx = tap & 3, kq = lane >> 4;
  const float* xb = xs + ky * kTwRS + kx * kTwAS;  // kx 0..3 -> arr O0, E0, O1, E1
  f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const float4 b0 = *reinterpret_cast<const float4*>(xb + 32 * ks + 8 * kq);
    const float4 b1 = *reinterpret_cast<const float4*>(xb + 32 * ks + 8 * kq + 4);
    const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    bf16x8 bh, bl, bl2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 hi, lo;
      split_bf16(bv[e], hi, lo);
      bh[e] = hi;
      bl[e] = lo;
      bl2[e] = (__bf16)(bv[e] - (float)hi - (float)lo);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const bf16x8 af = tr_frag<32>(img, 16 * mt, 32 * ks, lane);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bh, acc[mt], 0, 0, 0);
      if constexpr (sizeof(XT) == 4) {
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bl, acc[mt], 0, 0, 0);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bl2, acc[mt], 0, 0, 0);
      }
    }
  }
  // ---- the four waves' [32][16] partials, summed in wave order
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds);  // [4][512], aliases the images
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) red[w * 512 + (16 * mt + 4 * kq + rr) * 16 + tap] = acc[mt][rr];
  __syncthreads();
  float* out = a.out + (size_t)bid * 512;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    out[e] = ((red[e] + red[512 + e]) + red[1024 + e]) + red[1536 + e];
  }
}

}  // namespace mdt
