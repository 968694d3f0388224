// Device bodies of the direct single-channel edge-layer kernels (see
// conv_thin.hip for the design). Included by conv_thin.hip (stand-alone
// kernels) and conv_igemm.hip (horizontally fused job kernels).
#pragma once
#include <stdlib.h>

#include "common.h"
#include "conv_igemm.h"
#include "vae_mlp.h"

namespace mdt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <typename T>
__device__ __forceinline__ float ld1(const T* p) { return (float)*p; }

// Per-block column sums of v[CO] over the block's threads (deterministic):
// transpose through LDS, then thread c < CO adds its column in order.
template <int CO>
__device__ __forceinline__ void block_colsum(const float (&v)[CO], float* red, float* out) {
  const int t = threadIdx.x;
#pragma unroll
  for (int c = 0; c < CO; ++c) red[t * (CO + 1) + c] = v[c];
  __syncthreads();
  if (t < CO) {
    float s = 0.f;
    for (int r = 0; r < (int)blockDim.x; ++r) s += red[r * (CO + 1) + t];
    out[t] = s;
  }
}

struct ThinConvArgs {
  const void* X;       // TIN input (C = 1)
  const float* Wf;     // f32 master weights [CO][K][K]
  ConvDesc d;
  const float* bias;
  int relu;
  __bf16* y16;
  const __bf16* omask;
  float* colsum;       // per-block column sums [blocks][CO] or null
  // optional batch gather (first layer of a step): image n is X row
  // idx[st->cursor * B + n]; the gathered f32 rows are also written to xb
  // (the BCE target and wgrad input); with hp, block 0 also begins the step
  // (step++, Adam beta^t products) -- nothing else in this launch reads them.
  const int* idx;
  TrainState* st;
  const HParams* hp;
  int B;
  float* xb;
  int nblk;
  int mfma;            // 1: thin_conv_mfma_body (host: thin_conv_mfma_ok)
};

// Geometry of the MFMA form of thin_conv (the 128x128 model's enc1 and its
// last layer's backward-data): CO = 32, k4 s2 p1, 64-wide output rows, four
// output rows per 256-pixel workgroup (bit 1 of MDT_THIN_MFMA below).
// MDT_THIN_MFMA: bit mask of the MFMA edge-layer forms in use: 1 thin conv
// with f32 input (enc1 forward), 8 thin conv with bf16 input (last layer's
// backward-data), 2 transposed conv + BCE, 4 weight gradients; 0 keeps every
// VALU / im2col body with LDS weights. Default 15 (all MFMA forms). Bit 1 was
// opt-in through round 4: at the one seed of the model-level gradient test it
// moved the worst deviation from the bf16-emulating f64 reference 0.0178 ->
// 0.0201 (bound 0.02). Round 5 measured ten seeds each way
// (bench/thin_mfma_seeds.py, profiles/r5_thin_mfma): the VALU form itself
// exceeds 0.02 at 3 of 10 seeds (worst 0.0275), the MFMA form at 3 (worst
// 0.0230), mean worst 0.0139 vs 0.0138 -- the deviation is bf16 rounding-flip
// cascades (the worst tensors are dec_fc's, far from enc1), and both forms
// compute enc1 f32-accurately (hi/lo/lo2 bf16 terms of weights and inputs).
// conv128 B=64: 0.3581 -> 0.3555-0.3563 ms/step.
__host__ inline int thin_mfma_mask() {
  static const int m = [] {
    const char* e = getenv("MDT_THIN_MFMA");
    return e ? atoi(e) : 15;
  }();
  return m;
}

__host__ inline bool thin_mfma_geom(const ConvDesc& d) {
  return d.C == 1 && d.CO == 32 && d.KH == 4 && d.KW == 4 && d.S == 2 && d.P == 1 && d.OW == 64 &&
         d.W == 2 * d.OW && d.H == 2 * d.OH && d.OH % 4 == 0;
}

// bit 1: f32 input (enc1 forward), bit 8: bf16 input (last layer's backward-data).
// Returns the body selector of ThinConvArgs::mfma: 1 = MFMA form, 0 = VALU
// body with LDS-broadcast weights (a VALU form with the weights as SGPR
// operands measured slower: enc1 16.7 vs 15.2 us).
__host__ inline int thin_conv_mfma_ok(const ConvDesc& d, int x_is_f32) {
  return (thin_mfma_mask() & (x_is_f32 ? 1 : 8)) && thin_mfma_geom(d) ? 1 : 0;
}


// LDS: staged weights [TAPS][CO] + the colsum transpose (256 x (CO+1)).
template <int CO, int K>
constexpr int thin_conv_lds_bytes() { return (K * K * CO + 256 * (CO + 1)) * 4; }

template <typename TIN>
__device__ void thin_conv_mfma_body(const ThinConvArgs& ta, uint8_t* lds, int bid);

template <int CO, int K, typename TIN>
__device__ __forceinline__ void thin_conv_body(const ThinConvArgs& ta, uint8_t* lds, int bid) {
  if constexpr (CO == 32 && K == 4) {
    if (ta.mfma == 1) {
      thin_conv_mfma_body<TIN>(ta, lds, bid);
      return;
    }
  }
  constexpr int TAPS = K * K;
  const ConvDesc& d = ta.d;
  const TIN* X = reinterpret_cast<const TIN*>(ta.X);
  const float* Wf = ta.Wf;
  const float* bias = ta.bias;
  float* wl = reinterpret_cast<float*>(lds);
  float* red = wl + TAPS * CO;
  const int M = d.N * d.OH * d.OW;
  const int m = bid * blockDim.x + threadIdx.x;
  const bool live = m < M;
  const int mm = live ? m : 0;
  const int n = mm / (d.OH * d.OW);
  const int rem = mm - n * d.OH * d.OW;
  const int oy = rem / d.OW, ox = rem - oy * d.OW;
  const int iy0 = oy * d.S - d.P, ix0 = ox * d.S - d.P;
  const int* rows = ta.idx ? ta.idx + (size_t)ta.st->cursor * ta.B : nullptr;
  const TIN* img = X + (size_t)(rows ? rows[n] : n) * d.H * d.W;
  if (ta.xb) {
    const int p4 = (d.H * d.W) >> 2;
    const long long tot = (long long)d.N * p4;
    for (long long e = (long long)bid * blockDim.x + threadIdx.x; e < tot; e += (long long)ta.nblk * blockDim.x) {
      const int i = (int)(e / p4), c = (int)(e - (long long)i * p4);
      reinterpret_cast<float4*>(ta.xb + (size_t)i * d.H * d.W)[c] =
          reinterpret_cast<const float4*>(X + (size_t)(rows ? rows[i] : i) * d.H * d.W)[c];
    }
  }
  if (ta.hp && bid == 0 && threadIdx.x == 0) {
    TrainState* st = ta.st;
    st->step = st->step + 1;
    st->b1pow *= ta.hp->beta1_d;
    st->b2pow *= ta.hp->beta2_d;
  }
  float xin[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t) {
    const int iy = iy0 + t / K, ix = ix0 + t % K;
    const bool ok = live && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const float x = ld1(img + (ok ? iy * d.W + ix : 0));
    xin[t] = ok ? x : 0.f;
  }
  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = bias ? bias[c] : 0.f;
  {
    // weights staged once per block in LDS as [tap][co]; the FMA loop reads
    // them with wave-uniform (broadcast) ds_read_b128, 4 channels per read
    for (int e = threadIdx.x; e < TAPS * CO; e += blockDim.x) {
      const int c = e / TAPS, t = e - c * TAPS;
      wl[t * CO + c] = Wf[e];
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      const float x = xin[t];
#pragma unroll
      for (int c4 = 0; c4 < CO / 4; ++c4) {
        const float4 w = *reinterpret_cast<const float4*>(wl + t * CO + 4 * c4);
        acc[4 * c4 + 0] = fmaf(x, w.x, acc[4 * c4 + 0]);
        acc[4 * c4 + 1] = fmaf(x, w.y, acc[4 * c4 + 1]);
        acc[4 * c4 + 2] = fmaf(x, w.z, acc[4 * c4 + 2]);
        acc[4 * c4 + 3] = fmaf(x, w.w, acc[4 * c4 + 3]);
      }
    }
  }
  if (ta.relu) {
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = fmaxf(acc[c], 0.f);
  }
  if (ta.omask) {
#pragma unroll
    for (int c8 = 0; c8 < CO / 8; ++c8) {
      const bf16x8 mk = *reinterpret_cast<const bf16x8*>(ta.omask + (size_t)mm * CO + 8 * c8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[8 * c8 + j] = (float)mk[j] > 0.f ? acc[8 * c8 + j] : 0.f;
    }
  }
  {
    // The block's 256 output rows are one contiguous NHWC range: staged in
    // LDS (the colsum transpose area, free until block_colsum) and written as
    // consecutive 16-B chunks, so a wave store covers 1 KB of whole lines.
    // Stored straight from registers, lane l's 16-B chunk c sat 2 CO bytes
    // from lane l + 1's: each store instruction touched 64 separate pieces of
    // 4 KB and the enc1 forward (16.6 us, 20.5 MB written at 1.4 TB/s,
    // profiles/r4_pmc_conv128) was bound by it. Slots are XOR-swizzled by the
    // pixel so neither side of the hand-off piles onto one bank group.
    constexpr int NCH = CO / 8;
    bf16x8* stage = reinterpret_cast<bf16x8*>(red);
    const int t = threadIdx.x;
#pragma unroll
    for (int c8 = 0; c8 < NCH; ++c8) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (__bf16)acc[8 * c8 + j];
      stage[t * NCH + (c8 ^ (t & (NCH - 1)))] = o;
    }
    __syncthreads();
    const long long m0 = (long long)bid * blockDim.x;
    const int npx = (int)(M - m0 < (long long)blockDim.x ? M - m0 : (long long)blockDim.x);
    bf16x8* dst = reinterpret_cast<bf16x8*>(ta.y16 + (size_t)m0 * CO);
    for (int i = t; i < npx * NCH; i += blockDim.x) {
      const int px = i / NCH, c = i - px * NCH;
      dst[i] = stage[px * NCH + (c ^ (px & (NCH - 1)))];
    }
    if (ta.colsum) __syncthreads();  // block_colsum reuses the staging area
  }
  if (ta.colsum) {
    if (!live) {
#pragma unroll
      for (int c = 0; c < CO; ++c) acc[c] = 0.f;
    }
    block_colsum<CO>(acc, red, ta.colsum + (size_t)bid * CO);
  }
}

// Transposed conv with one output channel, conv view (input C = 1 is the
// convT output, CO = convT input channels): y[n, iy, ix] = bias +
// sum over the class taps (ty, tx) and co of G[n, oy, ox, co] * W[co][ky][kx].
// blockIdx.y = parity class (a, b); threads walk the class's pixels.
struct ThinTconvArgs {
  const __bf16* G;
  const float* Wf;
  ConvDesc d;
  const float* bias;
  float* y32;
  const float* X;      // target image (BCE) or null
  __bf16* dlog;
  float* recon;
  float* part;         // BCE partials per block
  float* gpart;        // dlogits partial sums per block (bias gradient)
  int gx;              // blocks per parity class
};

template <int CO, int K, int S>
constexpr int thin_tconv_lds_bytes() { return (16 + (K / S) * (K / S) * CO) * 4; }

// Block `bid` = class * gx + x.
template <int CO, int K, int S>
__device__ __forceinline__ void thin_tconv_body(const ThinTconvArgs& ta, uint8_t* lds, int bid) {
  constexpr int T = K / S;
  const ConvDesc& d = ta.d;
  const __bf16* G = ta.G;
  const float* Wf = ta.Wf;
  float* scratch = reinterpret_cast<float*>(lds);
  float* wl = scratch + 16;
  const int cls = bid / ta.gx, bx = bid - cls * ta.gx;
  const int ca = cls / S, cb = cls - ca * S;
  const int oa = ((ca - d.P) % S + S) % S, ob = ((cb - d.P) % S + S) % S;
  const int ea = (oa + d.P - ca) / S, eb = (ob + d.P - cb) / S;
  const int HS = d.H / S, WS = d.W / S;
  const int Mc = d.N * HS * WS;
  const int m = bx * blockDim.x + threadIdx.x;
  const bool live = m < Mc;
  const int mm = live ? m : 0;
  const int n = mm / (HS * WS);
  const int rem = mm - n * HS * WS;
  const int j = rem / WS, i = rem - j * WS;
  // gather the T*T input rows of CO channels once (16-byte loads)
  float gv[T * T][CO];
#pragma unroll
  for (int ty = 0; ty < T; ++ty)
#pragma unroll
    for (int tx = 0; tx < T; ++tx) {
      const int oy = j + ea - ty, ox = i + eb - tx;
      const bool ok = live && (unsigned)oy < (unsigned)d.OH && (unsigned)ox < (unsigned)d.OW;
      const __bf16* g = G + (((size_t)n * d.OH + (ok ? oy : 0)) * d.OW + (ok ? ox : 0)) * CO;
#pragma unroll
      for (int c8 = 0; c8 < CO / 8; ++c8) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(g + 8 * c8);
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) gv[ty * T + tx][8 * c8 + jj] = ok ? (float)v[jj] : 0.f;
      }
    }
  // this class's T*T taps x CO weights staged in LDS as [tap][co]
  for (int e = threadIdx.x; e < T * T * CO; e += blockDim.x) {
    const int tp = e / CO, c = e - tp * CO;
    const int ky = ca + S * (tp / T), kx = cb + S * (tp % T);
    wl[e] = Wf[(c * K + ky) * K + kx];
  }
  __syncthreads();
  float acc = ta.bias ? ta.bias[0] : 0.f;
#pragma unroll
  for (int tp = 0; tp < T * T; ++tp)
#pragma unroll
    for (int c4 = 0; c4 < CO / 4; ++c4) {
      const float4 w = *reinterpret_cast<const float4*>(wl + tp * CO + 4 * c4);
      acc = fmaf(gv[tp][4 * c4 + 0], w.x, acc);
      acc = fmaf(gv[tp][4 * c4 + 1], w.y, acc);
      acc = fmaf(gv[tp][4 * c4 + 2], w.z, acc);
      acc = fmaf(gv[tp][4 * c4 + 3], w.w, acc);
    }
  const int iy = S * j + oa, ix = S * i + ob;
  const size_t e = ((size_t)n * d.H + iy) * d.W + ix;
  if (!ta.X) {
    if (live && ta.y32) ta.y32[e] = acc;
    return;
  }
  // BCE, dlogits and both block partial sums first, the global stores last:
  // a barrier after a store waits for its acknowledgement (vmcnt counts
  // stores on CDNA). Same summation order as two block_sum calls.
  float loss = 0.f, gsum = 0.f, p = 0.f;
  if (live) {
    const float t = acc, x = ta.X[e];
    p = 1.f / (1.f + expf(-t));
    gsum = p - x;
    const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
    loss = x * fminf(sp_pos - t, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
  }
  const float wl_s = wave_sum(loss), wg_s = ta.gpart ? wave_sum(gsum) : 0.f;
  const int nw = blockDim.x >> 6;
  if (lane_id() == 0) {
    scratch[wave_id()] = wl_s;
    scratch[8 + wave_id()] = wg_s;
  }
  __syncthreads();
  float sl = 0.f, sg = 0.f;
  if (threadIdx.x < 64) {
    sl = wave_sum(threadIdx.x < nw ? scratch[threadIdx.x] : 0.f);
    if (ta.gpart) sg = wave_sum(threadIdx.x < nw ? scratch[8 + threadIdx.x] : 0.f);
  }
  if (live) {
    if (ta.y32) ta.y32[e] = acc;
    if (ta.dlog) ta.dlog[e] = (__bf16)gsum;
    if (ta.recon) ta.recon[e] = p;
  }
  if (threadIdx.x == 0) {
    ta.part[bid] = sl;
    if (ta.gpart) ta.gpart[bid] = sg;
  }
}


// k4/s2/p1 transposed conv with C_out = 1 (the VAE's last layer) where CO = 32
// and the class grid has WS columns with WS | 256: one workgroup = one image's
// R = 256 / WS class-grid rows x all WS columns, one thread per class pixel
// producing its 2x2 output block (one pixel of each stride-parity class) from
// the 3x3 input neighbourhood. The (R+2) x (WS+2) x CO bf16 neighbourhood is staged in LDS
// once with contiguous 16-B row loads (zero padding materialised), instead of
// every thread gathering its own 3x3 neighbourhood through the TA (each input
// chunk 9/4 times: 151 MB of 16-B gathers per 128x128 B=64 step, TA-bound at
// ~25 us). Chunk q of slot x sits at q ^ ((x >> 2) & 3): the 16 consecutive
// slots a lane group reads land on 16 different bank groups. Same fused
// BCE / dlogits / partials as the per-class kernel.
template <int CO, int WS>
constexpr int thin_tconv_patch_lds_bytes() { return (256 / WS + 2) * (WS + 2) * CO * 2 + (16 * CO + 16) * 4; }

template <int CO, int WS>
__device__ __forceinline__ void thin_tconv_patch_body(const ThinTconvArgs& ta, uint8_t* lds, int bid) {
  static_assert(CO == 32 && 256 % WS == 0, "thin_tconv_patch: CO = 32, WS | 256");
  constexpr int R = 256 / WS, PC = WS + 2, NCH = CO / 8, PB = CO * 2;
  const ConvDesc& d = ta.d;
  const int rbn = d.OH / R;
  const int n = bid / rbn, j0 = (bid - n * rbn) * R;
  uint8_t* patch = lds;
  float* wl = reinterpret_cast<float*>(lds + (R + 2) * PC * PB);
  float* scratch = wl + 16 * CO;
  const __bf16* Gn = ta.G + (size_t)n * d.OH * d.OW * CO;
  for (int e = threadIdx.x; e < (R + 2) * PC * NCH; e += blockDim.x) {
    const int pix = e / NCH, q = e - (e / NCH) * NCH;
    const int y = pix / PC, x = pix - (pix / PC) * PC;
    const int gy = j0 - 1 + y, gx = x - 1;
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (__bf16)0.f;
    if ((unsigned)gy < (unsigned)d.OH && (unsigned)gx < (unsigned)d.OW)
      v = *reinterpret_cast<const bf16x8*>(Gn + ((size_t)gy * d.OW + gx) * CO + 8 * q);
    *reinterpret_cast<bf16x8*>(patch + pix * PB + 16 * (q ^ ((x >> 2) & 3))) = v;
  }
  for (int e = threadIdx.x; e < 16 * CO; e += blockDim.x) {
    const int tap = e / CO, c = e - tap * CO;
    const int ca = tap >> 3, cb = (tap >> 2) & 1, ty = (tap >> 1) & 1, tx = tap & 1;
    wl[e] = ta.Wf[(c * 4 + ca + 2 * ty) * 4 + cb + 2 * tx];
  }
  __syncthreads();
  const int jr = threadIdx.x / WS, i = threadIdx.x - jr * WS, j = j0 + jr;
  const float b0 = ta.bias ? ta.bias[0] : 0.f;
  float acc[2][2] = {{b0, b0}, {b0, b0}};
#pragma unroll 1
  for (int c8 = 0; c8 < NCH; ++c8) {
    bf16x8 g[3][3];  // converted at use: 36 VGPRs instead of 72 per chunk
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int x = i + c;
        g[r][c] = *reinterpret_cast<const bf16x8*>(patch + ((jr + r) * PC + x) * PB + 16 * (c8 ^ ((x >> 2) & 3)));
      }
#pragma unroll
    for (int ca = 0; ca < 2; ++ca)
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int ty = 0; ty < 2; ++ty)
#pragma unroll
          for (int tx = 0; tx < 2; ++tx) {
            const int r = (1 - ca) - ty + 1, c = (1 - cb) - tx + 1;
            const float* w = wl + (((ca * 2 + cb) * 2 + ty) * 2 + tx) * CO + 8 * c8;
            const float4 w0 = *reinterpret_cast<const float4*>(w), w1 = *reinterpret_cast<const float4*>(w + 4);
            const bf16x8& gv = g[r][c];
            float a = acc[ca][cb];
            a = fmaf((float)gv[0], w0.x, a); a = fmaf((float)gv[1], w0.y, a);
            a = fmaf((float)gv[2], w0.z, a); a = fmaf((float)gv[3], w0.w, a);
            a = fmaf((float)gv[4], w1.x, a); a = fmaf((float)gv[5], w1.y, a);
            a = fmaf((float)gv[6], w1.z, a); a = fmaf((float)gv[7], w1.w, a);
            acc[ca][cb] = a;
          }
  }
  float loss = 0.f, gsum = 0.f;
#pragma unroll
  for (int ca = 0; ca < 2; ++ca) {
    const int iy = 2 * j + (1 - ca);
    const size_t e = ((size_t)n * d.H + iy) * d.W + 2 * i;
    const float t0 = acc[ca][1], t1 = acc[ca][0];  // columns 2i, 2i+1
    if (ta.y32) *reinterpret_cast<float2*>(ta.y32 + e) = make_float2(t0, t1);
    if (ta.X) {
      const float2 x2 = *reinterpret_cast<const float2*>(ta.X + e);
      const float tv[2] = {t0, t1}, xv[2] = {x2.x, x2.y};
      float pv[2], gv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float t = tv[u], x = xv[u];
        const float p = 1.f / (1.f + expf(-t));
        pv[u] = p;
        gv[u] = p - x;
        const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
        loss += x * fminf(sp_pos - t, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
        gsum += gv[u];
      }
      if (ta.dlog) {
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        bf16x2 g2;
        g2[0] = (__bf16)gv[0];
        g2[1] = (__bf16)gv[1];
        *reinterpret_cast<bf16x2*>(ta.dlog + e) = g2;
      }
      if (ta.recon) *reinterpret_cast<float2*>(ta.recon + e) = make_float2(pv[0], pv[1]);
    }
  }
  if (ta.X) {
    const float sl = block_sum(loss, scratch);
    if (threadIdx.x == 0) ta.part[bid] = sl;
    if (ta.gpart) {
      __syncthreads();
      const float gs = block_sum(gsum, scratch);
      if (threadIdx.x == 0) ta.gpart[bid] = gs;
    }
  }
}

// ---------------------------------------------------------------------------
// MFMA forms of the 128x128 edge layers (round 2). The VALU bodies above read
// every weight as a wave-uniform ds_read_b128 broadcast: an LDS instruction
// costs the same 8 clocks for one broadcast address as for 64 distinct ones,
// so per output pixel they spent ~2x more LDS time on weights than on data and
// ran LDS-bound at 16-23 us per 128x128 B=64 call. Here the weights are MFMA
// A fragments held in VGPRs for the whole workgroup, the activations are the B
// operand read once per tap from the LDS patch, and the f32 master weights are
// split w = hi + lo (two bf16, |w - hi - lo| <= 2^-18 |w|) so the result
// matches the f32-weight VALU kernels to ~1e-6 relative.
__device__ __forceinline__ void split_bf16(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}

// Transposed conv 32 -> 1 (k4 s2 p1, 64^2 -> 128^2) + fused BCE, MFMA form.
// Same grid / partial layout as thin_tconv_patch_body<32, 64> (one workgroup =
// one image's 4 class-grid rows, wave w = row j0 + w, four 16-pixel tiles).
// GEMM per tile (v_mfma_f32_16x16x32_bf16): D[16 x 16 px] = A[16 x K] B[K x 16
// px], K = 9 neighbours x 32 channels (one k-step per 3x3 neighbour); A rows
// 0-3 = hi weights of parity class (ca, cb) = (r >> 1, r & 1), rows 4-7 = lo,
// rows 8-11 = lo2 = bf16(w - hi - lo) (three bf16 terms: the f32 weight to
// ~2^-26), rows 12-15 zero; B = the bf16 activations of
// the tile's 16 pixels at that neighbour straight from the swizzled patch.
// Rows 0-3 + 4-7 + 8-11 (lanes l, l^16, l^32) are the four outputs of each
// pixel; they go through a wave-private LDS row pair so the BCE epilogue runs
// one float4 of an output row per lane.
constexpr int kTcMfmaPatch = 6 * 66 * 64;  // (R + 2) x (WS + 2) pixels x 64 B
constexpr int kTcMfmaAux = 16 * 32 * 4 + 9 * 64 * 16;  // wl [16][32] f32 + A fragments [9][64 lanes] (obuf aliases)
constexpr int thin_tconv_mfma_lds_bytes() { return kTcMfmaPatch + kTcMfmaAux + 16 * 4; }

__device__ __forceinline__ void thin_tconv_mfma_body(const ThinTconvArgs& ta, uint8_t* lds, int bid) {
  constexpr int R = 4, WS = 64, PC = WS + 2, PB = 64, CO = 32;
  static_assert(4 * 256 * 4 <= kTcMfmaAux, "obuf alias");
  const ConvDesc& d = ta.d;
  const int rbn = d.OH / R;
  const int n = bid / rbn, j0 = (bid - n * rbn) * R;
  uint8_t* patch = lds;
  float* wl = reinterpret_cast<float*>(lds + kTcMfmaPatch);                 // [16 taps][32 ch]
  bf16x8* afr = reinterpret_cast<bf16x8*>(lds + kTcMfmaPatch + 16 * CO * 4);  // [9][64]
  float* obuf = reinterpret_cast<float*>(lds + kTcMfmaPatch);               // [4 waves][2][128], after the A loads
  float* scratch = reinterpret_cast<float*>(lds + kTcMfmaPatch + kTcMfmaAux);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const __bf16* Gn = ta.G + (size_t)n * d.OH * d.OW * CO;
  // weights first: waiting for them (vmcnt counts in issue order) must not
  // wait for the patch loads issued after them
  const float wf0 = ta.Wf[tid], wf1 = ta.Wf[tid + 256];
  // this lane's epilogue pixels: output row 2 j + u, columns c4 .. c4 + 3;
  // the BCE target is loaded early so its latency overlaps everything below
  const int u = lane >> 5, c4 = (lane & 31) * 4;
  const size_t e_out = ((size_t)n * d.H + 2 * (j0 + w) + u) * d.W + c4;
  float4 x4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ta.X) x4 = *reinterpret_cast<const float4*>(ta.X + e_out);
  // patch fill, unrolled: every 16-B load is issued before the first LDS
  // store waits (a rolled loop paid one HBM round trip per iteration)
  constexpr int NFILL = (R + 2) * PC * 4, NIT = (NFILL + 255) / 256;
  bf16x8 fv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * 256;
    const int pix = e >> 2, q = e & 3;
    const int y = pix / PC, x = pix - y * PC;
    const int gy = j0 - 1 + y, gx = x - 1;
    const bool ok = e < NFILL && (unsigned)gy < (unsigned)d.OH && (unsigned)gx < (unsigned)d.OW;
    fv[it] = *reinterpret_cast<const bf16x8*>(Gn + (ok ? ((size_t)gy * d.OW + gx) * CO + 8 * q : 0));
    if (!ok) {
#pragma unroll
      for (int k = 0; k < 8; ++k) fv[it][k] = (__bf16)0.f;
    }
  }
  // Wf [ch][ky][kx] -> wl[tap][ch]; the A fragments are built while the
  // patch loads are still in flight (LDS-only barriers: __syncthreads()
  // would also wait for them)
  wl[(tid & 15) * CO + (tid >> 4)] = wf0;
  wl[((tid + 256) & 15) * CO + ((tid + 256) >> 4)] = wf1;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // A fragments, built ONCE per workgroup (each slot = one lane's 8 values of
  // one neighbour step; per-lane builds cost ~1.1k VALU per wave and 8-way
  // bank conflicts on the tap-strided weight reads): lane row m = lane & 15
  // (class m & 3, term m >> 2: hi / lo / lo2 / zero), channels 8 kq .. + 7
  for (int sl = tid; sl < 9 * 64; sl += 256) {
    const int nb = sl >> 6, l = sl & 63, m = l & 15, kq = l >> 4;
    const int r = nb / 3, c = nb - 3 * (nb / 3);
    const int ca = (m >> 1) & 1, cb = m & 1, term = m >> 2;
    const int ty = 2 - ca - r, tx = 2 - cb - c;
    const bool ok = term < 3 && (unsigned)ty < 2u && (unsigned)tx < 2u;
    const int tap = ok ? (ca + 2 * ty) * 4 + cb + 2 * tx : 0;
    const float4 w0 = *reinterpret_cast<const float4*>(wl + tap * CO + 8 * kq);
    const float4 w1 = *reinterpret_cast<const float4*>(wl + tap * CO + 8 * kq + 4);
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    bf16x8 a;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 hi, lo;
      split_bf16(wv[e], hi, lo);
      const __bf16 lo2 = (__bf16)(wv[e] - (float)hi - (float)lo);
      a[e] = ok ? (term == 0 ? hi : (term == 1 ? lo : lo2)) : (__bf16)0.f;
    }
    afr[sl] = a;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  const int kq = lane >> 4;
  bf16x8 af[9];
#pragma unroll
  for (int nb = 0; nb < 9; ++nb) af[nb] = afr[nb * 64 + lane];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * 256;
    const int pix = e >> 2, q = e & 3;
    const int y = pix / PC, x = pix - y * PC;
    if (e < NFILL) *reinterpret_cast<bf16x8*>(patch + pix * PB + 16 * (q ^ ((x >> 2) & 3))) = fv[it];
  }
  __syncthreads();  // patch complete; obuf aliases wl / afr (every wave has read its fragments)
  const float b0 = ta.bias ? ta.bias[0] : 0.f;
  float* ob = obuf + w * 256;
#pragma unroll 1
  for (int t = 0; t < 4; ++t) {
    const int x0 = 16 * t + (lane & 15);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nb = 0; nb < 9; ++nb) {
      const int r = nb / 3, c = nb - 3 * (nb / 3);
      const int x = x0 + c;
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(patch + ((w + r) * PC + x) * PB + 16 * (kq ^ ((x >> 2) & 3)));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[nb], bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {  // rows r + 4 r' (hi, lo, lo2) in lanes l, l + 16, l + 32: hi + (lo + lo2)
      const float lo = __shfl(acc[rr], (lane & 15) + 16, 64), lo2 = __shfl(acc[rr], (lane & 15) + 32, 64);
      acc[rr] += lo + lo2;
    }
    if (lane < 16) {  // class (ca, cb) -> output row 1 - ca, column 2 i + 1 - cb
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) ob[(1 - (rr >> 1)) * 128 + 2 * x0 + 1 - (rr & 1)] = acc[rr] + b0;
    }
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const float4 tv4 = *reinterpret_cast<const float4*>(ob + u * 128 + c4);
  const size_t e = e_out;
  if (ta.y32) *reinterpret_cast<float4*>(ta.y32 + e) = tv4;
  if (!ta.X) return;
  const float tv[4] = {tv4.x, tv4.y, tv4.z, tv4.w}, xv[4] = {x4.x, x4.y, x4.z, x4.w};
  float pv[4], gv[4], loss = 0.f, gsum = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float tq = tv[q], xq = xv[q];
    const float p = 1.f / (1.f + expf(-tq));
    pv[q] = p;
    gv[q] = p - xq;
    const float sp_pos = fmaxf(tq, 0.f) + log1pf(expf(-fabsf(tq)));
    loss += xq * fminf(sp_pos - tq, 100.f) + (1.f - xq) * fminf(sp_pos, 100.f);
    gsum += gv[q];
  }
  if (ta.dlog) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    bf16x4 g4;
#pragma unroll
    for (int q = 0; q < 4; ++q) g4[q] = (__bf16)gv[q];
    *reinterpret_cast<bf16x4*>(ta.dlog + e) = g4;
  }
  if (ta.recon) *reinterpret_cast<float4*>(ta.recon + e) = make_float4(pv[0], pv[1], pv[2], pv[3]);
  const float sl = block_sum(loss, scratch);
  if (threadIdx.x == 0) ta.part[bid] = sl;
  if (ta.gpart) {
    __syncthreads();
    const float gs = block_sum(gsum, scratch);
    if (threadIdx.x == 0) ta.gpart[bid] = gs;
  }
}

// Conv 1 -> 32 (k4 s2 p1, 64-wide output rows), MFMA form of thin_conv_body:
// the 128x128 model's first layer (f32 input gathered from the dataset, bias,
// ReLU) and its last layer's backward-data (bf16 dlogits, ReLU-backward mask,
// bias-gradient column sums). Workgroup = 4 output rows (256 pixels: the same
// blocks, hence the same colsum rows, as the VALU body), wave w = row oy0 + w,
// four 16-pixel tiles. D[32 co x 16 px] = A[co][k] B[k][px] with k = 16 taps
// of x_hi then 16 taps of x_lo, plus [x_lo2 | 0] for f32 input (x = x_hi +
// x_lo + x_lo2, three bf16; bf16 input is exact in x_hi) and A = [W_hi |
// W_hi], [W_lo | W_lo], [W_lo2 | W_lo2] (three bf16 terms of the f32
// weight): the f32 product to ~2^-24 of |x w| -- the same bf16 rounding
// decisions downstream as an f32 kernel (a two-term x split flipped ~0.2 %
// of the enc1 activations' bf16 roundings and doubled the model-level
// gradient deviation from the bf16-emulating reference). A rows are ordered co = 8 (m >> 2) + 4 mt + (m & 3), so lane (q, px)
// ends with channels 8q .. 8q + 7 of its pixel: one 16-B NHWC store.
constexpr int kTcPitch = 132;  // patch row pitch (floats): column ix at ix + 1
template <typename TIN>
__device__ void thin_conv_mfma_body(const ThinConvArgs& ta, uint8_t* lds, int bid) {
  const ConvDesc& d = ta.d;
  const TIN* X = reinterpret_cast<const TIN*>(ta.X);
  float* patch = reinterpret_cast<float*>(lds);  // [10][kTcPitch] f32
  float* red = patch + 10 * kTcPitch;            // [4][32]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rbn = d.OH / 4;
  const int n = bid / rbn, oy0 = (bid - n * rbn) * 4;
  const int* rows = ta.idx ? ta.idx + (size_t)ta.st->cursor * ta.B : nullptr;
  const TIN* img = X + (size_t)(rows ? rows[n] : n) * d.H * d.W;
  // (the gathered rows xb -- BCE target, weight-gradient input -- are written
  // from the patch below: this workgroup's own 8 input rows, no second read)
  if (ta.hp && bid == 0 && tid == 0) {
    TrainState* st = ta.st;
    st->step = st->step + 1;
    st->b1pow *= ta.hp->beta1_d;
    st->b2pow *= ta.hp->beta2_d;
  }
  // input rows 2 oy0 - 1 .. 2 oy0 + 8, columns -1 .. 128 (zero padding
  // stored; thin_conv_mfma_ok fixes W = 128), unrolled so every load is in
  // flight before the first LDS store waits
  constexpr int WP = 130, NFILL = 10 * WP, NIT = (NFILL + 255) / 256;
  float fv[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * 256;
    const int y = e / WP, xx = e - y * WP;
    const int iy = 2 * oy0 - 1 + y, ix = xx - 1;
    const bool ok = e < NFILL && (unsigned)iy < (unsigned)d.H && (unsigned)ix < 128u;
    const float v = (float)img[ok ? iy * 128 + ix : 0];
    fv[it] = ok ? v : 0.f;
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int e = tid + it * 256;
    const int y = e / WP, xx = e - y * WP;
    if (e < NFILL) patch[y * kTcPitch + xx] = fv[it];
    // rows 2 oy0 .. 2 oy0 + 7 (patch rows 1..8) belong to this workgroup
    if (ta.xb && e < NFILL && y >= 1 && y <= 8 && xx >= 1 && xx <= 128)
      ta.xb[((size_t)n * d.H + 2 * oy0 - 1 + y) * 128 + xx - 1] = fv[it];
  }
  // A fragments (weights), lane row m = lane & 15, taps 8 (kq & 1) .. + 7
  const int m = lane & 15, kq = lane >> 4, q = kq;
  bf16x8 ahi[2], alo[2], alo2[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int co = 8 * (m >> 2) + 4 * mt + (m & 3);
    const float4 w0 = *reinterpret_cast<const float4*>(ta.Wf + co * 16 + 8 * (kq & 1));
    const float4 w1 = *reinterpret_cast<const float4*>(ta.Wf + co * 16 + 8 * (kq & 1) + 4);
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      __bf16 hi, lo;
      split_bf16(wv[e], hi, lo);
      ahi[mt][e] = hi;
      alo[mt][e] = lo;
      alo2[mt][e] = (__bf16)(wv[e] - (float)hi - (float)lo);
    }
  }
  float bv[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) bv[c] = ta.bias ? ta.bias[8 * q + c] : 0.f;
  __syncthreads();
  const int oy = oy0 + w;
  float cs[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) cs[c] = 0.f;
  bf16x8 mks[4];
  if (ta.omask) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
      mks[t] = *reinterpret_cast<const bf16x8*>(ta.omask + (((size_t)n * d.OH + oy) * d.OW + 16 * t + (lane & 15)) *
                                                               32 + 8 * q);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ox = 16 * t + (lane & 15);
    const size_t pix = ((size_t)n * d.OH + oy) * d.OW + ox;
    const bf16x8 mk = mks[t];
    bf16x8 b, b2;  // b = [x_hi | x_lo] by k half; b2 = [x_lo2 | 0] (f32 input: x to ~2^-24)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float* pr = patch + (2 * w + 2 * (kq & 1) + r) * kTcPitch + 2 * ox;
      const float2 u0 = *reinterpret_cast<const float2*>(pr), u1 = *reinterpret_cast<const float2*>(pr + 2);
      const float xv[4] = {u0.x, u0.y, u1.x, u1.y};
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        __bf16 hi, lo;
        split_bf16(xv[kx], hi, lo);
        b[4 * r + kx] = kq < 2 ? hi : lo;
        b2[4 * r + kx] = kq < 2 ? (__bf16)(xv[kx] - (float)hi - (float)lo) : (__bf16)0.f;
      }
    }
    f32x4 acc[2];
    // smallest terms first, the hi x hi products last: the small partial sum
    // enters the final MFMA as its accumulator instead of being added to an
    // already large one
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo2[mt], b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo[mt], b, acc[mt], 0, 0, 0);
      if constexpr (sizeof(TIN) == 4) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi[mt], b2, acc[mt], 0, 0, 0);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi[mt], b, acc[mt], 0, 0, 0);
    }
    float v[8];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) v[4 * mt + rr] = acc[mt][rr] + bv[4 * mt + rr];
    if (ta.relu) {
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = fmaxf(v[c], 0.f);
    }
    if (ta.omask) {
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = (float)mk[c] > 0.f ? v[c] : 0.f;
    }
    bf16x8 o;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      o[c] = (__bf16)v[c];
      cs[c] += v[c];
    }
    *reinterpret_cast<bf16x8*>(ta.y16 + pix * 32 + 8 * q) = o;
  }
  if (ta.colsum) {  // column sums: 16 pixel lanes, then the 4 waves in order
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float s = cs[c];
      s += __shfl_xor(s, 1, 64);
      s += __shfl_xor(s, 2, 64);
      s += __shfl_xor(s, 4, 64);
      s += __shfl_xor(s, 8, 64);
      cs[c] = s;
    }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int c = 0; c < 8; ++c) red[w * 32 + 8 * q + c] = cs[c];
    }
    __syncthreads();
    if (tid < 32) ta.colsum[(size_t)bid * 32 + tid] = red[tid] + red[32 + tid] + red[64 + tid] + red[96 + tid];
  }
}

}  // namespace mdt
