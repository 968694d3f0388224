// Direct kernels for the single-channel edge layers of the conv-VAE (gfx950).
//
// The first encoder conv (1 -> 32 channels) and the last decoder transposed
// conv (32 -> 1) are GEMMs with K = 16 or N = 1: on MFMA they waste 4-16x of
// the tile and need per-element im2col gathers (measured 21-41 us per call at
// 128x128, B = 64). Here one thread owns one output pixel and all of its
// channels: the patch is read once, the weights are wave-uniform (the f32
// master copy, fetched with scalar loads and used as SGPR operands of
// v_fma), and the NHWC output row is written with 16-byte stores.
//   thin_conv_k     conv with C_in = 1, CO in {16, 32, 64}: encoder conv 1
//                   (bias + ReLU) and the last layer's backward-data
//                   (output mask + per-block bias-gradient column sums)
//   thin_tconv_k    transposed conv with C_out = 1 (conv view: C = 1), one
//                   stride-parity class per blockIdx.y so the taps, hence the
//                   weights, are uniform; fused logit-form BCE (-100 clamp),
//                   dlogits, reconstruction and loss / bias-gradient partials.
#include "common.h"
#include "conv_igemm.h"

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

template <int CO, int K, typename TIN>
__global__ void __launch_bounds__(256) thin_conv_k(const TIN* X, const float* Wf, ConvDesc d, const float* bias,
                                                   int relu, __bf16* y16, const __bf16* omask, float* colsum) {
  extern __shared__ float red[];  // 256 * (CO + 1) floats when colsum != null
  constexpr int TAPS = K * K;
  const int M = d.N * d.OH * d.OW;
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = m < M;
  const int mm = live ? m : 0;
  const int n = mm / (d.OH * d.OW);
  const int rem = mm - n * d.OH * d.OW;
  const int oy = rem / d.OW, ox = rem - oy * d.OW;
  const int iy0 = oy * d.S - d.P, ix0 = ox * d.S - d.P;
  const TIN* img = X + (size_t)n * d.H * d.W;
  float xin[TAPS];
#pragma unroll
  for (int t = 0; t < TAPS; ++t) {
    const int iy = iy0 + t / K, ix = ix0 + t % K;
    const bool ok = live && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
    const float x = ld1(img + (ok ? iy * d.W + ix : 0));
    xin[t] = ok ? x : 0.f;
  }
  // weights staged once per block in LDS as [tap][co]; the FMA loop reads
  // them with wave-uniform (broadcast) ds_read_b128, 4 channels per read
  __shared__ __attribute__((aligned(16))) float wl[TAPS * CO];
  for (int e = threadIdx.x; e < TAPS * CO; e += blockDim.x) {
    const int c = e / TAPS, t = e - c * TAPS;
    wl[t * CO + c] = Wf[e];
  }
  __syncthreads();
  float acc[CO];
#pragma unroll
  for (int c = 0; c < CO; ++c) acc[c] = bias ? bias[c] : 0.f;
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
  if (relu) {
#pragma unroll
    for (int c = 0; c < CO; ++c) acc[c] = fmaxf(acc[c], 0.f);
  }
  if (omask) {
#pragma unroll
    for (int c8 = 0; c8 < CO / 8; ++c8) {
      const bf16x8 mk = *reinterpret_cast<const bf16x8*>(omask + (size_t)mm * CO + 8 * c8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[8 * c8 + j] = (float)mk[j] > 0.f ? acc[8 * c8 + j] : 0.f;
    }
  }
  if (live) {
#pragma unroll
    for (int c8 = 0; c8 < CO / 8; ++c8) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (__bf16)acc[8 * c8 + j];
      *reinterpret_cast<bf16x8*>(y16 + (size_t)m * CO + 8 * c8) = o;
    }
  }
  if (colsum) {
    if (!live) {
#pragma unroll
      for (int c = 0; c < CO; ++c) acc[c] = 0.f;
    }
    block_colsum<CO>(acc, red, colsum + (size_t)blockIdx.x * CO);
  }
}

// Transposed conv with one output channel, conv view (input C = 1 is the
// convT output, CO = convT input channels): y[n, iy, ix] = bias +
// sum over the class taps (ty, tx) and co of G[n, oy, ox, co] * W[co][ky][kx].
// blockIdx.y = parity class (a, b); threads walk the class's pixels.
template <int CO, int K, int S>
__global__ void __launch_bounds__(256) thin_tconv_k(const __bf16* G, const float* Wf, ConvDesc d, const float* bias,
                                                    float* y32, const float* X, __bf16* dlog, float* recon,
                                                    float* part, float* gpart) {
  __shared__ float scratch[16];
  constexpr int T = K / S;
  const int cls = blockIdx.y;
  const int ca = cls / S, cb = cls - ca * S;
  const int oa = ((ca - d.P) % S + S) % S, ob = ((cb - d.P) % S + S) % S;
  const int ea = (oa + d.P - ca) / S, eb = (ob + d.P - cb) / S;
  const int HS = d.H / S, WS = d.W / S;
  const int Mc = d.N * HS * WS;
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
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
  __shared__ __attribute__((aligned(16))) float wl[T * T * CO];
  for (int e = threadIdx.x; e < T * T * CO; e += blockDim.x) {
    const int tp = e / CO, c = e - tp * CO;
    const int ky = ca + S * (tp / T), kx = cb + S * (tp % T);
    wl[e] = Wf[(c * K + ky) * K + kx];
  }
  __syncthreads();
  float acc = bias ? bias[0] : 0.f;
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
  if (live && y32) y32[e] = acc;
  float loss = 0.f, gsum = 0.f;
  if (X) {
    if (live) {
      const float t = acc, x = X[e];
      const float p = 1.f / (1.f + expf(-t));
      const float g = p - x;
      if (dlog) dlog[e] = (__bf16)g;
      if (recon) recon[e] = p;
      const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
      loss = x * fminf(sp_pos - t, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
      gsum = g;
    }
    const int pb = blockIdx.y * gridDim.x + blockIdx.x;
    const float s = block_sum(loss, scratch);
    if (threadIdx.x == 0) part[pb] = s;
    if (gpart) {
      __syncthreads();
      const float gs = block_sum(gsum, scratch);
      if (threadIdx.x == 0) gpart[pb] = gs;
    }
  }
}

}  // namespace mdt

using namespace mdt;

static inline int cdiv_t(long long a, long long b) { return (int)((a + b - 1) / b); }

extern "C" {

// conv with a single input channel; x_is_f32 selects f32 / bf16 input.
int mdt_thin_conv(const void* X, int x_is_f32, const float* Wf, ConvDesc d, const float* bias, int relu, void* y16,
                  const void* omask, float* colsum, hipStream_t s) {
  if (d.C != 1 || d.KH != 4 || d.KW != 4) return 1;
  const long long M = (long long)d.N * d.OH * d.OW;
  dim3 grid(cdiv_t(M, 256)), blk(256);
  __bf16* y = reinterpret_cast<__bf16*>(y16);
  const __bf16* mk = reinterpret_cast<const __bf16*>(omask);
#define THIN(CO_)                                                                                                  \
  {                                                                                                                \
    const size_t sh = colsum ? 256 * (CO_ + 1) * sizeof(float) : 0;                                                \
    if (x_is_f32)                                                                                                  \
      hipLaunchKernelGGL((thin_conv_k<CO_, 4, float>), grid, blk, sh, s, reinterpret_cast<const float*>(X), Wf, d, \
                         bias, relu, y, mk, colsum);                                                               \
    else                                                                                                           \
      hipLaunchKernelGGL((thin_conv_k<CO_, 4, __bf16>), grid, blk, sh, s, reinterpret_cast<const __bf16*>(X), Wf,  \
                         d, bias, relu, y, mk, colsum);                                                            \
  }
  switch (d.CO) {
    case 16: THIN(16); break;
    case 32: THIN(32); break;
    case 64: THIN(64); break;
    default: return 2;
  }
#undef THIN
  return (int)hipGetLastError();
}

// blocks of the per-block partial outputs (colsum rows for thin_conv,
// loss partials for thin_tconv)
int mdt_thin_blocks(int tconv, ConvDesc d) {
  if (!tconv) return cdiv_t((long long)d.N * d.OH * d.OW, 256);
  return cdiv_t((long long)d.N * (d.H / d.S) * (d.W / d.S), 256) * d.S * d.S;
}

int mdt_thin_tconv(const void* G16, const float* Wf, ConvDesc d, const float* bias, float* y32, const float* X,
                   void* dlog16, float* recon, float* part, float* gpart, hipStream_t s) {
  if (d.C != 1 || d.KH != 4 || d.KW != 4 || d.S != 2 || d.H % 2 || d.W % 2) return 1;
  if (X && !part) return 1;
  const long long Mc = (long long)d.N * (d.H / d.S) * (d.W / d.S);
  dim3 grid(cdiv_t(Mc, 256), d.S * d.S), blk(256);
  const __bf16* G = reinterpret_cast<const __bf16*>(G16);
  __bf16* dl = reinterpret_cast<__bf16*>(dlog16);
  switch (d.CO) {
    case 16: hipLaunchKernelGGL((thin_tconv_k<16, 4, 2>), grid, blk, 0, s, G, Wf, d, bias, y32, X, dl, recon, part, gpart); break;
    case 32: hipLaunchKernelGGL((thin_tconv_k<32, 4, 2>), grid, blk, 0, s, G, Wf, d, bias, y32, X, dl, recon, part, gpart); break;
    case 64: hipLaunchKernelGGL((thin_tconv_k<64, 4, 2>), grid, blk, 0, s, G, Wf, d, bias, y32, X, dl, recon, part, gpart); break;
    default: return 2;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
