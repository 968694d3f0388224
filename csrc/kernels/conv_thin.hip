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
#include <stdlib.h>

#include "conv_thin.h"

namespace mdt {

template <int CO, int K, typename TIN>
__global__ void __launch_bounds__(256) thin_conv_k(ThinConvArgs ta) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[thin_conv_lds_bytes<CO, K>()];
  thin_conv_body<CO, K, TIN>(ta, lds, blockIdx.x);
}

template <int CO, int WS>
__global__ void __launch_bounds__(256) thin_tconv_patch_k(ThinTconvArgs ta) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[thin_tconv_patch_lds_bytes<CO, WS>()];
  thin_tconv_patch_body<CO, WS>(ta, lds, blockIdx.x);
}

__global__ void __launch_bounds__(256) thin_tconv_mfma_k(ThinTconvArgs ta) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[thin_tconv_mfma_lds_bytes()];
  thin_tconv_mfma_body(ta, lds, blockIdx.x);
}

template <int CO, int K, int S>
__global__ void __launch_bounds__(256) thin_tconv_k(ThinTconvArgs ta) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[thin_tconv_lds_bytes<CO, K, S>()];
  thin_tconv_body<CO, K, S>(ta, lds, blockIdx.x);
}

}  // namespace mdt


using namespace mdt;

static inline int cdiv_t(long long a, long long b) { return (int)((a + b - 1) / b); }

extern "C" {

// conv with a single input channel; x_is_f32 selects f32 / bf16 input.
int mdt_thin_conv(const void* X, int x_is_f32, const float* Wf, ConvDesc d, const float* bias, int relu, void* y16,
                  const void* omask, float* colsum, const int* idx, void* st, const void* hp, int B, float* xb,
                  hipStream_t s) {
  if (d.C != 1 || d.KH != 4 || d.KW != 4) return 1;
  if ((idx || xb || hp) && (!st || !x_is_f32 || (d.H * d.W) % 4)) return 1;
  const long long M = (long long)d.N * d.OH * d.OW;
  dim3 grid(cdiv_t(M, 256)), blk(256);
  const ThinConvArgs ta{X, Wf, d, bias, relu, reinterpret_cast<__bf16*>(y16), reinterpret_cast<const __bf16*>(omask),
                        colsum, idx, reinterpret_cast<TrainState*>(st), reinterpret_cast<const HParams*>(hp), B, xb,
                        (int)grid.x, thin_conv_mfma_ok(d, x_is_f32)};
#define THIN(CO_)                                                                     \
  {                                                                                   \
    if (x_is_f32)                                                                     \
      hipLaunchKernelGGL((thin_conv_k<CO_, 4, float>), grid, blk, 0, s, ta);          \
    else                                                                              \
      hipLaunchKernelGGL((thin_conv_k<CO_, 4, __bf16>), grid, blk, 0, s, ta);         \
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

// Halo-patch kernel (thin_tconv_patch_body): CO = 32, square 4x4/s2/p1, class
// grid width 64 (the 128x128 model's last layer). MDT_THIN_PATCH=0 disables.
static bool tconv_patch_ok(const ConvDesc& d) {
  static const bool on = [] {
    const char* e = getenv("MDT_THIN_PATCH");
    return !(e && e[0] == '0');
  }();
  return on && d.CO == 32 && d.KH == 4 && d.KW == 4 && d.S == 2 && d.P == 1 && d.H == d.W && d.OH == d.OW &&
         d.H == 2 * d.OH && d.OW == 64;
}

// MFMA form of the patch kernel (thin_tconv_mfma_body, same grid and
// partials): bit 2 of MDT_THIN_MFMA (conv_thin.h thin_mfma_mask).
static bool thin_mfma_on() { return (thin_mfma_mask() & 2) != 0; }

// blocks of the per-block partial outputs (colsum rows for thin_conv,
// loss partials for thin_tconv)
int mdt_thin_blocks(int tconv, ConvDesc d) {
  if (!tconv) return cdiv_t((long long)d.N * d.OH * d.OW, 256);
  if (tconv_patch_ok(d)) return d.N * (d.OH / 4);
  return cdiv_t((long long)d.N * (d.H / d.S) * (d.W / d.S), 256) * d.S * d.S;
}

int mdt_thin_tconv(const void* G16, const float* Wf, ConvDesc d, const float* bias, float* y32, const float* X,
                   void* dlog16, float* recon, float* part, float* gpart, hipStream_t s) {
  if (d.C != 1 || d.KH != 4 || d.KW != 4 || d.S != 2 || d.H % 2 || d.W % 2) return 1;
  if (X && !part) return 1;
  const long long Mc = (long long)d.N * (d.H / d.S) * (d.W / d.S);
  const int gx = cdiv_t(Mc, 256);
  if (tconv_patch_ok(d)) {
    const ThinTconvArgs tp{reinterpret_cast<const __bf16*>(G16), Wf, d, bias, y32, X,
                           reinterpret_cast<__bf16*>(dlog16), recon, part, gpart, gx};
    if (thin_mfma_on())
      hipLaunchKernelGGL(thin_tconv_mfma_k, dim3(d.N * (d.OH / 4)), dim3(256), 0, s, tp);
    else
      hipLaunchKernelGGL((thin_tconv_patch_k<32, 64>), dim3(d.N * (d.OH / 4)), dim3(256), 0, s, tp);
    return (int)hipGetLastError();
  }
  dim3 grid(gx * d.S * d.S), blk(256);
  const ThinTconvArgs ta{reinterpret_cast<const __bf16*>(G16), Wf, d, bias, y32, X, reinterpret_cast<__bf16*>(dlog16),
                         recon, part, gpart, gx};
  switch (d.CO) {
    case 16: hipLaunchKernelGGL((thin_tconv_k<16, 4, 2>), grid, blk, 0, s, ta); break;
    case 32: hipLaunchKernelGGL((thin_tconv_k<32, 4, 2>), grid, blk, 0, s, ta); break;
    case 64: hipLaunchKernelGGL((thin_tconv_k<64, 4, 2>), grid, blk, 0, s, ta); break;
    default: return 2;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
