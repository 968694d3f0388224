// Implicit-GEMM convolution / transposed convolution in NHWC on CDNA4 bf16
// MFMA (v_mfma_f32_16x16x32_bf16, f32 accumulate) for the conv-VAE family.
//
// Three kernels cover every layer of a conv/deconv encoder-decoder (and
// Linear layers as 1x1 convs on 1x1 images):
//   conv_fwd    Y[m, co]  = sum_{ky,kx,ci} X[n, oy*S-P+ky, ox*S-P+kx, ci] W[co][ky][kx][ci]
//               (conv forward; transposed-conv backward-data)
//   conv_dgrad  Y[m, ci]  = sum_{ky,kx,co} G[n, (iy+P-ky)/S, (ix+P-kx)/S, co] Wt[ci][ky][kx][co]
//               over the taps where the division is exact (zero-insertion form):
//               conv backward-data; transposed-conv forward
//   conv_wgrad  dW[co][ky][kx][ci] += sum_m G[m, co] X[n, oy*S-P+ky, ox*S-P+kx, ci]
//               (+ db[co] += sum_m G[m, co]); split over m, f32 atomics
// GEMM mapping: rows = output pixels (n, y, x), cols = output channels, K =
// (tap, channel) with the channel fastest, so each lane's 8 consecutive k of a
// 32-deep MFMA chunk are 8 consecutive channels of one tap: ONE 16-byte load
// (channels % 8 == 0), or 8 element gathers for thin layers (C = 1, 4).
// Weights are stored [Cout][KH][KW][Cin] (bf16 copy of the fp32 master) and
// transposed [Cin][KH][KW][Cout] for dgrad, both written by the fused
// Adam+cast pass (adam_cast below), so every weight fragment is contiguous.
// Epilogues fuse bias, ReLU, the ReLU mask of the incoming gradient, bf16
// packing, and (BCE layer) nothing else; split-K over waves through LDS.
#include "common.h"
#include "vae_mlp.h"
#include "adam_common.h"

namespace mdt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct ConvDesc {
  int N, H, W, C;      // conv input  (NHWC)
  int OH, OW, CO;      // conv output
  int KH, KW, S, P;
};

// ------------------------------------------------------------ loaders ----
template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&o)[8]);
template <>
__device__ __forceinline__ void load8<__bf16>(const __bf16* p, float (&o)[8]) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

__device__ __forceinline__ bf16x8 to_bf16x8(const float (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p) { return (float)*p; }

// A fragment of conv_fwd: lane row m = (n, oy, ox), k = kbase..kbase+7.
// X is either an NHWC activation (rows == nullptr) or dataset rows gathered
// by sample index (image n -> X + rows[n] * H*W*C).
template <typename TIN, bool VEC>
__device__ __forceinline__ bf16x8 conv_a_frag(const TIN* X, const int* rows, const ConvDesc& d, int m, int kbase,
                                              int K) {
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int M = d.N * d.OH * d.OW;
  if (m < M) {
    const int n = m / (d.OH * d.OW);
    const int rem = m - n * d.OH * d.OW;
    const int oy = rem / d.OW, ox = rem - oy * d.OW;
    const TIN* img = X + (size_t)(rows ? rows[n] : n) * d.H * d.W * d.C;
    if constexpr (VEC) {
      if (kbase < K) {
        const int tap = kbase / d.C, ci = kbase - tap * d.C;
        const int ky = tap / d.KW, kx = tap - ky * d.KW;
        const int iy = oy * d.S - d.P + ky, ix = ox * d.S - d.P + kx;
        if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) load8<TIN>(img + ((size_t)iy * d.W + ix) * d.C + ci, v);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kbase + j;
        if (k < K) {
          const int tap = k / d.C, ci = k - tap * d.C;
          const int ky = tap / d.KW, kx = tap - ky * d.KW;
          const int iy = oy * d.S - d.P + ky, ix = ox * d.S - d.P + kx;
          if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) v[j] = ldf(img + ((size_t)iy * d.W + ix) * d.C + ci);
        }
      }
    }
  }
  return to_bf16x8(v);
}

// A fragment of conv_dgrad: lane row m = (n, iy, ix) of the conv INPUT space,
// k = (ky, kx, co); G is [N, OH, OW, CO] bf16, optionally masked by mask > 0.
template <bool VEC>
__device__ __forceinline__ bf16x8 dgrad_a_frag(const __bf16* G, const __bf16* mask, const ConvDesc& d, int m,
                                               int kbase, int K) {
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int M = d.N * d.H * d.W;
  if (m < M) {
    const int n = m / (d.H * d.W);
    const int rem = m - n * d.H * d.W;
    const int iy = rem / d.W, ix = rem - iy * d.W;
#pragma unroll
    for (int j = 0; j < (VEC ? 1 : 8); ++j) {
      const int k = kbase + j;
      if (k < K) {
        const int tap = k / d.CO, co = k - tap * d.CO;
        const int ky = tap / d.KW, kx = tap - ky * d.KW;
        const int ty = iy + d.P - ky, tx = ix + d.P - kx;
        if (ty >= 0 && tx >= 0 && ty % d.S == 0 && tx % d.S == 0) {
          const int oy = ty / d.S, ox = tx / d.S;
          if (oy < d.OH && ox < d.OW) {
            const size_t o = (((size_t)n * d.OH + oy) * d.OW + ox) * d.CO + co;
            if constexpr (VEC) {
              load8<__bf16>(G + o, v);
              if (mask) {
                float mk[8];
                load8<__bf16>(mask + o, mk);
#pragma unroll
                for (int t = 0; t < 8; ++t) v[t] = mk[t] > 0.f ? v[t] : 0.f;
              }
            } else {
              const float g = (float)G[o];
              v[j] = (mask && !((float)mask[o] > 0.f)) ? 0.f : g;
            }
          }
        }
      }
    }
  }
  return to_bf16x8(v);
}

// B fragment: weights row `col` (K contiguous), k = kbase..kbase+7 (K % 8 == 0)
__device__ __forceinline__ bf16x8 w_frag(const __bf16* Wrow, int kbase, int K, bool colok) {
  if (colok && kbase < K) return *reinterpret_cast<const bf16x8*>(Wrow + kbase);
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

// -------------------------------------------------------------- epilogue ----
struct ConvOut {
  __bf16* y16;         // bf16 NHWC output (or null)
  float* y32;          // f32 output (or null)
  const float* bias;   // per output channel (or null)
  int relu;
  const __bf16* omask; // zero outputs where omask <= 0 (fused ReLU backward) (or null)
};

__device__ __forceinline__ void conv_store(const ConvOut& o, int M, int NC, int m0, int col, const f32x4& acc) {
  if (col >= NC) return;
  const float b = o.bias ? o.bias[col] : 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = m0 + r;
    if (m >= M) continue;
    float v = acc[r] + b;
    if (o.relu) v = fmaxf(v, 0.f);
    if (o.omask && !((float)o.omask[(size_t)m * NC + col] > 0.f)) v = 0.f;
    if (o.y16) o.y16[(size_t)m * NC + col] = (__bf16)v;
    if (o.y32) o.y32[(size_t)m * NC + col] = v;
  }
}

constexpr int kCW = 8;            // waves per block
constexpr int kCThreads = kCW * 64;

// One 16x16 output tile per KSPLIT waves (TPB tiles per block), K split over
// the KSPLIT waves in 32-deep chunks, combined through LDS.
template <int TPB, typename AFRAG, typename BFRAG>
__device__ __forceinline__ void igemm_block(AFRAG afrag, BFRAG bfrag, int M, int NC, int K, const ConvOut& out,
                                            float* lds) {
  constexpr int KSPLIT = kCW / TPB;
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int tiles_n = (NC + 15) / 16;
  const int ntiles = ((M + 15) / 16) * tiles_n;
  const int tile = blockIdx.x * TPB + w / KSPLIT;
  const int ks = w % KSPLIT;
  const bool live = tile < ntiles;
  const int tt = live ? tile : ntiles - 1;
  const int ti = tt / tiles_n, tj = tt - ti * tiles_n;
  const int nch = (K + 31) / 32;
  const int kc0 = (ks * nch) / KSPLIT, kc1 = ((ks + 1) * nch) / KSPLIT;
  const int r = lane & 15, q = lane >> 4;
  const int m = ti * 16 + r, col = tj * 16 + r;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int NB = 4;  // chunks whose loads are issued together
  for (int kc = kc0; kc < kc1; kc += NB) {
    bf16x8 a[NB], b[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const int c = kc + u;
      const int kb = (c < kc1 ? c : kc1 - 1) * 32 + 8 * q;
      a[u] = afrag(m, c < kc1 ? kb : K);  // k >= K -> zero fragment
      b[u] = bfrag(col, kb);
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) acc = mfma_bf16(a[u], b[u], acc);
  }
  if constexpr (KSPLIT > 1) {
    *reinterpret_cast<f32x4*>(lds + w * 256 + lane * 4) = acc;
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int s = 1; s < KSPLIT; ++s) acc += *reinterpret_cast<const f32x4*>(lds + (w + s) * 256 + lane * 4);
    }
  }
  if (live && ks == 0) conv_store(out, M, NC, ti * 16 + 4 * q, col, acc);
}

template <typename TIN, bool VEC, int TPB>
__global__ void __launch_bounds__(kCThreads) conv_fwd_k(const TIN* X, const int* rows, const __bf16* Wt16,
                                                        ConvDesc d, ConvOut out) {
  __shared__ __attribute__((aligned(16))) float lds[kCW * 256];
  const int K = d.KH * d.KW * d.C;
  const int M = d.N * d.OH * d.OW;
  auto af = [&](int m, int kb) { return conv_a_frag<TIN, VEC>(X, rows, d, m, kb, K); };
  auto bf = [&](int col, int kb) {
    return w_frag(Wt16 + (size_t)min(col, d.CO - 1) * K, kb, K, col < d.CO);
  };
  igemm_block<TPB>(af, bf, M, d.CO, K, out, lds);
}

template <bool VEC, int TPB>
__global__ void __launch_bounds__(kCThreads) conv_dgrad_k(const __bf16* G, const __bf16* mask, const __bf16* Wtr,
                                                          ConvDesc d, ConvOut out) {
  __shared__ __attribute__((aligned(16))) float lds[kCW * 256];
  const int K = d.KH * d.KW * d.CO;
  const int M = d.N * d.H * d.W;
  auto af = [&](int m, int kb) { return dgrad_a_frag<VEC>(G, mask, d, m, kb, K); };
  auto bf = [&](int col, int kb) { return w_frag(Wtr + (size_t)min(col, d.C - 1) * K, kb, K, col < d.C); };
  igemm_block<TPB>(af, bf, M, d.C, K, out, lds);
}

// dW[co][k'] (k' = (ky, kx, ci)) += sum over this block's m-slice of
// G[m][co] (x mask) * X[gather(m, k')]; one 16x16 (co, k') tile per wave,
// 8 waves per block each on a different m-range; db from the G row sums.
template <typename TX>
__global__ void __launch_bounds__(kCThreads) conv_wgrad_k(const __bf16* G, const __bf16* mask, const TX* X,
                                                          const int* rows, ConvDesc d, float* dW, float* db,
                                                          int msplit) {
  const int lane = lane_id(), w = __builtin_amdgcn_readfirstlane(wave_id());
  const int K2 = d.KH * d.KW * d.C;  // columns
  const int M = d.N * d.OH * d.OW;   // reduction
  const int tiles_k = (K2 + 15) / 16;
  const int tile = blockIdx.x / msplit;
  const int part = (blockIdx.x - tile * msplit) * kCW + w;
  const int nparts = msplit * kCW;
  const int ti = tile / tiles_k, tj = tile - ti * tiles_k;
  const int r = lane & 15, q = lane >> 4;
  const int co = ti * 16 + r;   // A row (output channel)
  const int kcol = tj * 16 + r; // B column
  const bool co_ok = co < d.CO, k_ok = kcol < K2;
  int ky = 0, kx = 0, ci = 0;
  if (k_ok) {
    const int tap = kcol / d.C;
    ci = kcol - tap * d.C;
    ky = tap / d.KW;
    kx = tap - ky * d.KW;
  }
  const int nch = (M + 31) / 32;
  const int c0 = (part * nch) / nparts, c1 = ((part + 1) * nch) / nparts;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float rs = 0.f;
  for (int c = c0; c < c1; ++c) {
    float av[8], bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = c * 32 + 8 * q + j;
      av[j] = 0.f;
      bv[j] = 0.f;
      if (m < M) {
        if (co_ok) {
          const size_t o = (size_t)m * d.CO + co;
          const float g = (float)G[o];
          av[j] = (mask && !((float)mask[o] > 0.f)) ? 0.f : g;
        }
        if (k_ok) {
          const int n = m / (d.OH * d.OW);
          const int rem = m - n * d.OH * d.OW;
          const int oy = rem / d.OW, ox = rem - oy * d.OW;
          const int iy = oy * d.S - d.P + ky, ix = ox * d.S - d.P + kx;
          if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W) {
            const TX* img = X + (size_t)(rows ? rows[n] : n) * d.H * d.W * d.C;
            bv[j] = ldf(img + ((size_t)iy * d.W + ix) * d.C + ci);
          }
        }
      }
    }
    bf16x8 a = to_bf16x8(av), b = to_bf16x8(bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) rs += av[j];
    acc = mfma_bf16(a, b, acc);
  }
  rs += __shfl_xor(rs, 16, 64);
  rs += __shfl_xor(rs, 32, 64);
  if (c0 < c1) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int orow = ti * 16 + 4 * q + rr;
      if (orow < d.CO && k_ok) atomicAdd(dW + (size_t)orow * K2 + kcol, acc[rr]);
    }
    if (db && tj == 0 && q == 0 && co_ok) atomicAdd(db + co, rs);
  }
}

// Per-channel sum of a bf16 [M][C] gradient (bias grad of transposed convs).
__global__ void __launch_bounds__(256) chan_sum_k(const __bf16* G, int M, int C, float* db) {
  const int c = blockIdx.y * 64 + (threadIdx.x & 63);
  const int part = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nparts = gridDim.x * 4;
  if (c >= C) return;
  float s = 0.f;
  for (int m = part; m < M; m += nparts) s += (float)G[(size_t)m * C + c];
  atomicAdd(db + c, s);
}

// --------------------------------------------------- VAE head / loss ----
// mulv [B, 2Z] f32 -> z (bf16 [B, Z] = a 1x1 "image" for the decoder Linear),
// eps f32, KLD partials. Philox stream identical to the MLP kernels.
__global__ void __launch_bounds__(256) reparam_k(const float* mulv, float* eps, __bf16* z16, float* z32, int B,
                                                 int Z, const TrainState* st, const HParams* hp, uint32_t stream,
                                                 float* kld_part) {
  __shared__ float scratch[16];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  float kl = 0.f;
  if (e < B * Z) {
    const int i = e / Z, c = e - i * Z;
    const float mu = mulv[(size_t)i * 2 * Z + c], lv = mulv[(size_t)i * 2 * Z + Z + c];
    const long long stp = st->step - 1;
    const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(i * Z + c), stream, (uint32_t)((unsigned long long)stp & 0xffffffffu),
                                           (uint32_t)((unsigned long long)stp >> 32)},
                                     hp->seed_lo, hp->seed_hi);
    const float ep = normal_from_bits(bits.x, bits.y);
    const float sd = expf(0.5f * lv);
    const float zz = mu + ep * sd;
    eps[e] = ep;
    z16[e] = (__bf16)zz;
    if (z32) z32[e] = zz;
    kl = 1.f + lv - mu * mu - sd * sd;
  }
  const float s = block_sum(kl, scratch);
  if (threadIdx.x == 0) kld_part[blockIdx.x] = -0.5f * s;
}

// dz (f32 [B, Z], from the decoder Linear's dgrad) -> d[mu|lv] (f32 [B, 2Z]).
__global__ void __launch_bounds__(256) reparam_bwd_k(const float* dz, const float* mulv, const float* eps,
                                                     float* dmulv, __bf16* dmulv16, int B, int Z, const HParams* hp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * Z) return;
  const int i = e / Z, c = e - i * Z;
  const float beta = hp->kl_beta;
  const float mu = mulv[(size_t)i * 2 * Z + c], lv = mulv[(size_t)i * 2 * Z + Z + c];
  const float sd = expf(0.5f * lv);
  const float g = dz[e];
  const float dm = g + beta * mu;
  const float dl = 0.5f * g * eps[e] * sd + 0.5f * beta * (sd * sd - 1.f);
  dmulv[(size_t)i * 2 * Z + c] = dm;
  dmulv[(size_t)i * 2 * Z + Z + c] = dl;
  if (dmulv16) {
    dmulv16[(size_t)i * 2 * Z + c] = (__bf16)dm;
    dmulv16[(size_t)i * 2 * Z + Z + c] = (__bf16)dl;
  }
}

// xb[i, :] = X[idx[cursor*B + i], :] for the current batch (f32 rows).
__global__ void __launch_bounds__(256) gather_rows_k(const float* X, const int* idx, const TrainState* st, int B,
                                                     int M, int P, float* xb) {
  const int* rows = idx + (size_t)st->cursor * B;
  const int p4 = P >> 2;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < (long long)M * p4;
       e += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(e / p4), c = (int)(e - (long long)i * p4);
    reinterpret_cast<float4*>(xb + (size_t)i * P)[c] = reinterpret_cast<const float4*>(X + (size_t)rows[i] * P)[c];
  }
}

// logits f32 [B*P] vs target rows (dataset f32 [N, P] gathered by rows):
// BCE (logit form, -100 log clamp) partials + dlogits (bf16) for the decoder.
__global__ void __launch_bounds__(256) bce_logits_k(const float* logits, const float* X, const int* rows, int B,
                                                    int P, __bf16* dlog, float* recon, float* part) {
  __shared__ float scratch[16];
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f;
  if (e < (long long)B * P) {
    const int i = (int)(e / P), j = (int)(e - (long long)i * P);
    const float t = logits[e];
    const float x = X[(size_t)(rows ? rows[i] : i) * P + j];
    const float p = 1.f / (1.f + expf(-t));
    if (dlog) dlog[e] = (__bf16)(p - x);
    if (recon) recon[e] = p;
    const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
    loss = x * fminf(sp_pos - t, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
  }
  const float s = block_sum(loss, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// Sum loss partials -> loss ring; advance step (optionally cursor).
__global__ void __launch_bounds__(256) conv_loss_finalize_k(const float* bce_part, int nb, const float* kld_part, int nk,
                                                            TrainState* st, const HParams* hp, int advance_cursor) {
  __shared__ float scratch[16];
  float sb = 0.f, sk = 0.f;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) sb += bce_part[i];
  for (int i = threadIdx.x; i < nk; i += blockDim.x) sk += kld_part[i];
  const float bce = block_sum(sb, scratch);
  __syncthreads();
  const float kld = block_sum(sk, scratch);
  if (threadIdx.x == 0) {
    const float loss = bce + hp->kl_beta * kld;
    st->loss_hist[(st->step - 1) % kLossHist] = loss;
    st->epoch_loss += (double)loss;
    st->epoch_count += 1.0;
    if (advance_cursor) {
      int c = st->cursor + 1;
      if (st->nbatches > 0 && c >= st->nbatches) c = 0;
      st->cursor = c;
    }
  }
}

// step++ and the Adam beta^t running products (first launch of a step).
__global__ void step_begin_k(TrainState* st, const HParams* hp) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st->step = st->step + 1;
    st->b1pow *= hp->beta1_d;
    st->b2pow *= hp->beta2_d;
  }
}

// --------------------------------------------------- fused Adam + casts ----
// One launch over every parameter segment: Adam on the fp32 master, then the
// bf16 compute copy (same layout) and, for conv weights, the bf16 transpose
// [Cin][KH][KW][Cout] used by conv_dgrad. seg table: {offset, numel, co, taps,
// ci, t_offset (or -1)} per segment; blocks are dealt round-robin.
struct AdamSeg {
  long long off, numel;
  int co, taps, ci;
  long long toff;  // offset of the transposed copy in w16t, -1 if none
};

__global__ void __launch_bounds__(256) adam_cast_k(float* P, const float* G, float* Mo, float* Vo, __bf16* w16,
                                                   __bf16* w16t, const AdamSeg* segs, int nseg,
                                                   const TrainState* st, const HParams* hp, int do_adam) {
  __shared__ AdamC cs;
  const AdamC c = adam_consts_block(st, hp, &cs);
  for (int s = 0; s < nseg; ++s) {
    const AdamSeg sg = segs[s];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < sg.numel;
         i += (long long)gridDim.x * blockDim.x) {
      const long long o = sg.off + i;
      float p = P[o];
      if (do_adam) {
        float m = Mo[o], v = Vo[o];
        adam_update(p, m, v, G[o], c);
        P[o] = p; Mo[o] = m; Vo[o] = v;
      }
      const __bf16 pb = (__bf16)p;
      w16[o] = pb;
      if (sg.toff >= 0) {
        const int per = sg.taps * sg.ci;
        const int co = (int)(i / per);
        const int rem = (int)(i - (long long)co * per);
        const int tap = rem / sg.ci, ci = rem - tap * sg.ci;
        w16t[sg.toff + ((long long)ci * sg.taps + tap) * sg.co + co] = pb;
      }
    }
  }
}

}  // namespace mdt

using namespace mdt;

// ------------------------------------------------------------ host API ----
static inline int cdivh(long long a, long long b) { return (int)((a + b - 1) / b); }

extern "C" int mdt_conv_fwd(const void* X, int x_is_f32, const int* rows, const void* W16, ConvDesc d,
                            const float* bias, int relu, void* y16, float* y32, const void* omask, hipStream_t s) {
  const int K = d.KH * d.KW * d.C;
  if (K % 8) return 1;
  ConvOut o{reinterpret_cast<__bf16*>(y16), y32, bias, relu, reinterpret_cast<const __bf16*>(omask)};
  const long long M = (long long)d.N * d.OH * d.OW;
  const long long tiles = ((M + 15) / 16) * ((d.CO + 15) / 16);
  const bool vec = (d.C % 8) == 0;
  const bool deep = K >= 512;  // split K over 8 waves for deep reductions
  const int tpb = deep ? 1 : 8;
  dim3 grid(cdivh(tiles, tpb)), blk(kCThreads);
  const __bf16* W = reinterpret_cast<const __bf16*>(W16);
#define LAUNCH_FWD(T, V, TP) \
  hipLaunchKernelGGL((conv_fwd_k<T, V, TP>), grid, blk, 0, s, reinterpret_cast<const T*>(X), rows, W, d, o)
  if (x_is_f32) {
    if (vec) { if (deep) LAUNCH_FWD(float, true, 1); else LAUNCH_FWD(float, true, 8); }
    else { if (deep) LAUNCH_FWD(float, false, 1); else LAUNCH_FWD(float, false, 8); }
  } else {
    if (vec) { if (deep) LAUNCH_FWD(__bf16, true, 1); else LAUNCH_FWD(__bf16, true, 8); }
    else { if (deep) LAUNCH_FWD(__bf16, false, 1); else LAUNCH_FWD(__bf16, false, 8); }
  }
#undef LAUNCH_FWD
  return (int)hipGetLastError();
}

extern "C" int mdt_conv_dgrad(const void* G16, const void* mask16, const void* Wt16, ConvDesc d, const float* bias,
                              int relu, void* y16, float* y32, const void* omask, hipStream_t s) {
  const int K = d.KH * d.KW * d.CO;
  if (K % 8) return 1;
  ConvOut o{reinterpret_cast<__bf16*>(y16), y32, bias, relu, reinterpret_cast<const __bf16*>(omask)};
  const long long M = (long long)d.N * d.H * d.W;
  const long long tiles = ((M + 15) / 16) * ((d.C + 15) / 16);
  const bool vec = (d.CO % 8) == 0;
  const bool deep = K >= 512;
  const int tpb = deep ? 1 : 8;
  dim3 grid(cdivh(tiles, tpb)), blk(kCThreads);
  const __bf16* G = reinterpret_cast<const __bf16*>(G16);
  const __bf16* mk = reinterpret_cast<const __bf16*>(mask16);
  const __bf16* W = reinterpret_cast<const __bf16*>(Wt16);
  if (vec) {
    if (deep) hipLaunchKernelGGL((conv_dgrad_k<true, 1>), grid, blk, 0, s, G, mk, W, d, o);
    else hipLaunchKernelGGL((conv_dgrad_k<true, 8>), grid, blk, 0, s, G, mk, W, d, o);
  } else {
    if (deep) hipLaunchKernelGGL((conv_dgrad_k<false, 1>), grid, blk, 0, s, G, mk, W, d, o);
    else hipLaunchKernelGGL((conv_dgrad_k<false, 8>), grid, blk, 0, s, G, mk, W, d, o);
  }
  return (int)hipGetLastError();
}

extern "C" int mdt_conv_wgrad(const void* G16, const void* mask16, const void* X, int x_is_f32, const int* rows,
                              ConvDesc d, float* dW, float* db, hipStream_t s) {
  const int K2 = d.KH * d.KW * d.C;
  const long long M = (long long)d.N * d.OH * d.OW;
  const int tiles = cdivh(d.CO, 16) * cdivh(K2, 16);
  // enough m-slices that every wave owns a few 32-deep chunks and the grid
  // covers the chip (>= ~512 blocks when the reduction is long)
  const int nch = cdivh(M, 32);
  int msplit = cdivh(nch, 4 * kCW);
  const int cap = tiles >= 512 ? 1 : cdivh(1024, tiles);
  if (msplit > cap) msplit = cap;
  if (msplit < 1) msplit = 1;
  dim3 grid(tiles * msplit), blk(kCThreads);
  const __bf16* G = reinterpret_cast<const __bf16*>(G16);
  const __bf16* mk = reinterpret_cast<const __bf16*>(mask16);
  if (x_is_f32)
    hipLaunchKernelGGL((conv_wgrad_k<float>), grid, blk, 0, s, G, mk, reinterpret_cast<const float*>(X), rows, d,
                       dW, db, msplit);
  else
    hipLaunchKernelGGL((conv_wgrad_k<__bf16>), grid, blk, 0, s, G, mk, reinterpret_cast<const __bf16*>(X), rows, d,
                       dW, db, msplit);
  return (int)hipGetLastError();
}

extern "C" int mdt_chan_sum(const void* G16, int M, int C, float* db, hipStream_t s) {
  dim3 grid(cdivh(M, 4 * 64) > 256 ? 256 : cdivh(M, 4 * 64), cdivh(C, 64));
  hipLaunchKernelGGL(chan_sum_k, grid, dim3(256), 0, s, reinterpret_cast<const __bf16*>(G16), M, C, db);
  return (int)hipGetLastError();
}

extern "C" int mdt_reparam(const float* mulv, float* eps, void* z16, float* z32, int B, int Z, const void* st,
                           const void* hp, unsigned stream, float* kld_part, hipStream_t s) {
  hipLaunchKernelGGL(reparam_k, dim3(cdivh((long long)B * Z, 256)), dim3(256), 0, s, mulv, eps,
                     reinterpret_cast<__bf16*>(z16), z32, B, Z, reinterpret_cast<const TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp), (uint32_t)stream, kld_part);
  return (int)hipGetLastError();
}

extern "C" int mdt_reparam_bwd(const float* dz, const float* mulv, const float* eps, float* dmulv, void* dmulv16,
                               int B, int Z, const void* hp, hipStream_t s) {
  hipLaunchKernelGGL(reparam_bwd_k, dim3(cdivh((long long)B * Z, 256)), dim3(256), 0, s, dz, mulv, eps, dmulv,
                     reinterpret_cast<__bf16*>(dmulv16), B, Z, reinterpret_cast<const HParams*>(hp));
  return (int)hipGetLastError();
}

extern "C" int mdt_gather_rows(const float* X, const int* idx, const void* st, int B, int M, int P, float* xb,
                               hipStream_t s) {
  if (P % 4) return 1;
  int blocks = cdivh((long long)M * (P / 4), 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(gather_rows_k, dim3(blocks), dim3(256), 0, s, X, idx, reinterpret_cast<const TrainState*>(st),
                     B, M, P, xb);
  return (int)hipGetLastError();
}

extern "C" int mdt_bce_logits(const float* logits, const float* X, const int* rows, int B, int P, void* dlog16,
                              float* recon, float* part, hipStream_t s) {
  hipLaunchKernelGGL(bce_logits_k, dim3(cdivh((long long)B * P, 256)), dim3(256), 0, s, logits, X, rows, B, P,
                     reinterpret_cast<__bf16*>(dlog16), recon, part);
  return (int)hipGetLastError();
}

extern "C" int mdt_conv_loss_finalize(const float* bce_part, int nb, const float* kld_part, int nk, void* st,
                                      const void* hp, int advance_cursor, hipStream_t s) {
  hipLaunchKernelGGL(conv_loss_finalize_k, dim3(1), dim3(256), 0, s, bce_part, nb, kld_part, nk,
                     reinterpret_cast<TrainState*>(st), reinterpret_cast<const HParams*>(hp), advance_cursor);
  return (int)hipGetLastError();
}

extern "C" int mdt_step_begin(void* st, const void* hp, hipStream_t s) {
  hipLaunchKernelGGL(step_begin_k, dim3(1), dim3(64), 0, s, reinterpret_cast<TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp));
  return (int)hipGetLastError();
}

extern "C" int mdt_adam_cast(float* P, const float* G, float* Mo, float* Vo, void* w16, void* w16t,
                             const void* segs, int nseg, long long total, const void* st, const void* hp, int do_adam,
                             hipStream_t s) {
  int blocks = cdivh(total, 256 * 4);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_cast_k, dim3(blocks), dim3(256), 0, s, P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16),
                     reinterpret_cast<__bf16*>(w16t), reinterpret_cast<const AdamSeg*>(segs), nseg,
                     reinterpret_cast<const TrainState*>(st), reinterpret_cast<const HParams*>(hp), do_adam);
  return (int)hipGetLastError();
}
