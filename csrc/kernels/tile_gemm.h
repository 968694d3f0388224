// Latency-oriented exact-f32 MFMA tile GEMM building blocks for skinny
// training GEMMs (M = batch = 128, N/K in {20, 40, 400, 784}).
//
// Design (MI355X-first, see docs/KERNELS.md):
//  * one wave owns one 16x16 output tile and runs v_mfma_f32_16x16x4_f32
//    (exact f32, same numerics class as the reference's fp32 addmm);
//  * the k axis is consumed 16 at a time: lane (r = l&15, q = l>>4) loads
//    A(i0+r, k0+4q .. +3) and B(k0+4q .. +3, j0+r), which feed four MFMAs
//    whose local k index q maps to global k = k0 + 4q + t. Contiguous-k
//    operands load as one dwordx4 per lane;
//  * two accumulators alternate so the 40-cycle dependent MFMA latency hides
//    behind the 32-cycle issue interval;
//  * operands are L2/MALL-resident (the whole MLP-VAE step touches < 12 MB),
//    so LDS staging would only add a round trip: the loads go straight to
//    VGPRs and the next k-chunk is prefetched in registers;
//  * a block is 4 waves; KSPLIT waves share a tile (split-K, reduced through
//    LDS) so small-N problems still put >= 200 workgroups on the 256 CUs.
#pragma once
#include "common.h"

namespace mdt {

// ----------------------------- A operand loaders ---------------------------
// A(i, k). `row(i)` binds the lane's row once; `load(c, k0, out)` fetches
// A(i, k0..k0+3) with zero fill outside [0,M) x [0,K).

struct ARowMajor {  // A(i,k) = p[i*ld + k]     (k contiguous)
  const float* p; int ld, M, K;
  __device__ __forceinline__ const float* row(int i) const { return i < M ? p + (size_t)i * ld : nullptr; }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
    if (c && k0 + 3 < K) {
      const float4 v = *reinterpret_cast<const float4*>(c + k0);
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[k0 + t] : 0.f;
    }
  }
};

struct ARowGather {  // A(i,k) = p[rows[i]*ld + k]  (sampler-indexed batch rows)
  const float* p; const int* rows; int ld, M, K;
  __device__ __forceinline__ const float* row(int i) const {
    return i < M ? p + (size_t)rows[i] * ld : nullptr;
  }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
    if (c && k0 + 3 < K) {
      const float4 v = *reinterpret_cast<const float4*>(c + k0);
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[k0 + t] : 0.f;
    }
  }
};

struct ATrans {  // A(i,k) = p[k*ld + i]     (i contiguous: dY^T in weight grads)
  const float* p; int ld, M, K;
  __device__ __forceinline__ const float* row(int i) const { return i < M ? p + i : nullptr; }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[(size_t)(k0 + t) * ld] : 0.f;
  }
};

// ----------------------------- B operand loaders ---------------------------
// B(k, j). `col(j)` binds the lane's column; `load(c, k0, out)` -> B(k0..k0+3, j).

struct BWeightNT {  // B(k,j) = W[j*ld + k]   (torch Linear weight [N,K], forward)
  const float* p; int ld, N, K;
  __device__ __forceinline__ const float* col(int j) const { return j < N ? p + (size_t)j * ld : nullptr; }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
    if (c && k0 + 3 < K) {
      const float4 v = *reinterpret_cast<const float4*>(c + k0);
      o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[k0 + t] : 0.f;
    }
  }
};

struct BRowMajor {  // B(k,j) = p[k*ld + j]   (j contiguous)
  const float* p; int ld, N, K;
  __device__ __forceinline__ const float* col(int j) const { return j < N ? p + j : nullptr; }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[(size_t)(k0 + t) * ld] : 0.f;
  }
};

struct BRowGather {  // B(k,j) = p[rows[k]*ld + j]
  const float* p; const int* rows; int ld, N, K;
  __device__ __forceinline__ const float* col(int j) const { return j < N ? p + j : nullptr; }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? c[(size_t)rows[k0 + t] * ld] : 0.f;
  }
};

struct BOnes {  // B(k,j) = [j == 0] : turns a weight-grad tile into the bias-grad row sum
  int K;
  __device__ __forceinline__ const float* col(int j) const {
    return j == 0 ? reinterpret_cast<const float*>(1) : nullptr;
  }
  __device__ __forceinline__ void load(const float* c, int k0, float o[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) o[t] = (c && k0 + t < K) ? 1.f : 0.f;
  }
};

// One wave: acc(16x16) = sum_{k in chunks [kc0,kc1)} A(i0.., k) B(k, j0..).
template <class AL, class BL>
__device__ __forceinline__ f32x4 wave_tile(const AL& A, const BL& B, int i0, int j0, int kc0, int kc1) {
  const int lane = lane_id();
  const int r = lane & 15, q = lane >> 4;
  const float* ca = A.row(i0 + r);
  const float* cb = B.col(j0 + r);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
  if (kc0 >= kc1) return acc0;
  float a[4], b[4];
  A.load(ca, kc0 * 16 + 4 * q, a);
  B.load(cb, kc0 * 16 + 4 * q, b);
  for (int kc = kc0; kc < kc1; ++kc) {
    float an[4], bn[4];
    const bool more = kc + 1 < kc1;
    if (more) {
      A.load(ca, (kc + 1) * 16 + 4 * q, an);
      B.load(cb, (kc + 1) * 16 + 4 * q, bn);
    }
    acc0 = mfma16x16x4(a[0], b[0], acc0);
    acc1 = mfma16x16x4(a[1], b[1], acc1);
    acc0 = mfma16x16x4(a[2], b[2], acc0);
    acc1 = mfma16x16x4(a[3], b[3], acc1);
    if (more) {
#pragma unroll
      for (int t = 0; t < 4; ++t) { a[t] = an[t]; b[t] = bn[t]; }
    }
  }
  return acc0 + acc1;
}

// Block of 4 waves over a tiled problem. TPB tiles per block, KSPLIT = 4/TPB
// waves per tile. Tile t -> (ti, tj) row-major over tiles_j columns; when
// `bias_tj >= 0` the tile column `bias_tj` is a bias-grad column computed with
// BOnes. Epilogue signature: float epi(i, j, v, is_bias) -> contribution to a
// block-level sum (returned in wave 0 lane 0 by the caller's reduction).
// `lds` must hold 4*256 floats.
template <int TPB, class AL, class BL, class EPI>
__device__ __forceinline__ float gemm_tiles(const AL& A, const BL& B, EPI& epi, int K, int tiles_i,
                                            int tiles_j, int bias_tj, int blk, float* lds) {
  constexpr int KSPLIT = 4 / TPB;
  const int w = wave_id();
  const int lane = lane_id();
  const int tile = blk * TPB + w / KSPLIT;
  const int ks = w % KSPLIT;
  const int ntiles = tiles_i * tiles_j;
  const int nch = (K + 15) >> 4;
  const int kc0 = (ks * nch) / KSPLIT, kc1 = ((ks + 1) * nch) / KSPLIT;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int ti = 0, tj = 0;
  const bool live = tile < ntiles;
  if (live) {
    ti = tile / tiles_j;
    tj = tile - ti * tiles_j;
    if (tj == bias_tj) acc = wave_tile(A, BOnes{K}, ti * 16, 0, kc0, kc1);
    else acc = wave_tile(A, B, ti * 16, tj * 16, kc0, kc1);
  }
  if constexpr (KSPLIT > 1) {
    float* mine = lds + w * 256 + lane * 4;
    mine[0] = acc[0]; mine[1] = acc[1]; mine[2] = acc[2]; mine[3] = acc[3];
    __syncthreads();
    if (ks == 0) {
#pragma unroll
      for (int s = 1; s < KSPLIT; ++s) {
        const float* o = lds + (w + s) * 256 + lane * 4;
        acc[0] += o[0]; acc[1] += o[1]; acc[2] += o[2]; acc[3] += o[3];
      }
    }
  }
  float contrib = 0.f;
  if (live && ks == 0) {
    const bool is_bias = (tj == bias_tj);
    const int col = (is_bias ? 0 : tj * 16) + (lane & 15);
    const int row0 = ti * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int r = 0; r < 4; ++r) contrib += epi(row0 + r, col, acc[r], is_bias);
  }
  return contrib;
}

}  // namespace mdt
