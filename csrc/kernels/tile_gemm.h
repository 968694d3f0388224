// Latency-oriented exact-f32 MFMA tile GEMM building blocks for skinny
// training GEMMs (M = batch = 128, N/K in {20, 40, 400, 784}).
//
// Design (MI355X-first, see docs/KERNELS.md):
//  * one wave owns one 16x16 output tile (or NT tiles sharing the A operand)
//    and runs v_mfma_f32_16x16x4_f32 (exact f32: same numerics class as the
//    reference's fp32 addmm);
//  * the k axis is consumed 16 at a time: lane (r = l&15, q = l>>4) holds
//    A(i0+r, k0+4q .. +3) and B(k0+4q .. +3, j0+r), which feed four MFMAs
//    whose local k index q maps to global k = k0 + 4q + t. Contiguous-k
//    operands load as one dwordx4 per lane;
//  * the whole step is L2/MALL resident (< 12 MB), so time is set by load
//    LATENCY (~870 cycles to MALL, measured by obs/probe.py), not bandwidth:
//    a wave issues the loads of all NCW k-chunks it owns back to back (one
//    round trip), then runs the MFMAs. The chunk loop has a compile-time trip
//    count and no branches: out-of-range chunks / rows / columns load a
//    clamped in-bounds address and are zeroed by a 0/1 multiplier, so hipcc
//    never branches around a load (cdna_hip_programming.md §5 trap (c));
//  * KSPLIT waves share a tile (split-K over waves, combined through LDS) so
//    a 128-row problem spreads over ~200 workgroups, one load round each;
//  * no __syncthreads() after global stores anywhere on the hot path: on
//    gfx950 the barrier's implied vmcnt(0) waits for store acknowledgements
//    (measured ~3 us with obs/stamps.py), so reductions go through per-wave
//    partial slots instead.
#pragma once
#include "common.h"

namespace mdt {


struct Frag {  // a lane's bound operand row/column
  const float* base;
  float mask;
};

// ----------------------------- A operand loaders ---------------------------
// A(i, k): row(i) binds the lane's row; load(f, k0, m, o) -> m * A(i, k0..k0+3).

struct ARowMajor {  // A(i,k) = p[i*ld + k]  (k contiguous; K % 4 == 0)
  const float* p; int ld, M, K;
  __device__ __forceinline__ Frag row(int i) const {
    return {p + (size_t)min(i, M - 1) * ld, i < M ? 1.f : 0.f};
  }
  __device__ __forceinline__ void load(const Frag& f, int k0, float m, float o[4]) const {
    const float4 v = *reinterpret_cast<const float4*>(f.base + min(k0, K - 4));
    m = (k0 < K) ? m * f.mask : 0.f;
    o[0] = v.x * m; o[1] = v.y * m; o[2] = v.z * m; o[3] = v.w * m;
  }
};

struct ARowGather {  // A(i,k) = p[rows[i]*ld + k]  (sampler-indexed batch rows)
  const float* p; const int* rows; int ld, M, K;
  __device__ __forceinline__ Frag row(int i) const {
    return {p + (size_t)rows[min(i, M - 1)] * ld, i < M ? 1.f : 0.f};
  }
  __device__ __forceinline__ void load(const Frag& f, int k0, float m, float o[4]) const {
    const float4 v = *reinterpret_cast<const float4*>(f.base + min(k0, K - 4));
    m = (k0 < K) ? m * f.mask : 0.f;
    o[0] = v.x * m; o[1] = v.y * m; o[2] = v.z * m; o[3] = v.w * m;
  }
};

struct ATrans {  // A(i,k) = p[k*ld + i]  (i contiguous: dY^T in weight grads)
  const float* p; int ld, M, K;
  // single element for the 32x32x2 path: lanes of equal k read 128 contiguous bytes
  __device__ __forceinline__ float load1(const Frag& f, int k, float m) const {
    return f.base[(size_t)min(k, K - 1) * ld] * (k < K ? m * f.mask : 0.f);
  }
  __device__ __forceinline__ Frag row(int i) const { return {p + min(i, M - 1), i < M ? 1.f : 0.f}; }
  __device__ __forceinline__ void load(const Frag& f, int k0, float m, float o[4]) const {
    m *= f.mask;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = k0 + t;
      o[t] = f.base[(size_t)min(k, K - 1) * ld] * (k < K ? m : 0.f);
    }
  }
};

// ----------------------------- B operand loaders ---------------------------
// B(k, j): col(j) binds the lane's column; load(f, k0, o) -> B(k0..k0+3, j).

struct BWeightNT {  // B(k,j) = W[j*ld + k]  (torch Linear weight [N,K]; K % 4 == 0)
  const float* p; int ld, N, K;
  __device__ __forceinline__ Frag col(int j) const {
    return {p + (size_t)min(j, N - 1) * ld, j < N ? 1.f : 0.f};
  }
  __device__ __forceinline__ void load(const Frag& f, int k0, float o[4]) const {
    const float4 v = *reinterpret_cast<const float4*>(f.base + min(k0, K - 4));
    const float m = k0 < K ? f.mask : 0.f;
    o[0] = v.x * m; o[1] = v.y * m; o[2] = v.z * m; o[3] = v.w * m;
  }
};

struct BRowMajor {  // B(k,j) = p[k*ld + j]  (j contiguous)
  const float* p; int ld, N, K;
  __device__ __forceinline__ float load1(const Frag& f, int k) const {
    return f.base[(size_t)min(k, K - 1) * ld] * (k < K ? f.mask : 0.f);
  }
  __device__ __forceinline__ Frag col(int j) const { return {p + min(j, N - 1), j < N ? 1.f : 0.f}; }
  __device__ __forceinline__ void load(const Frag& f, int k0, float o[4]) const {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = k0 + t;
      o[t] = f.base[(size_t)min(k, K - 1) * ld] * (k < K ? f.mask : 0.f);
    }
  }
};

// NT tiles (rows i0.., columns j0 + t*jstride) over k-chunks [kc0, kc1), at
// most NCW chunks per round; the A fragment is shared by the NT tiles.
// Rounds are uniform (wave-level) and usually exactly one. With ROWSUM the
// lane also accumulates sum_k A(i0 + (lane&15), k) over ITS k values (the
// caller reduces across the 4 lane quarters): bias gradients for free.
template <int NT, int NCW, bool ROWSUM = false, class AL, class BL>
__device__ __forceinline__ void wave_tiles(const AL& A, const BL& B, int i0, int j0, int jstride,
                                           int kc0, int kc1, f32x4 (&acc)[NT], float* rowsum = nullptr) {
  const int lane = lane_id();
  const int r = lane & 15, q = lane >> 4;
  const Frag fa = A.row(i0 + r);
  Frag fb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) fb[t] = B.col(j0 + t * jstride + r);
  f32x4 acc2[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc2[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float rs = 0.f;
  for (int kc = kc0; kc < kc1; kc += NCW) {
    float a[NCW][4], b[NT][NCW][4];
#pragma unroll
    for (int u = 0; u < NCW; ++u) {
      const int c = kc + u;
      const int k0 = min(c, kc1 - 1) * 16 + 4 * q;
      A.load(fa, k0, c < kc1 ? 1.f : 0.f, a[u]);
#pragma unroll
      for (int t = 0; t < NT; ++t) B.load(fb[t], k0, b[t][u]);
    }
    // every load of the round is issued before the first MFMA waits: left
    // alone the scheduler sinks the later chunks' loads between the MFMAs,
    // each behind its own vmcnt(0) (one round trip per chunk)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < NCW; ++u) {
      if constexpr (ROWSUM) rs += (a[u][0] + a[u][1]) + (a[u][2] + a[u][3]);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        acc[t] = mfma16x16x4(a[u][0], b[t][u][0], acc[t]);
        acc2[t] = mfma16x16x4(a[u][1], b[t][u][1], acc2[t]);
        acc[t] = mfma16x16x4(a[u][2], b[t][u][2], acc[t]);
        acc2[t] = mfma16x16x4(a[u][3], b[t][u][3], acc2[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] += acc2[t];
  if constexpr (ROWSUM) {
    rs += __shfl_xor(rs, 16, 64);
    rs += __shfl_xor(rs, 32, 64);
    *rowsum = rs;
  }
}

template <int NCW, class AL, class BL>
__device__ __forceinline__ f32x4 wave_tile(const AL& A, const BL& B, int i0, int j0, int kc0, int kc1) {
  f32x4 acc[1];
  wave_tiles<1, NCW>(A, B, i0, j0, 0, kc0, kc1, acc);
  return acc[0];
}

// Block of WAVES waves over a tiled problem. A wave job = (row tile ti, group
// of NT adjacent 16-column tiles). TPB jobs per block, KSPLIT = WAVES/TPB
// waves per job (split-K combined through LDS). Epilogue: a functor with
// `template <int N> float run(const int (&rows)[N], int col, const float (&v)[N])`
// called once per fragment column (all loads issued before any store, so the
// fragment costs one memory round trip), and with ROWSUM (KSPLIT == 1 only)
// run<1>({i}, -1, {rowsum}) once per row from the jobs of column group 0. Returns the wave's summed epilogue
// contributions (leader waves only). `lds` must hold WAVES*256 floats; the
// only barrier precedes every store.
template <int WAVES, int TPB, int NT, int NCW, bool ROWSUM, class AL, class BL, class EPI>
__device__ __forceinline__ float gemm_tiles(const AL& A, const BL& B, EPI& epi, int K, int tiles_i,
                                            int tiles_j, int blk, float* lds) {
  constexpr int KSPLIT = WAVES / TPB;
  static_assert(KSPLIT * TPB == WAVES, "WAVES must be a multiple of TPB");
  static_assert(!ROWSUM || KSPLIT == 1, "ROWSUM needs whole-K waves");
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  const int lane = lane_id();
  const int groups_j = (tiles_j + NT - 1) / NT;
  const int njobs = tiles_i * groups_j;
  const int job = blk * TPB + w / KSPLIT;
  const int ks = w % KSPLIT;
  const int nch = (K + 15) >> 4;
  const int kc0 = (ks * nch) / KSPLIT, kc1 = ((ks + 1) * nch) / KSPLIT;
  const bool live = job < njobs;
  const int jj = live ? job : njobs - 1;  // dead waves compute a real job, never store it
  const int ti = jj / groups_j;
  const int tg = jj - ti * groups_j;
  f32x4 acc[NT];
  float rs = 0.f;
  wave_tiles<NT, NCW, ROWSUM>(A, B, ti * 16, tg * NT * 16, 16, kc0, kc1, acc, &rs);
  if constexpr (KSPLIT > 1) {
    // split-K combine + epilogue spread over the tile's waves: wave ks sums
    // (in wave order, the same additions as one wave summing all four) and
    // finishes VPW of the lane's four rows, so no single wave carries the
    // whole epilogue's load round trip and stores
    static_assert(NT == 1, "split-K reduction implemented for NT == 1");
    constexpr int VPW = KSPLIT >= 4 ? 1 : 4 / KSPLIT;
    *reinterpret_cast<f32x4*>(lds + w * 256 + lane * 4) = acc[0];
    __syncthreads();
    float contrib = 0.f;
    if (live && ks < 4 / VPW) {
      const float* base = lds + (w - ks) * 256 + lane * 4 + ks * VPW;
      const int row0 = ti * 16 + 4 * (lane >> 4) + ks * VPW;
      int rows[VPW];
      float v[VPW];
#pragma unroll
      for (int u = 0; u < VPW; ++u) {
        float t = base[u];
#pragma unroll
        for (int s = 1; s < KSPLIT; ++s) t += base[s * 256 + u];
        v[u] = t;
        rows[u] = row0 + u;
      }
      contrib = epi.template run<VPW>(rows, tg * 16 + (lane & 15), v);
    }
    return contrib;
  }
  float contrib = 0.f;
  if (live && ks == 0) {
    const int row0 = ti * 16 + 4 * (lane >> 4);
    const int rows[4] = {row0, row0 + 1, row0 + 2, row0 + 3};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = (tg * NT + t) * 16 + (lane & 15);
      const float v[4] = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
      contrib += epi.template run<4>(rows, col, v);
    }
    if constexpr (ROWSUM) {
      if (tg == 0 && (lane >> 4) == 0) {
        const int rr[1] = {ti * 16 + (lane & 15)};
        const float vv[1] = {rs};
        contrib += epi.template run<1>(rr, -1, vv);
      }
    }
  }
  return contrib;
}

// ---------------------------------------------------------------------------
// Weight-gradient GEMMs dW[i, j] = sum_k A(i, k) B(k, j) with k = batch: both
// operands are batch-major (k is the SLOW index), so 16x16x4 fragments would
// need 4 strided dword loads per chunk. v_mfma_f32_32x32x2_f32 takes ONE f32
// per operand per lane with lanes 0-31 spanning i (resp. j) at fixed k: every
// load instruction reads two fully used 128-byte rows. A wave owns a 32x32
// tile over a k-slice of NPW pairs (2 k per MFMA); KSPLIT waves per tile are
// combined through LDS. With ROWSUM the A values give the bias row sums.
template <int NPW, bool ROWSUM, class AL, class BL>
__device__ __forceinline__ f32x16 wave_tile32(const AL& A, const BL& B, int i0, int j0, int kp0, int kp1,
                                              float* rowsum) {
  const int lane = lane_id();
  const int r = lane & 31, h = lane >> 5;
  const Frag fa = A.row(i0 + r);
  const Frag fb = B.col(j0 + r);
  f32x16 acc0 = {}, acc1 = {};
  float rs = 0.f;
  for (int kp = kp0; kp < kp1; kp += NPW) {
    float a[NPW], b[NPW];
#pragma unroll
    for (int u = 0; u < NPW; ++u) {
      const int p = kp + u;
      const int k = min(p, kp1 - 1) * 2 + h;
      a[u] = A.load1(fa, k, p < kp1 ? 1.f : 0.f);
      b[u] = B.load1(fb, k);
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads of the round first (see wave_tiles)
#pragma unroll
    for (int u = 0; u < NPW; u += 2) {
      acc0 = mfma32x32x2(a[u], b[u], acc0);
      if (u + 1 < NPW) acc1 = mfma32x32x2(a[u + 1], b[u + 1], acc1);
    }
    if constexpr (ROWSUM) {
#pragma unroll
      for (int u = 0; u < NPW; ++u) rs += a[u];
    }
  }
  if constexpr (ROWSUM) {
    rs += __shfl_xor(rs, 32, 64);
    *rowsum = rs;
  }
  return acc0 + acc1;
}

// Block of WAVES waves: TPB 32x32 tiles per block, KSPLIT = WAVES/TPB waves
// per tile. Epilogue run<16>(rows, col, v) per lane (see gemm_tiles); with
// ROWSUM run<1>({i}, -1, {rowsum}) from the tiles of column 0. `lds` must hold WAVES*1024 floats.
// `stamp` (profiling only, obs/stamps.py): the wave's stamp row; slots 2 and 3
// get the time after the wave's GEMM and after the combine barrier.
__device__ __forceinline__ void stamp_at(unsigned long long* row, int slot) {
  if (row && lane_id() == 0) row[slot] = __builtin_amdgcn_s_memrealtime();
}

template <int WAVES, int TPB, int NPW, bool ROWSUM, class AL, class BL, class EPI>
__device__ __forceinline__ void gemm_tiles32(const AL& A, const BL& B, EPI& epi, int K, int tiles_i,
                                             int tiles_j, int blk, float* lds,
                                             unsigned long long* stamp = nullptr) {
  constexpr int KSPLIT = WAVES / TPB;
  static_assert(KSPLIT * TPB == WAVES, "WAVES must be a multiple of TPB");
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  const int lane = lane_id();
  const int ntiles = tiles_i * tiles_j;
  const int tile = blk * TPB + w / KSPLIT;
  const int ks = w % KSPLIT;
  const int npairs = (K + 1) >> 1;
  const int kp0 = (ks * npairs) / KSPLIT, kp1 = ((ks + 1) * npairs) / KSPLIT;
  const bool live = tile < ntiles;
  const int tt = live ? tile : ntiles - 1;
  const int ti = tt / tiles_j, tj = tt - ti * tiles_j;
  float rs = 0.f;
  f32x16 acc = wave_tile32<NPW, ROWSUM>(A, B, ti * 32, tj * 32, kp0, kp1, &rs);
  if constexpr (KSPLIT > 1) {
    // combine + epilogue spread over the tile's KSPLIT waves (see gemm_tiles):
    // wave ks sums values [ks*VPW, +VPW) of the lane's 16 in wave order and
    // runs their epilogue (a weight-gradient + Adam epilogue is 3 loads and
    // 4 stores per value: one wave doing all 16 doubled the block's time)
    static_assert(16 % KSPLIT == 0, "KSPLIT must divide the 16 values per lane");
    constexpr int VPW = 16 / KSPLIT;
    float* mine = lds + w * 1024 + lane * 16;
#pragma unroll
    for (int v = 0; v < 16; v += 4) *reinterpret_cast<f32x4*>(mine + v) = f32x4{acc[v], acc[v + 1], acc[v + 2], acc[v + 3]};
    if constexpr (ROWSUM) lds[WAVES * 1024 + w * 64 + lane] = rs;
    __syncthreads();
    if (!live) return;
    const float* base = lds + (w - ks) * 1024 + lane * 16 + ks * VPW;
    const int col = tj * 32 + (lane & 31);
    const int rb = ti * 32 + 4 * (lane >> 5);
    int rows[VPW];
    float vals[VPW];
#pragma unroll
    for (int u = 0; u < VPW; ++u) {
      float t = base[u];
#pragma unroll
      for (int s = 1; s < KSPLIT; ++s) t += base[s * 1024 + u];
      const int v = ks * VPW + u;
      vals[u] = t;
      rows[u] = rb + (v & 3) + 8 * (v >> 2);
    }
    epi.template run<VPW>(rows, col, vals);
    if constexpr (ROWSUM) {
      if (ks == 0 && tj == 0 && (lane >> 5) == 0) {
#pragma unroll
        for (int s = 1; s < KSPLIT; ++s) rs += lds[WAVES * 1024 + (w + s) * 64 + lane];
        const int rr[1] = {ti * 32 + lane};
        const float vv[1] = {rs};
        epi.template run<1>(rr, -1, vv);
      }
    }
    return;
  }
  if (live && ks == 0) {
    const int col = tj * 32 + (lane & 31);
    const int rb = ti * 32 + 4 * (lane >> 5);
    int rows[16];
    float vals[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      rows[v] = rb + (v & 3) + 8 * (v >> 2);
      vals[v] = acc[v];
    }
    epi.template run<16>(rows, col, vals);
    if constexpr (ROWSUM) {
      if (tj == 0 && (lane >> 5) == 0) {
        const int rr[1] = {ti * 32 + lane};
        const float vv[1] = {rs};
        epi.template run<1>(rr, -1, vv);
      }
    }
  }
}

}  // namespace mdt
