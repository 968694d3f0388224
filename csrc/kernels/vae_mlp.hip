// Fused MLP-VAE training step for MI355X (gfx950).
//
// Model (parity: /root/reference/vae-hpo.py:19-58): fc1 D->H, fc21/fc22 H->Z,
// fc3 Z->H, fc4 H->D, ELBO = BCE(sum) + beta*KLD. The whole step is six
// launches (captured in one hipGraph by the runtime), 512-thread workgroups:
//
//   F1  h1 = relu(X[rows] W1^T + b1) ; copy batch rows -> xb ; step++
//   F2  [mu|lv] = h1 W2^T + b2 ; z = mu + eps*exp(lv/2) (Philox) ; KLD partial ;
//       h3 = relu(z W3^T + b3) ; cursor++                     (16 rows / block)
//   F3  logits = h3 W4^T + b4 ; dlogits = sigmoid - x ; BCE partial (logit form)
//   B1  dh3 = (dlogits W4) . [h3>0] (+ its dz split-K slab)
//   B2  dz = dh3 W3 -> dmu, dlv (reparam + beta-KLD) ; dh1 = ([dmu|dlv] W2) . [h1>0]
//       ||  dW3 = dh3^T z, db3  ||  dW4 = dlogits^T h3, db4  || loss reduction
//   B3  dW2 = [dmu|dlv]^T h1, db2      ||  dW1 = dh1^T xb, db1
//       with fuse_adam: Adam applied in those epilogues, + Adam streamed over
//       the fc3/fc4 slice of the arena (gradients final since B2). Without
//       it (intra-group DDP), the bucketed all-reduce runs on the comm stream
//       and adam.hip updates the whole arena afterwards.
//
// Gradients are written (not accumulated) straight into the flat gradient
// arena: no zero_grad, no bucket copy-back. The batch rows are gathered by
// sampler index inside F1 (no host collate, no H2D copy). The batch cursor
// and step counter are device-resident (see TrainState), so one captured
// graph replays over an entire epoch.
#include "common.h"
#include "tile_gemm.h"
#include "vae_mlp.h"
#include "adam_common.h"

namespace mdt {

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;

__device__ __forceinline__ int cdiv_d(int a, int b) { return (a + b - 1) / b; }

// Phase timestamps for the profiling tool (obs/stamps.py); a null pointer
// (production) costs one uniform branch. Slot 7 holds where the wave ran:
// (XCC id << 16) | HW_ID's CU/SH/SE bits (written with slot 0).
#define STAMP(K, S)                                                                         \
  do {                                                                                      \
    if (a.stamps && lane_id() == 0 && blockIdx.x < kStampBlocks) {                          \
      unsigned long long* sp_ = a.stamps + (((size_t)(K) * kStampBlocks + blockIdx.x) * 8 + wave_id()) * 8; \
      sp_[S] = __builtin_amdgcn_s_memrealtime();                                            \
      if ((S) == 0) {                                                                       \
        unsigned hw_, xcc_;                                                                 \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));                   \
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_));           \
        sp_[7] = ((unsigned long long)xcc_ << 16) | (hw_ & 0xff00u);                        \
      }                                                                                     \
    }                                                                                       \
  } while (0)

// ------------------------------------------------------------------- F1 ----
// Epilogues: `run<N>` receives one lane's N outputs of one column; every load
// is issued before the first store (one round trip per fragment).
struct EpiBiasRelu {
  float* out; const float* bias; int ld, M, N;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= N) return 0.f;
    const float b = bias[j];
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rows[r] < M) out[(size_t)rows[r] * ld + j] = fmaxf(v[r] + b, 0.f);
    return 0.f;
  }
};

// Slab geometry: TH = H/16 slices; [mu|lv] slabs are NTM = ceil(2Z/16) tiles
// wide (SW floats), dz slabs NTZ = ceil(Z/16) tiles (SWZ floats). F2/B2 run
// GROUPS = ceil(TH/8) blocks per row tile, one 16-column output tile per wave.
struct SlabGeo {
  int th, ntm, sw, ntz, swz, groups;
  __device__ __host__ SlabGeo(int H, int Z)
      : th((H + 15) / 16), ntm((2 * Z + 15) / 16), sw(((2 * Z + 15) / 16) * 16), ntz((Z + 15) / 16),
        swz(((Z + 15) / 16) * 16), groups(((H + 15) / 16 + kWaves - 1) / kWaves) {}
};

// Transposes a 16x16 C-layout tile (wave 0's registers: col = lane&15,
// rows 4q..4q+3) into an LDS [row][k] image readable as A fragments.
__device__ __forceinline__ void tile_to_lds(float (*t)[20], const float (&v)[4]) {
  const int lane = lane_id();
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) t[4 * (lane >> 4) + rr][lane & 15] = v[rr];
}

// 16x16 MFMA with A from the LDS tile (k = 16) and a prefetched B fragment.
__device__ __forceinline__ f32x4 lds_tile_mma(float (*t)[20], const float (&b)[4]) {
  const int lane = lane_id();
  const float4 av = *reinterpret_cast<const float4*>(&t[lane & 15][4 * (lane >> 4)]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = mfma16x16x4(av.x, b[0], acc);
  acc = mfma16x16x4(av.y, b[1], acc);
  acc = mfma16x16x4(av.z, b[2], acc);
  acc = mfma16x16x4(av.w, b[3], acc);
  return acc;
}

// One block = one 16x16 tile (ti, tj) of h1, its K = D split over the 8
// waves. The relu'd tile then feeds the encoder head as a split-K slice:
// waves 0..NTM-1 compute slab[ti][tj] = h1[:, tj*16:+16] W2[:, tj*16:+16]^T
// (one 16-deep MFMA chunk each), so F2 only sums TH slabs instead of running
// a 400-deep GEMM on 8 CUs.
__global__ void __launch_bounds__(kThreads) vae_f1(VaeArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kWaves * 256];
  __shared__ __attribute__((aligned(16))) float ht[16][20];
  STAMP(0, 0);
  const SlabGeo geo(a.H, a.Z);
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int tiles_j = geo.th;
  const int ti = blockIdx.x / tiles_j, tj = blockIdx.x - ti * tiles_j;
  const int i0 = ti * 16, j = tj * 16 + (lane & 15);
  const int q = lane >> 4;
  const int Z2 = 2 * a.Z;
  // The cursor heads the launch's one dependent chain (cursor -> batch row
  // index -> image row), so it is loaded first; the bias and the W2 slice of
  // the slab step are prefetched raw and masked only where they are used, so
  // no wait for them lands in front of the GEMM's loads.
  const int cursor = a.st->cursor;
  const float bj = a.b1[min(j, a.H - 1)];
  float4 w2v = {0.f, 0.f, 0.f, 0.f};
  float w2m = 0.f;
  if (w < geo.ntm) {
    const int n = w * 16 + (lane & 15);
    const int k0 = tj * 16 + 4 * q;
    w2v = *reinterpret_cast<const float4*>(a.W2 + (size_t)min(n, Z2 - 1) * a.H + min(k0, a.H - 4));
    w2m = (n < Z2 && k0 < a.H) ? 1.f : 0.f;
  }
  const int* rows = a.idx + (size_t)cursor * a.B;
  ARowGather A{a.X, rows, a.D, a.M, a.D};
  BWeightNT Bw{a.W1, a.D, a.H, a.D};
  const int nch = cdiv_d(a.D, 16);
  const int kc0 = (w * nch) / kWaves, kc1 = ((w + 1) * nch) / kWaves;
  f32x4 acc = wave_tile<7>(A, Bw, i0, tj * 16, kc0, kc1);
  *reinterpret_cast<f32x4*>(lds + w * 256 + lane * 4) = acc;
  __syncthreads();
  float h[4];
  if (w == 0) {
#pragma unroll
    for (int s = 1; s < kWaves; ++s) acc += *reinterpret_cast<const f32x4*>(lds + s * 256 + lane * 4);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) h[rr] = (i0 + 4 * q + rr < a.M && j < a.H) ? fmaxf(acc[rr] + bj, 0.f) : 0.f;
    tile_to_lds(ht, h);
  }
  __syncthreads();
  STAMP(0, 1);
  if (w < geo.ntm) {
    const float wb[4] = {w2v.x * w2m, w2v.y * w2m, w2v.z * w2m, w2v.w * w2m};
    const f32x4 sl = lds_tile_mma(ht, wb);
    float* dst = a.slab_mv + ((size_t)(ti * geo.th + tj) * 16) * geo.sw + w * 16 + (lane & 15);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) dst[(size_t)(4 * q + rr) * geo.sw] = sl[rr];
  }
  if (w == 0 && j < a.H) {
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      if (i0 + 4 * q + rr < a.M) a.h1[(size_t)(i0 + 4 * q + rr) * a.H + j] = h[rr];
  }
  // the TH blocks of a row tile materialise its 16 batch rows into xb for
  // F3/B3, each a 1/TH column slice (L2-hot lines: the block's waves just
  // loaded every column of these rows), on the waves the slab step leaves idle.
  // (Round 4 gave the whole copy to the tile-column-0 blocks: 2.4 us of tail.)
  if (w >= geo.ntm) {
    const int d4 = a.D >> 2;
    const int q0 = (tj * d4) / geo.th, nq = ((tj + 1) * d4) / geo.th - q0;
    for (int e = (w - geo.ntm) * 64 + lane; e < 16 * nq; e += (kWaves - geo.ntm) * 64) {
      const int r = e / nq, k4 = q0 + (e - r * nq);
      const int i = i0 + r;
      if (i < a.M)
        reinterpret_cast<float4*>(a.xb + (size_t)i * a.D)[k4] =
            reinterpret_cast<const float4*>(a.X + (size_t)rows[i] * a.D)[k4];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    TrainState* st = a.st;
    st->step = st->step + 1;
    st->b1pow = st->b1pow * a.hp->beta1_d;
    st->b2pow = st->b2pow * a.hp->beta2_d;
  }
  STAMP(0, 2);
}

// ------------------------------------------------------------------- F2 ----
// Block (row tile ti, group g), 8 waves. Sums the TH [mu|lv] slabs of the row
// tile (two half-sums in LDS), reparameterises (Philox eps, KLD), then wave w
// computes h3 tile g*8+w = relu(z W3^T + b3) with K = Z from LDS. Group 0
// stores mu/lv/eps/z and the KLD partials. All global stores follow the last
// barrier. Requires Z <= 32, Z % 4 == 0, H <= 512.
__global__ void __launch_bounds__(kThreads) vae_f2(VaeArgs a) {
  __shared__ __attribute__((aligned(16))) float part[2][16][64];
  __shared__ __attribute__((aligned(16))) float zt[16][36];
  const SlabGeo geo(a.H, a.Z);
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int ti = blockIdx.x / geo.groups, g = blockIdx.x - ti * geo.groups;
  const int i0 = ti * 16;
  const int Z2 = 2 * a.Z;
  const int q = lane >> 4;
  STAMP(1, 0);
  // prefetch: W3 fragments (K = Z <= 32 -> 2 chunks) and b3 for this wave's tile
  const int jt = g * kWaves + w;
  const int j = jt * 16 + (lane & 15);
  // (raw prefetch, masked where used: no wait in front of the slab loads)
  float4 w3v[2];
  float w3m[2];
  {
    const float* wr = a.W3 + (size_t)min(j, a.H - 1) * a.Z;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int k0 = c * 16 + 4 * q;
      w3v[c] = *reinterpret_cast<const float4*>(wr + min(k0, a.Z - 4));
      w3m[c] = (j < a.H && k0 < a.Z) ? 1.f : 0.f;
    }
  }
  const float bj = a.b3[min(j, a.H - 1)];
  // phase 1: two half-sums over the slabs, float4 per (row, quad)
  {
    const int quads = geo.sw / 4;
    const int pairs = 16 * quads;
    const int t = threadIdx.x;
    if (t < 2 * pairs) {
      const int half = t / pairs, pr = t - half * pairs;
      const int r = pr / quads, cq = pr - r * quads;
      const float4* base = reinterpret_cast<const float4*>(a.slab_mv + ((size_t)(ti * geo.th) * 16 + r) * geo.sw) + cq;
      const size_t sstride = (size_t)16 * geo.sw / 4;
      float4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = base[min(half * 16 + u, geo.th - 1) * sstride];
      __builtin_amdgcn_sched_barrier(0);  // all 16 slab loads in flight before the first add
      float4 acc4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float m = half * 16 + u < geo.th ? 1.f : 0.f;
        acc4.x += v[u].x * m; acc4.y += v[u].y * m; acc4.z += v[u].z * m; acc4.w += v[u].w * m;
      }
      *reinterpret_cast<float4*>(&part[half][r][cq * 4]) = acc4;
    }
  }
  __syncthreads();
  // phase 2: one (row, latent) element per thread (16*Z <= 512)
  const long long stp = a.st->step - 1;  // F1 of this step already incremented it
  const uint32_t step_lo = (uint32_t)((unsigned long long)stp & 0xffffffffu);
  const uint32_t step_hi = (uint32_t)((unsigned long long)stp >> 32);
  const int e = threadIdx.x;
  const int r = e / a.Z, c = e - r * a.Z;
  const int i = i0 + r;
  const bool mine = e < 16 * a.Z;
  const bool valid = mine && i < a.M;
  float mu = 0.f, lv = 0.f, ep = 0.f, zz = 0.f, kld = 0.f;
  if (mine) {
    mu = part[0][r][c] + part[1][r][c] + a.b2[c];
    lv = part[0][r][a.Z + c] + part[1][r][a.Z + c] + a.b2[a.Z + c];
    const float sd = expf(0.5f * lv);
    // counter (row*Z + c, stream, step): replicas of a group differ by
    // `rng_stream` (like per-process randn_like streams in the reference)
    const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(i * a.Z + c), a.rng_stream, step_lo, step_hi},
                                     a.hp->seed_lo, a.hp->seed_hi);
    ep = normal_from_bits(bits.x, bits.y);
    zz = valid ? mu + ep * sd : 0.f;
    kld = valid ? 1.f + lv - mu * mu - sd * sd : 0.f;
    zt[r][c] = zz;
  }
  kld = wave_sum(kld);
  __syncthreads();
  STAMP(1, 1);
  {
    const int rr0 = lane & 15;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int k0 = cc * 16 + 4 * q;
      const float4 av = *reinterpret_cast<const float4*>(&zt[rr0][min(k0, 32)]);
      const bool in = k0 < a.Z;  // select, not multiply: unwritten LDS may hold NaN bits
      acc = mfma16x16x4(in ? av.x : 0.f, w3v[cc].x * w3m[cc], acc);
      acc = mfma16x16x4(in ? av.y : 0.f, w3v[cc].y * w3m[cc], acc);
      acc = mfma16x16x4(in ? av.z : 0.f, w3v[cc].z * w3m[cc], acc);
      acc = mfma16x16x4(in ? av.w : 0.f, w3v[cc].w * w3m[cc], acc);
    }
    if (j < a.H) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int ii = i0 + 4 * q + rr;
        if (ii < a.M) a.h3[(size_t)ii * a.H + j] = fmaxf(acc[rr] + bj, 0.f);
      }
    }
  }
  if (g == 0) {
    if (valid) {
      const size_t o = (size_t)i * Z2;
      a.mulv[o + c] = mu;
      a.mulv[o + a.Z + c] = lv;
      a.eps[(size_t)i * a.Z + c] = ep;
      a.z[(size_t)i * a.Z + c] = zz;
    }
    if (lane == 0) a.partials[kKldPartial + ti * kWaves + w] = -0.5f * kld;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int cur = a.st->cursor + 1;
    if (a.st->nbatches > 0 && cur >= a.st->nbatches) cur = 0;
    a.st->cursor = cur;
  }
  STAMP(1, 2);
}

// ------------------------------------------------------------------- F3 ----
struct EpiBce {
  const float* xb; const float* bias; float* dlog; float* recon;
  int D, M, train;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= D) return 0.f;
    const float b = bias[j];
    float x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = xb[(size_t)min(rows[r], M - 1) * D + j];
    float loss = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (rows[r] >= M) continue;
      const float t = v[r] + b;
      const size_t o = (size_t)rows[r] * D + j;
      const float p = 1.f / (1.f + expf(-t));
      if (train) dlog[o] = p - x[r];
      if (recon) recon[o] = p;
      // -[x log p + (1-x) log(1-p)] in the overflow-free logit form, with the
      // reference's log clamp at -100 (torch binary_cross_entropy) preserved.
      const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));  // -log(1-p)
      const float sp_neg = sp_pos - t;                                 // -log p
      loss += x[r] * fminf(sp_neg, 100.f) + (1.f - x[r]) * fminf(sp_pos, 100.f);
    }
    return loss;
  }
};

__global__ void __launch_bounds__(kThreads) vae_f3(VaeArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kWaves * 256];
  STAMP(2, 0);
  ARowMajor A{a.h3, a.H, a.M, a.H};
  BWeightNT Bw{a.W4, a.H, a.D, a.H};
  EpiBce epi{a.xb, a.b4, a.dlog, a.recon, a.D, a.M, a.train};
  const float c = gemm_tiles<kWaves, 2, 1, 7, false>(A, Bw, epi, a.H, cdiv_d(a.M, 16), cdiv_d(a.D, 16),
                                                     blockIdx.x, lds);
  const float s = wave_sum(c);
  if (lane_id() == 0) a.partials[kBcePartial + blockIdx.x * kWaves + wave_id()] = s;
  STAMP(2, 1);
}

// ------------------------------------------------------------------- B1 ----
struct EpiMask {
  float* out; const float* mask; int ld, M, N;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= N) return 0.f;
    float mk[R];
#pragma unroll
    for (int r = 0; r < R; ++r) mk[r] = mask[(size_t)min(rows[r], M - 1) * ld + j];
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rows[r] < M) out[(size_t)rows[r] * ld + j] = mk[r] > 0.f ? v[r] : 0.f;
    return 0.f;
  }
};

struct EpiWGrad {  // weight grad [M=out, N=in] (j >= 0) and bias grad [M] (j == -1)
  float* gw; float* gb; int ld, M, N;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= N) return 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (rows[r] >= M) continue;
      if (j < 0) gb[rows[r]] = v[r];
      else gw[(size_t)rows[r] * ld + j] = v[r];
    }
    return 0.f;
  }
};

// Weight/bias grad + in-place Adam on (param, exp_avg, exp_avg_sq) of the same
// elements: the gradient never round-trips through HBM before the update, and
// the R parameter/moment loads of a fragment are issued together.
struct EpiWGradAdam {
  float* G; float* P; float* Mo; float* Vo; long long ow, ob; int ld, M, N; AdamC c;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= N) return 0.f;
    long long o[R];
    float p[R], m[R], vv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = min(rows[r], M - 1);
      o[r] = (j < 0) ? ob + i : ow + (long long)i * ld + j;
      p[r] = P[o[r]]; m[r] = Mo[o[r]]; vv[r] = Vo[o[r]];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) adam_update(p[r], m[r], vv[r], v[r], c);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (rows[r] >= M) continue;
      G[o[r]] = v[r]; P[o[r]] = p[r]; Mo[o[r]] = m[r]; Vo[o[r]] = vv[r];
    }
    return 0.f;
  }
};

// dW GEMMs (K = batch): 32x32x2 f32 MFMA tiles, 2 tiles per block, k split
// over 4 waves each; bias from the A-operand row sums (gemm_tiles32).
constexpr int kWgTPB = 2;
constexpr int kWgNPW = 16;  // k pairs per wave per round: B = 128 -> 64 pairs / 4 waves
constexpr int kWgLds = kWaves * 1024 + kWaves * 64;
__host__ __device__ inline int wgrad_blocks(int out_rows, int in_cols) {
  return ((out_rows + 31) / 32 * ((in_cols + 31) / 32) + kWgTPB - 1) / kWgTPB;
}
#define WGRAD(A, B, EPI, OUT, IN, BLK, LDS) \
  gemm_tiles32<kWaves, kWgTPB, kWgNPW, true>(A, B, EPI, a.M, cdiv_d(OUT, 32), cdiv_d(IN, 32), BLK, LDS)
#define WGRAD_ST(A, B, EPI, OUT, IN, BLK, LDS, K)                                                     \
  gemm_tiles32<kWaves, kWgTPB, kWgNPW, true>(                                                         \
      A, B, EPI, a.M, cdiv_d(OUT, 32), cdiv_d(IN, 32), BLK, LDS,                                      \
      (a.stamps && blockIdx.x < kStampBlocks)                                                         \
          ? a.stamps + (((size_t)(K) * kStampBlocks + blockIdx.x) * 8 + wave_id()) * 8 : nullptr)

__global__ void __launch_bounds__(kThreads) vae_b1(VaeArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kWaves * 256];
  __shared__ __attribute__((aligned(16))) float ht[16][20];
  STAMP(3, 0);
  {
    // one 16x16 tile (ti, tj) of dh3 = (dlog W4) . [h3 > 0], K = D over 8 waves;
    // then waves 0..NTZ-1 emit the dz split-K slab dh3[:, tj] W3[tj, :].
    const SlabGeo geo(a.H, a.Z);
    const int w = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
    const int ti = blockIdx.x / geo.th, tj = blockIdx.x - ti * geo.th;
    const int i0 = ti * 16, j = tj * 16 + (lane & 15);
    const int q = lane >> 4;
    float mk[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) mk[rr] = a.h3[(size_t)min(i0 + 4 * q + rr, a.M - 1) * a.H + min(j, a.H - 1)];
    // raw prefetch, masked where used (no wait in front of the GEMM's loads)
    float wr[4] = {0.f, 0.f, 0.f, 0.f}, wm[4] = {0.f, 0.f, 0.f, 0.f};
    if (w < geo.ntz) {  // B(k, n) = W3[(tj*16 + k) * Z + w*16 + n]
      const int n = w * 16 + (lane & 15);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int k = tj * 16 + 4 * q + t;
        wr[t] = a.W3[(size_t)min(k, a.H - 1) * a.Z + min(n, a.Z - 1)];
        wm[t] = (k < a.H && n < a.Z) ? 1.f : 0.f;
      }
    }
    ARowMajor A{a.dlog, a.D, a.M, a.D};
    BRowMajor Bw{a.W4, a.H, a.H, a.D};
    const int nch = cdiv_d(a.D, 16);
    const int kc0 = (w * nch) / kWaves, kc1 = ((w + 1) * nch) / kWaves;
    f32x4 acc = wave_tile<7>(A, Bw, i0, tj * 16, kc0, kc1);
    *reinterpret_cast<f32x4*>(lds + w * 256 + lane * 4) = acc;
    __syncthreads();
    float d[4];
    if (w == 0) {
#pragma unroll
      for (int s = 1; s < kWaves; ++s) acc += *reinterpret_cast<const f32x4*>(lds + s * 256 + lane * 4);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) d[rr] = (mk[rr] > 0.f && i0 + 4 * q + rr < a.M && j < a.H) ? acc[rr] : 0.f;
      tile_to_lds(ht, d);
    }
    __syncthreads();
    if (w < geo.ntz) {
      const float wb[4] = {wr[0] * wm[0], wr[1] * wm[1], wr[2] * wm[2], wr[3] * wm[3]};
      const f32x4 sl = lds_tile_mma(ht, wb);
      float* dst = a.slab_dz + ((size_t)(ti * geo.th + tj) * 16) * geo.swz + w * 16 + (lane & 15);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) dst[(size_t)(4 * q + rr) * geo.swz] = sl[rr];
    }
    if (w == 0 && j < a.H) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        if (i0 + 4 * q + rr < a.M) a.dh3[(size_t)(i0 + 4 * q + rr) * a.H + j] = d[rr];
    }
  }
  STAMP(3, 1);
}

// ------------------------------------------------------------------- B2 ----
// Blocks [0, nrow): (row tile ti, group g): sum the TH dz slabs (4 quarter
// sums in LDS), dmu/dlv (reparam + beta-KLD grads), then wave w computes dh1
// tile g*8+w = ([dmu|dlv] W2) . [h1 > 0] with K = 2Z from LDS; group 0 stores
// dmulv. Blocks [nrow, nrow + nw3): dW3 = dh3^T z, db3. Last block: loss.
__global__ void __launch_bounds__(kThreads) vae_b2(VaeArgs a, int nrow, int nw3, int nw4) {
  __shared__ __attribute__((aligned(16))) float red[kWgLds];
  __shared__ __attribute__((aligned(16))) float dml[16][68];  // [row][dmu(Z) | dlv(Z)]
  __shared__ float scratch[16];
  const int bid = blockIdx.x;
  STAMP(4, 0);
  if (bid >= nrow + nw3 + nw4) {
    // loss = sum(BCE partials) + beta * sum(KLD partials) of this step's forward
    const int nk = cdiv_d(a.M, 16) * kWaves;
    const int nb = cdiv_d(cdiv_d(a.M, 16) * cdiv_d(a.D, 16), 2) * kWaves;
    float sb = 0.f, sk = 0.f;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) sb += a.partials[kBcePartial + i];
    for (int i = threadIdx.x; i < nk; i += blockDim.x) sk += a.partials[kKldPartial + i];
    const float bce = block_sum(sb, scratch);
    __syncthreads();
    const float kld = block_sum(sk, scratch);
    if (threadIdx.x == 0) {
      const float loss = bce + a.hp->kl_beta * kld;
      TrainState* st = a.st;
      st->loss_hist[(st->step - 1) % kLossHist] = loss;
      st->epoch_loss += (double)loss;
      st->epoch_count += 1.0;
    }
    return;
  }
  if (bid >= nrow + nw3) {
    // dW4[D, H] = dlog^T h3 (k = batch), db4 = column sums of dlog. Needs only
    // F2/F3 outputs; here (not in B1 beside the 200 dh3 blocks) the launch
    // stays within one workgroup per CU
    ATrans A{a.dlog, a.D, a.D, a.M};
    BRowMajor Bh{a.h3, a.H, a.H, a.M};
    EpiWGrad epi{a.gW4, a.gb4, a.H, a.D, a.H};
    WGRAD(A, Bh, epi, a.D, a.H, bid - nrow - nw3, red);
    return;
  }
  if (bid >= nrow) {
    ATrans A{a.dh3, a.H, a.H, a.M};
    BRowMajor Bz{a.z, a.Z, a.Z, a.M};
    EpiWGrad epi{a.gW3, a.gb3, a.Z, a.H, a.Z};
    WGRAD(A, Bz, epi, a.H, a.Z, bid - nrow, red);
    return;
  }
  const SlabGeo geo(a.H, a.Z);
  const int w = __builtin_amdgcn_readfirstlane(wave_id()), lane = lane_id();
  const int ti = bid / geo.groups, g = bid - ti * geo.groups;
  const int i0 = ti * 16;
  const int Z2 = 2 * a.Z;
  const int q = lane >> 4;
  const int jt = g * kWaves + w;
  const int j = jt * 16 + (lane & 15);
  // prefetch: W2 fragments (K = 2Z <= 64 -> up to 4 chunks), h1 mask, and
  // this thread's mu / lv / eps
  float wb[4][4];  // raw; masked where used (no wait in front of the slab loads)
#pragma unroll
  for (int cc = 0; cc < 4; ++cc)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int k = cc * 16 + 4 * q + t;
      wb[cc][t] = a.W2[(size_t)min(k, Z2 - 1) * a.H + min(j, a.H - 1)];
    }
  float mk[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) mk[rr] = a.h1[(size_t)min(i0 + 4 * q + rr, a.M - 1) * a.H + min(j, a.H - 1)];
  const int e = threadIdx.x;
  const int r = e / a.Z, c = e - r * a.Z;
  const int i = i0 + r;
  const bool mine = e < 16 * a.Z;
  const bool valid = mine && i < a.M;
  float mu = 0.f, lv = 0.f, ep = 0.f;
  if (mine) {
    const int ic = min(i, a.M - 1);
    mu = a.mulv[(size_t)ic * Z2 + c];
    lv = a.mulv[(size_t)ic * Z2 + a.Z + c];
    ep = a.eps[(size_t)ic * a.Z + c];
  }
  // phase 1: quarter sums of the dz slabs, float4 per (row, quad)
  float* part = red;  // [4][16][SWZ]
  {
    const int quads = geo.swz / 4;
    const int pairs = 16 * quads;
    const int t = threadIdx.x;
    if (t < 4 * pairs) {
      const int qq = t / pairs, pr = t - qq * pairs;
      const int rr = pr / quads, cq = pr - rr * quads;
      const float4* base = reinterpret_cast<const float4*>(a.slab_dz + ((size_t)(ti * geo.th) * 16 + rr) * geo.swz) + cq;
      const size_t sstride = (size_t)16 * geo.swz / 4;
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = base[min(qq * 8 + u, geo.th - 1) * sstride];
      __builtin_amdgcn_sched_barrier(0);  // all slab loads in flight before the first add
      float4 acc4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float m = qq * 8 + u < geo.th ? 1.f : 0.f;
        acc4.x += v[u].x * m; acc4.y += v[u].y * m; acc4.z += v[u].z * m; acc4.w += v[u].w * m;
      }
      *reinterpret_cast<float4*>(&part[(qq * 16 + rr) * geo.swz + cq * 4]) = acc4;
    }
  }
  __syncthreads();
  STAMP(4, 1);
  const float beta = a.hp->kl_beta;
  float dmu = 0.f, dlv = 0.f;
  if (mine) {
    float dz = 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) dz += part[(qq * 16 + r) * geo.swz + c];
    if (valid) {
      const float sd = expf(0.5f * lv);
      // L = BCE + beta * (-0.5 sum(1 + lv - mu^2 - e^lv)), z = mu + eps*sd
      dmu = dz + beta * mu;
      dlv = 0.5f * dz * ep * sd + 0.5f * beta * (sd * sd - 1.f);
    }
    dml[r][c] = dmu;
    dml[r][a.Z + c] = dlv;
  }
  __syncthreads();
  STAMP(4, 2);
  {
    const int rr0 = lane & 15;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < 4; ++cc) {
      const int k0 = cc * 16 + 4 * q;
      const float4 av = *reinterpret_cast<const float4*>(&dml[rr0][min(k0, 64)]);
      const bool in = k0 < Z2;  // select, not multiply: unwritten LDS may hold NaN bits
      float b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) b[t] = wb[cc][t] * ((k0 + t < Z2 && j < a.H) ? 1.f : 0.f);
      acc = mfma16x16x4(in ? av.x : 0.f, b[0], acc);
      acc = mfma16x16x4(in ? av.y : 0.f, b[1], acc);
      acc = mfma16x16x4(in ? av.z : 0.f, b[2], acc);
      acc = mfma16x16x4(in ? av.w : 0.f, b[3], acc);
    }
    if (j < a.H) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int ii = i0 + 4 * q + rr;
        if (ii < a.M) a.dh1[(size_t)ii * a.H + j] = mk[rr] > 0.f ? acc[rr] : 0.f;
      }
    }
  }
  if (g == 0 && valid) {
    a.dmulv[(size_t)i * Z2 + c] = dmu;
    a.dmulv[(size_t)i * Z2 + a.Z + c] = dlv;
  }
  STAMP(4, 3);
}

// ------------------------------------------------------------------- B3 ----
__global__ void __launch_bounds__(kThreads) vae_b3(VaeArgs a, int nblk_w2, int nblk_w1) {
  __shared__ __attribute__((aligned(16))) float lds[kWgLds];
  __shared__ AdamC cs;
  const int Z2 = 2 * a.Z;
  const int bid = blockIdx.x;
  STAMP(5, 0);
  if (!a.fuse_adam) {
    if (bid < nblk_w2) {
      ATrans A{a.dmulv, Z2, Z2, a.M};
      BRowMajor Bh{a.h1, a.H, a.H, a.M};
      EpiWGrad epi{a.gW2, a.gb2, a.H, Z2, a.H};
      WGRAD(A, Bh, epi, Z2, a.H, bid, lds);
    } else {
      ATrans A{a.dh1, a.H, a.H, a.M};
      BRowMajor Bx{a.xb, a.D, a.D, a.M};
      EpiWGrad epi{a.gW1, a.gb1, a.D, a.H, a.D};
      WGRAD(A, Bx, epi, a.H, a.D, bid - nblk_w2, lds);
    }
    STAMP(5, 1);
    return;
  }
  const AdamC c = adam_consts_block(a.st, a.hp, &cs);
  if (bid < nblk_w2) {
    ATrans A{a.dmulv, Z2, Z2, a.M};
    BRowMajor Bh{a.h1, a.H, a.H, a.M};
    EpiWGradAdam epi{a.G, a.P, a.Mo, a.Vo, a.oW2, a.ob2, a.H, Z2, a.H, c};
    WGRAD(A, Bh, epi, Z2, a.H, bid, lds);
  } else if (bid < nblk_w2 + nblk_w1) {
    ATrans A{a.dh1, a.H, a.H, a.M};
    BRowMajor Bx{a.xb, a.D, a.D, a.M};
    EpiWGradAdam epi{a.G, a.P, a.Mo, a.Vo, a.oW1, a.ob1, a.D, a.H, a.D, c};
    WGRAD_ST(A, Bx, epi, a.H, a.D, bid - nblk_w2, lds, 5);
  } else {
    const int nb = gridDim.x - nblk_w2 - nblk_w1;
    adam_stream(a.P, a.G, a.Mo, a.Vo, a.s_beg, a.s_end, bid - nblk_w2 - nblk_w1, nb, c);
  }
  STAMP(5, 1);
}

// --------------------------------------------------------------- decode ----
// Sampling path (/root/reference/vae-hpo.py:163-170): x = sigmoid(fc4(relu(fc3(z)))).
struct EpiSigmoid {
  float* out; const float* bias; int ld, M, N;
  template <int R>
  __device__ __forceinline__ float run(const int (&rows)[R], int j, const float (&v)[R]) const {
    if (j >= N) return 0.f;
    const float b = bias[j];
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (rows[r] < M) out[(size_t)rows[r] * ld + j] = 1.f / (1.f + expf(-(v[r] + b)));
    return 0.f;
  }
};

__global__ void __launch_bounds__(kThreads) vae_dec1(VaeArgs a, const float* zin) {
  __shared__ __attribute__((aligned(16))) float lds[kWaves * 256];
  ARowMajor A{zin, a.Z, a.M, a.Z};
  BWeightNT Bw{a.W3, a.Z, a.H, a.Z};
  EpiBiasRelu epi{a.h3, a.b3, a.H, a.M, a.H};
  gemm_tiles<kWaves, kWaves, 1, 2, false>(A, Bw, epi, a.Z, cdiv_d(a.M, 16), cdiv_d(a.H, 16), blockIdx.x, lds);
}

__global__ void __launch_bounds__(kThreads) vae_dec2(VaeArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kWaves * 256];
  ARowMajor A{a.h3, a.H, a.M, a.H};
  BWeightNT Bw{a.W4, a.H, a.D, a.H};
  EpiSigmoid epi{a.recon, a.b4, a.D, a.M, a.D};
  gemm_tiles<kWaves, 2, 1, 7, false>(A, Bw, epi, a.H, cdiv_d(a.M, 16), cdiv_d(a.D, 16), blockIdx.x, lds);
}

// -------------------------------------------------------------- host side ----
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

VaeGrid vae_grid(const VaeArgs& a) {
  VaeGrid g;
  const SlabGeo geo(a.H, a.Z);
  g.th = geo.th; g.ntm = geo.ntm; g.sw = geo.sw; g.ntz = geo.ntz; g.swz = geo.swz; g.groups = geo.groups;
  const int ti = cdiv(a.M, 16);
  g.f1 = ti * cdiv(a.H, 16);
  g.f2 = ti * geo.groups;
  g.f3 = cdiv(ti * cdiv(a.D, 16), 2);
  g.b1_dh3 = ti * cdiv(a.H, 16);
  g.b1 = g.b1_dh3;
  g.b2_rows = ti * geo.groups;
  g.b2 = g.b2_rows + wgrad_blocks(a.H, a.Z) + wgrad_blocks(a.D, a.H) + 1;
  g.b3_w2 = wgrad_blocks(2 * a.Z, a.H);
  g.b3_w1 = wgrad_blocks(a.H, a.D);
  const long long n4 = (a.s_end - a.s_beg) / 4;
  // Adam streaming blocks: ~2 float4 per thread keeps B3 within one CU round
  g.b3_stream = a.fuse_adam ? (int)((n4 + 2 * kThreads - 1) / (2 * kThreads)) : 0;
  g.b3 = g.b3_w2 + g.b3_w1 + g.b3_stream;
  return g;
}

}  // namespace mdt

using namespace mdt;

extern "C" int mdt_vae_check(const VaeArgs* a) {
  if (a->M <= 0 || a->M > a->B || a->B > kMaxBatch) return 1;
  if (a->Z > 32 || a->Z <= 0 || (a->Z & 3)) return 2;
  if ((a->D & 3) || (a->H & 3)) return 3;      // float4 alignment of row-major operands
  if (a->H > kWaves * 16 * 4) return 6;        // F2/B2 stage C: <= 4 n-tiles per wave
  const VaeGrid g = vae_grid(*a);
  if (cdiv(a->M, 16) * kWaves > kBcePartial - kKldPartial) return 4;
  if (a->H > 16 * 32 || !a->slab_mv || !a->slab_dz) return 8;  // slab half-sums cover <= 32 slices
  if (g.f3 * kWaves > kPartials - kBcePartial) return 5;
  if (16 * a->Z > kThreads) return 2;
  if (a->fuse_adam && (!a->P || !a->G || !a->Mo || !a->Vo || (a->s_beg & 3) || (a->s_end & 3))) return 7;
  return 0;
}

extern "C" int mdt_vae_forward(const VaeArgs* a, hipStream_t s) {
  const int rc = mdt_vae_check(a);
  if (rc) return rc;
  const VaeGrid g = vae_grid(*a);
  hipLaunchKernelGGL(vae_f1, dim3(g.f1), dim3(kThreads), 0, s, *a);
  hipLaunchKernelGGL(vae_f2, dim3(g.f2), dim3(kThreads), 0, s, *a);
  hipLaunchKernelGGL(vae_f3, dim3(g.f3), dim3(kThreads), 0, s, *a);
  return (int)hipGetLastError();
}

extern "C" int mdt_vae_backward(const VaeArgs* a, hipStream_t s, int part) {
  const int rc = mdt_vae_check(a);
  if (rc) return rc;
  const VaeGrid g = vae_grid(*a);
  if (part == 0 || part == 1) hipLaunchKernelGGL(vae_b1, dim3(g.b1), dim3(kThreads), 0, s, *a);
  if (part == 0 || part == 2)
    hipLaunchKernelGGL(vae_b2, dim3(g.b2), dim3(kThreads), 0, s, *a, g.b2_rows, wgrad_blocks(a->H, a->Z),
                       wgrad_blocks(a->D, a->H));
  if (part == 0 || part == 3)
    hipLaunchKernelGGL(vae_b3, dim3(g.b3), dim3(kThreads), 0, s, *a, g.b3_w2, g.b3_w1);
  return (int)hipGetLastError();
}

extern "C" int mdt_vae_decode(const VaeArgs* a, const float* zin, hipStream_t s) {
  if (a->M <= 0 || a->M > a->B || !a->recon || (a->Z & 3)) return 1;
  const int ti = cdiv(a->M, 16);
  hipLaunchKernelGGL(vae_dec1, dim3(cdiv(ti * cdiv(a->H, 16), kWaves)), dim3(kThreads), 0, s, *a, zin);
  hipLaunchKernelGGL(vae_dec2, dim3(cdiv(ti * cdiv(a->D, 16), 2)), dim3(kThreads), 0, s, *a);
  return (int)hipGetLastError();
}
