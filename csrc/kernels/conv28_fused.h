// Per-sample fused 28x28 conv-VAE training step for MI355X (gfx950): shared
// helpers, LDS maps and the one-workgroup-per-sample ("solo") bodies. The
// kernels and launchers live in conv28_fused.hip; the two-workgroups-per-
// sample body in conv28_pair.h.
//
// Why a different decomposition than conv_igemm.hip's layer-by-layer GEMMs:
// at 28x28 every layer is tiny (M <= 25k rows, K <= 3136, N <= 3136) and a
// layer-per-launch step is a chain of ~15 dependent launches that each pay a
// kernel boundary (~1.3 us), a cold first load from another XCD's writes and a
// short k-loop whose iterations are load-latency bound -- ~116 us per step at
// B = 128 for 2.8 GFLOP (profiles/r2_bench). A conv-VAE's forward and its
// backward-data chain, however, never mix samples: every layer of sample n
// reads only sample n. So one workgroup per sample runs the WHOLE chain with
// the activations resident in LDS (<= 25 KB per sample), and only the weight
// gradients (a reduction over the batch) and the optimizer need the batch:
//
//   launch 1  f28_fwd_k   (B workgroups): batch gather -> enc1 -> enc2 -> head
//             -> reparam (Philox) + KLD -> dec_fc -> dec1 -> dec2 -> BCE, dlogits
//   launch 2  f28_bwd_k   (B workgroups): dec2 / dec1 / dec_fc backward-data,
//             reparam backward, head / enc2 backward-data, ReLU masks, per-sample
//             bias-gradient partials
//   launch 3  jobs_multi_k: the six weight-gradient GEMMs (m-split partial
//             slabs, conv_igemm_dev.h bodies) + loss reduction / step advance
//   launch 4  grad_finalize_k: slab reduction + Adam + bf16 re-cast
//
// Inside a workgroup (512 threads = 8 waves, one sample) the convolutions run
// on v_mfma_f32_16x16x32_bf16 with the A operand gathered straight out of the
// LDS activation image (implicit im2col) and the B operand either streamed
// from L2 into registers (conv-layout weights, k contiguous) or read with
// ds_read_b64_tr_b16 from per-tap LDS images (transposed-conv weights), so no
// transposed weight copies exist. The Linear layers stream their bf16 weights
// (head 400 KB, dec_fc 200 KB) from L2 with up to 16 loads in flight per lane;
// that weight stream, not arithmetic, bounds each fused launch.
//
// Numerics: f32 accumulation, bf16 activations (same rounding points as the
// layer-by-layer path), f32 loss / dlogits / mu / logvar / eps; Philox keyed
// exactly like combine_reparam (element n*Z+c, stream, step) so the torch
// reference (ops/philox.py) reproduces eps.
#pragma once
#include "conv_igemm_dev.h"
#include "conv_small.h"
#include "vae_mlp.h"

namespace mdt {
namespace f28 {

constexpr int kThreads = 512;
constexpr int kFlat = 3136;  // 7 * 7 * 64

struct Weights {
  const float* W1f;   // enc1 f32 master [32][4][4][1]
  const float* b1;
  const __bf16* W2;   // enc2 [64][4][4][32]
  const float* b2;
  const __bf16* Wh;   // enc_head [64][3136]
  const float* bh;
  const __bf16* Wd;   // dec_fc [3136][32]
  const float* bd;
  const __bf16* W3;   // dec1 (convT) [64][4][4][32]
  const float* b3;
  const float* W4f;   // dec2 (convT) f32 master [32][4][4][1]
  const float* b4;
};

struct FwdArgs {
  Weights w;
  const float* X;        // dataset [N][784]
  const int* idx;        // epoch index list
  const TrainState* st;  // train or eval state (cursor, step)
  const HParams* hp;
  int B;
  uint32_t stream;
  int train;             // write the backward's inputs (activations, dlogits)
  float* xb;             // [M][784] gathered batch
  __bf16* a1;            // [M][196][32]
  __bf16* a2;            // [M][3136]
  float* mulv;           // [M][64]
  float* eps;            // [M][32]
  __bf16* z16;           // [M][32]
  __bf16* d0;            // [M][3136]
  __bf16* d1;            // [M][196][32]
  float* dlog;           // [M][784]
  float* recon;          // optional sigmoid [M][784]
  float* bce_part;       // [M]
  float* kld_part;       // [M]
  float* db4_part;       // [M] (dec2 bias gradient partials)
  unsigned long long* stamps;  // optional [grid][16] s_memrealtime at phase ends (profiling)
  int pf_slices;         // P0 L2-prefetch slices per XCD (workgroups sharing one XCD)
  // next-batch prefetch (training only, null = off): the previous step's
  // finalize gathered this step's rows into xn [B][784] and wrote xtag[n] =
  // the TrainState.step they are for (grad_finalize_k, BatchGather)
  const float* xn;
  const unsigned* xtag;
};

struct BwdArgs {
  Weights w;
  const HParams* hp;
  const float* mulv;
  const float* eps;
  const __bf16* a1;
  const __bf16* a2;
  const __bf16* d0;
  const __bf16* d1;
  const float* dlog;
  __bf16* gd1;       // [M][196][32] masked grad of dec1's output
  __bf16* gd0;       // [M][3136]    masked grad of dec_fc's output
  float* dbd_part;   // [M][3136]    dec_fc bias partials (f32 of gd0)
  float* dmulv;      // [M][64]      d[mu|logvar] (also the head-bias partials)
  __bf16* dmulv16;   // [M][64]
  __bf16* ga2;       // [M][3136]    masked grad of enc2's output
  __bf16* ga1;       // [M][196][32] masked grad of enc1's output
  float* db3_part;   // [M][32]
  float* db2_part;   // [M][64]
  float* db1_part;   // [M][32]
  unsigned long long* stamps;  // optional [grid][16] phase-end timestamps
  int db2_m2;        // > 0: db2_part is [2][M][64] (M = db2_m2), the solo body zeroes the second row
};

// 14x14x32 bf16 LDS image, 64-B pixel rows: 16-B chunk ch of pixel p at slot
// ch ^ ((p >> 1) & 3) -- the stride-2 im2col gathers of 16 lanes then spread
// over all four chunk slots of a bank row instead of hitting one.
// Workgroup barrier for the phase hand-offs: LDS writes visible, global
// stores NOT waited for. __syncthreads() waits vmcnt(0), i.e. for the
// acknowledgement of every global store of the phase (the activations and
// gradients the weight-gradient launch reads later), which put an L2 write
// round trip on every phase boundary. Inside these kernels every cross-thread
// hand-off goes through LDS; a thread re-reading global data reads its own
// earlier stores (P4 -> Q4), which program order covers.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Phase timestamp (100 MHz s_memrealtime) of workgroup blockIdx.x, slot k.
__device__ __forceinline__ void stamp(unsigned long long* st, int k) {
  if (st && threadIdx.x == 0) st[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ int img14(int pix, int ch) { return (pix << 6) + ((ch ^ ((pix >> 1) & 3)) << 4); }

// 7x7x64 bf16 LDS image, 128-B pixel rows: 16-B chunk c of pixel p at slot
// c ^ (p & 7), so the transposed-conv A gathers (16 class pixels at one chunk)
// spread over the banks.
__device__ __forceinline__ int img49(int pix, int ch) { return (pix << 7) + ((ch ^ (pix & 7)) << 4); }
__device__ __forceinline__ int img49e(int pix, int c) { return img49(pix, c >> 3) + ((c & 7) << 1); }

// Per-tap images of a [64][16][32] bf16 weight (rows c64 = reduction index,
// 32 columns) are laid out for tr_frag<32> reads: 16 images of 4 KB
// (TapImageRegs below fills them).

// Weight stream with double buffering: items 0 .. CH*NCH-1, CH 16-B loads per
// lane in flight while the previous CH are consumed. ld(i) must tolerate i past
// the end (clamp the address), use(i, v) must skip it. The outer loop is not
// unrolled so at most 2*CH fragments are live.
template <int CH, int NCH, class Load, class Use>
__device__ __forceinline__ void stream2(Load ld, Use use) {
  bf16x8 bc[CH], bn[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) bc[i] = ld(i);
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) {
#pragma unroll
      for (int i = 0; i < CH; ++i) bn[i] = ld((c + 1) * CH + i);
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) use(c * CH + i, bc[i]);
#pragma unroll
    for (int i = 0; i < CH; ++i) bc[i] = bn[i];
  }
}

// stream2 whose first CH loads were issued earlier (during a previous phase).
template <int CH, int NCH, class Load, class Use>
__device__ __forceinline__ void stream2_pre(const bf16x8 (&first)[CH], Load ld, Use use) {
  bf16x8 bc[CH], bn[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) bc[i] = first[i];
#pragma unroll 1
  for (int c = 0; c < NCH; ++c) {
    if (c + 1 < NCH) {
#pragma unroll
      for (int i = 0; i < CH; ++i) bn[i] = ld((c + 1) * CH + i);
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) use(c * CH + i, bc[i]);
#pragma unroll
    for (int i = 0; i < CH; ++i) bc[i] = bn[i];
  }
}

// Conv-layout [64][16][32] bf16 weight staged in LDS: row co = 1 KB, 16-B
// chunk (tap, ch) of row co at slot (tap*4 + ch) ^ (co & 15), so the 16 rows a
// B-fragment read touches land on 16 different bank groups.
__device__ __forceinline__ int cimg(int co, int tap, int ch) { return (co << 10) + (((tap * 4 + ch) ^ (co & 15)) << 4); }

__device__ __forceinline__ void stage_conv_image(const __bf16* W, uint8_t* img) {
  for (int q = threadIdx.x; q < 4096; q += kThreads) {
    const int co = q >> 6, tap = (q >> 2) & 15, ch = q & 3;
    *reinterpret_cast<bf16x8*>(img + cimg(co, tap, ch)) = *reinterpret_cast<const bf16x8*>(W + q * 8);
  }
}

// stage_conv_image split in two: the loads now, the LDS stores later.
struct ConvImageRegs {
  bf16x8 v[8];
  __device__ __forceinline__ void load(const __bf16* W) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const bf16x8*>(W + (threadIdx.x + i * kThreads) * 8);
  }
  __device__ __forceinline__ void store(uint8_t* img) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = threadIdx.x + i * kThreads;
      const int co = q >> 6, tap = (q >> 2) & 15, ch = q & 3;
      *reinterpret_cast<bf16x8*>(img + cimg(co, tap, ch)) = v[i];
    }
  }
};

// B fragment of n-tile j, k-step (tap) t: lane holds W[16j + (l & 15)][t][8(l >> 4) ..]
__device__ __forceinline__ bf16x8 conv_bfrag(const uint8_t* img, int j, int t, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + cimg(16 * j + (lane & 15), t, lane >> 4));
}

// Per-tap image loads held in registers across phases (8 chunks per thread),
// then written: the LDS-staged weight of a LATER phase streams in while the
// phases in between run.
struct TapImageRegs {
  bf16x8 v[8];
  __device__ __forceinline__ void load(const __bf16* W) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = *reinterpret_cast<const bf16x8*>(W + (threadIdx.x + i * kThreads) * 8);
  }
  __device__ __forceinline__ void store(uint8_t* img) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int q = threadIdx.x + i * kThreads;
      const int c64 = q >> 6, tap = (q >> 2) & 15, ch = q & 3;
      *reinterpret_cast<bf16x8*>(img + tap * 4096 + timg<32>(c64, ch)) = v[i];
    }
  }
};

// Stride-2 4x4 conv 14x14x32 -> 7x7x64 (+ per-element epilogue) of one sample:
// GEMM rows = 49 output pixels (4 m-tiles), cols = 64 (4 n-tiles), k = 16 taps
// x 32 channels. Wave w owns n-tile w & 3 and m-tiles (w >> 2) and (w >> 2) + 2.
// pre(p, col) is evaluated for every output element BEFORE the MFMA loop (its
// global loads -- bias, ReLU mask -- overlap the loop instead of stalling the
// epilogue); epi(p, col, acc, pre_value).
template <class BFrag, class Pre, class Epi>
__device__ __forceinline__ void conv14to7(const uint8_t* in_img, BFrag bfrag, Pre pre, Epi epi) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = w & 3;
  float pv[2][4];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int p = ((w >> 2) + 2 * q) * 16 + 4 * (lane >> 4) + rr;
      pv[q][rr] = p < 49 ? pre(p, 16 * j + (lane & 15)) : 0.f;
    }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int mt = (w >> 2) + 2 * q;
    const int r = mt * 16 + (lane & 15);
    const int oy = r / 7, ox = r - 7 * (r / 7);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int iy = 2 * oy - 1 + (t >> 2), ix = 2 * ox - 1 + (t & 3);
      const bool ok = r < 49 && (unsigned)iy < 14u && (unsigned)ix < 14u;
      const bf16x8 a = ok ? *reinterpret_cast<const bf16x8*>(in_img + img14(iy * 14 + ix, lane >> 4)) : zero8();
      acc = mfma_bf16(a, bfrag(j, t), acc);
    }
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int p = mt * 16 + 4 * (lane >> 4) + rr;
      if (p < 49) epi(p, 16 * j + (lane & 15), acc[rr], pv[q][rr]);
    }
  }
}

// Stride-2 4x4 transposed conv 7x7x64 -> 14x14x32 of one sample, as four
// stride-parity classes (a, b) = (oy & 1, ox & 1) without zero-insertion taps:
// class rows = 49 pixels (jy, jx) with (oy, ox) = (2jy + a, 2jx + b), k = 2x2
// taps (ky = 1 - a + 2ty, iy = jy + a - ty) x 64 channels, cols = 32. A from the
// img49 LDS image `in`, B via tr_frag from the per-tap images `wimg`.
// 32 items (class, m-tile, n-tile), four per wave. `cs[q]` receives the
// per-column sum of the epilogue values of this wave's item of class q
// (column 16 nj + (lane & 15), nj = w & 1; m-tile (w >> 1) & 3), kept per
// item so a caller can add them in the paired step's order.
template <class Pre, class Epi>
__device__ __forceinline__ void tconv7to14(const uint8_t* in, const uint8_t* wimg, Pre pre, Epi epi, float (&cs)[4]) {
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // items it = w + 8q: class q, m-tile (w >> 1) & 3, n-tile w & 1 (fixed per wave)
  const int mt = (w >> 1) & 3, nj = w & 1;
  float pv[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r2 = mt * 16 + 4 * (lane >> 4) + rr;
      const int jy2 = r2 / 7, jx2 = r2 - 7 * (r2 / 7);
      pv[q][rr] = r2 < 49 ? pre((2 * jy2 + (q >> 1)) * 14 + 2 * jx2 + (q & 1), 16 * nj + (lane & 15)) : 0.f;
    }
#pragma unroll 2
  for (int q = 0; q < 4; ++q) {
    const int a = q >> 1, b = q & 1;
    const int r = mt * 16 + (lane & 15);
    const int jy = r / 7, jx = r - 7 * (r / 7);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int ty = ks >> 2, tx = (ks >> 1) & 1, hh = ks & 1;
      const int iy = jy + a - ty, ix = jx + b - tx;
      const bool ok = r < 49 && (unsigned)iy < 7u && (unsigned)ix < 7u;
      const bf16x8 av = ok ? *reinterpret_cast<const bf16x8*>(in + img49(iy * 7 + ix, 4 * hh + (lane >> 4))) : zero8();
      const int tap = ((1 - a) + 2 * ty) * 4 + (1 - b) + 2 * tx;
      const bf16x8 bv = tr_frag<32>(wimg + tap * 4096, 16 * nj, 32 * hh, lane);
      acc = mfma_bf16(av, bv, acc);
    }
    float s = 0.f;
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int r2 = mt * 16 + 4 * (lane >> 4) + rr;
      if (r2 < 49) {
        const int jy2 = r2 / 7, jx2 = r2 - 7 * (r2 / 7);
        s += epi((2 * jy2 + a) * 14 + 2 * jx2 + b, 16 * nj + (lane & 15), acc[rr], pv[q][rr]);
      }
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    cs[q] = s;
  }
}

// ------------------------------------------------------------------ forward
// LDS map (bytes)
constexpr int kFX = 0;                      // f32 [784] input image
constexpr int kFW1 = kFX + 784 * 4;         // f32 [16][32] enc1 weights, tap-major
constexpr int kFW4 = kFW1 + 512 * 4;        // f32 [16][32] dec2 weights, tap-major
constexpr int kFA1 = kFW4 + 512 * 4;        // bf16 img14 [196][32] (enc1 out, later dec1 out)
constexpr int kFA2 = kFA1 + 196 * 64;       // bf16 [3136] enc2 out (NHWC flatten)
constexpr int kFD0 = kFA2 + kFlat * 2;      // bf16 [3136] dec_fc out
constexpr int kFH = kFD0 + kFlat * 2;       // f32 [64] head out
constexpr int kFZ = kFH + 64 * 4;           // bf16 [32] z
constexpr int kFRed = kFZ + 64;             // f32 [4][16] head k-half partials
constexpr int kFScr = kFRed + 64 * 4;       // f32 [32] block-sum scratch
constexpr int kFW3 = kFScr + 32 * 4;        // 16 x 4 KB dec1 tap images
constexpr int kFDummy = kFW3 + 65536;       // 8 x 1 KB landing zone of the L2 prefetch DMAs
constexpr int kFBd = kFDummy + 8192;        // f32 [3136] dec_fc bias
constexpr int kFBias = kFBd + kFlat * 4;     // f32 [256] small biases (LDS bias map below)
constexpr int kFLds = kFBias + 1024;
static_assert(kFA1 % 16 == 0 && kFA2 % 16 == 0 && kFD0 % 16 == 0 && kFW3 % 16 == 0, "LDS alignment");

struct FwdLayout {
  static constexpr int X = kFX, W1 = kFW1, W4 = kFW4, A1 = kFA1, A2 = kFA2, D0 = kFD0, H = kFH, Z = kFZ;
  static constexpr int Red = kFRed, Scr = kFScr, IMG = kFW3, Dummy = kFDummy, Bd = kFBd;
  static constexpr int G = -1;  // dlogits stay in global memory only
  static constexpr int D1 = kFA1;
  static constexpr int Bias = kFBias;
  static constexpr int LDS = kFLds;
};

// f32 offsets of the small biases inside L::Bias, staged in P0 so no later
// phase waits on a global bias load (vmcnt is in order: such a load also
// waits for every store the wave issued before it)
constexpr int kB1 = 0, kB2 = 32, kBh = 96, kB3 = 160, kB4 = 192, kNBias = 193;
constexpr int kZero = 252;  // f32 index of a 16-B zero chunk (the paired body's out-of-image gathers read it)

// P0 + P1 of the forward (the part a paired workgroup runs in full before it
// knows whether its partner arrived, conv28_pair.h). n = sample; after_p0()
// runs right after P0's barrier (the paired step issues its pairing atomic there).
template <class L, class AfterP0>
__device__ __forceinline__ void fwd_p01(const FwdArgs& a, uint8_t* lds, int n, AfterP0 after_p0) {
  float* Xs = reinterpret_cast<float*>(lds + L::X);
  float* W1s = reinterpret_cast<float*>(lds + L::W1);
  float* W4s = reinterpret_cast<float*>(lds + L::W4);
  uint8_t* A1s = lds + L::A1;
  uint8_t* W3s = lds + L::IMG;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Weights& W = a.w;
  stamp(a.stamps, 0);
  ConvImageRegs w2regs;  // enc2's conv-layout image: loaded in P0, written to LDS after P1

  // ---- P0: batch row gather, small weights, enc2's B image (into registers,
  // written to LDS after P1), L2 prefetch of the Linear weights.
  // Issue order matters: vmcnt retires in order, so the loads P1 needs (the
  // row, W1, biases) go first; the enc2 image loads and the prefetch DMAs go
  // after them and stay in flight through P1 (P0 ends on an LDS-only barrier).
  {
    // The batch row: when the previous step's finalize already gathered it
    // (xtag[n] == step), ONE round trip (the row load is issued before the
    // tag is known); otherwise the dependent cursor -> index -> row chain
    // (first step after the host moved the cursor / data, eval passes, DDP
    // steps). profiles/r6_f28_gather: the chain is ~0.4 us of P0.
    float4 xv = {0.f, 0.f, 0.f, 0.f};
    const bool pre_ok = a.train && a.xn != nullptr;
    if (pre_ok && tid < 196) xv = reinterpret_cast<const float4*>(a.xn + (size_t)n * 784)[tid];
    if (!pre_ok || a.xtag[n] != (unsigned)a.st->step) {
      const int row = a.idx[(size_t)a.st->cursor * a.B + n];
      const float4* src = reinterpret_cast<const float4*>(a.X + (size_t)row * 784);
      if (tid < 196) xv = src[tid];
    }
    const float w1 = W.W1f[tid], w4 = W.W4f[tid];
    float bv = 0.f;
    if (tid < kNBias)
      bv = tid < kB2 ? W.b1[tid] : tid < kBh ? W.b2[tid - kB2] : tid < kB3 ? W.bh[tid - kBh]
         : tid < kB4 ? W.b3[tid - kB3] : W.b4[0];
    float4 bdv[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * kThreads;
      bdv[i] = e < kFlat / 4 ? reinterpret_cast<const float4*>(W.bd)[e] : float4{0.f, 0.f, 0.f, 0.f};
    }
    w2regs.load(W.W2);
    // The head (400 KB) and dec_fc (200 KB) weights were just rewritten by
    // the optimizer on other XCDs, so P3 / P5 would stream them from the
    // Infinity Cache. The workgroups that share an XCD (block ids b, b+8, ...:
    // round-robin dispatch; a wrong guess costs speed only; 16 of them for
    // one workgroup per sample, 32 for two) each pull one slice into that
    // XCD's L2 now, through LDS-DMA loads into a scratch LDS zone (nothing
    // reads it). The builtin (not asm) keeps them in the compiler's vmcnt
    // accounting, so no wait above includes them.
    if (a.pf_slices > 0) {
      constexpr int kWh = kFlat * 64 * 2, kWd = kFlat * 32 * 2;
      const int nsl = a.pf_slices, kSlice = (kWh + kWd) / nsl;
      const int r = (int)(blockIdx.x >> 3) % nsl;
      for (int k = w; k * 1024 < kSlice; k += 8) {
        const int off = r * kSlice + k * 1024 + lane * 16;
        const uint8_t* psrc = off < kWh ? reinterpret_cast<const uint8_t*>(W.Wh) + off
                                        : reinterpret_cast<const uint8_t*>(W.Wd) + (off - kWh < kWd ? off - kWh : 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)psrc,
                                         (__attribute__((address_space(3))) void*)(lds + L::Dummy + w * 1024), 16, 0,
                                         0);
      }
    }
    if (tid < 196) {
      reinterpret_cast<float4*>(Xs)[tid] = xv;
      if (a.train) reinterpret_cast<float4*>(a.xb + (size_t)n * 784)[tid] = xv;
    }
    const int c = tid >> 4, t = tid & 15;  // 512 threads = 32 channels x 16 taps
    W1s[t * 32 + c] = w1;
    W4s[t * 32 + c] = w4;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * kThreads;
      if (e < kFlat / 4) reinterpret_cast<float4*>(lds + L::Bd)[e] = bdv[i];
    }
    if (tid < kNBias) {
      reinterpret_cast<float*>(lds + L::Bias)[tid] = bv;
    } else if (tid >= kZero && tid < kZero + 4) {
      reinterpret_cast<float*>(lds + L::Bias)[tid] = 0.f;
    }
  }
  lds_barrier();
  after_p0();

  stamp(a.stamps, 1);
  // ---- P1: enc1 (1 -> 32, 28x28 -> 14x14), ReLU, on exact-f32 MFMA
  // (v_mfma_f32_16x16x4_f32): D[channel][pixel] = W1[channel][tap] x
  // im2col(x)[tap][pixel] + bias, 2 channel tiles x 13 pixel tiles x 4 tap
  // steps; wave w takes pixel tiles w and w + 8. A lane ends with four
  // consecutive channels of one pixel: one 8-B bf16 store to the LDS image
  // and one to a1. The f32 VALU form (392 threads x 256 FMAs) spent 1.56 us
  // of this phase in its tap loop (profiles/r6_f28_gather).
  {
    const int col = lane & 15, kq = lane >> 4;
    float wa[2][4];  // A: W1[16 mt + col][4 ks + kq] (tap-major LDS copy)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wa[mt][ks] = W1s[(4 * ks + kq) * 32 + 16 * mt + col];
    const float* Bias1 = reinterpret_cast<const float*>(lds + L::Bias) + kB1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 8 * j;
      if (nt < 13) {
        const int pix = 16 * nt + col;
        const bool live = pix < 196;
        const int oy = pix / 14, ox = pix - 14 * (pix / 14);
        float xb4[4];  // B: im2col(x)[4 ks + kq][pix]
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int t = 4 * ks + kq;
          const int iy = 2 * oy - 1 + (t >> 2), ix = 2 * ox - 1 + (t & 3);
          xb4[ks] = live && (unsigned)iy < 28u && (unsigned)ix < 28u ? Xs[iy * 28 + ix] : 0.f;
        }
        f32x4 acc[2];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[mt][r] = Bias1[16 * mt + 4 * kq + r];
        }
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) acc[mt] = mfma16x16x4(wa[mt][ks], xb4[ks], acc[mt]);
        if (live) {
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int c0 = 16 * mt + 4 * kq;  // four consecutive channels
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            bf16x4 o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (__bf16)fmaxf(acc[mt][r], 0.f);
            *reinterpret_cast<bf16x4*>(A1s + img14(pix, c0 >> 3) + ((c0 & 7) << 1)) = o;
            if (a.train) *reinterpret_cast<bf16x4*>(a.a1 + ((size_t)n * 196 + pix) * 32 + c0) = o;
          }
        }
      }
    }
  }
  w2regs.store(W3s);  // enc2 weights (dec1's tap images replace them after P2); the caller's barrier publishes
}

// P2 .. P7 of the forward, one workgroup per sample.
template <class L>
__device__ __forceinline__ void fwd_rest(const FwdArgs& a, uint8_t* lds, int n) {
  float* Xs = reinterpret_cast<float*>(lds + L::X);
  float* W4s = reinterpret_cast<float*>(lds + L::W4);
  uint8_t* A1s = lds + L::A1;
  __bf16* A2s = reinterpret_cast<__bf16*>(lds + L::A2);
  uint8_t* D0u = lds + L::D0;  // img49 image
  float* Hs = reinterpret_cast<float*>(lds + L::H);
  __bf16* Zs = reinterpret_cast<__bf16*>(lds + L::Z);
  float* Scr = reinterpret_cast<float*>(lds + L::Scr);
  uint8_t* W3s = lds + L::IMG;
  __bf16* D1s = reinterpret_cast<__bf16*>(lds + L::D1);  // FwdLayout: aliases A1s (dead after enc2)

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Weights& W = a.w;

  stamp(a.stamps, 2);
  // the head's first weight row per wave (P3) is loaded now: its latency
  // hides under the enc2 MFMAs instead of opening P3
  bf16x8 wh0[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int k = 512 * i + 8 * lane;
    wh0[i] = *reinterpret_cast<const bf16x8*>(W.Wh + (size_t)w * kFlat + (k < kFlat ? k : 0));
  }
  // ---- P2: enc2 (32 -> 64, 14x14 -> 7x7, MFMA), ReLU
  const float* Bias = reinterpret_cast<const float*>(lds + L::Bias);
  conv14to7(A1s, [&](int j, int t) { return conv_bfrag(W3s, j, t, lane); }, [&](int, int col) { return Bias[kB2 + col]; },
            [&](int p, int col, float v, float bias) {
    const __bf16 o = (__bf16)fmaxf(v + bias, 0.f);
    A2s[p * 64 + col] = o;
    if (a.train) a.a2[(size_t)n * kFlat + p * 64 + col] = o;
  });
  lds_barrier();

  TapImageRegs w3r;
  w3r.load(W.W3);  // dec1 tap images: in flight during P3-P5, written after P5
  stamp(a.stamps, 3);
  // ---- P3: encoder head (3136 -> 64) on VALU with fully contiguous weight
  // loads. Wave w owns output rows o = w + 8c (c = 0..7); one row = 7 wave
  // loads of 1 KB (lane l covers k = 512i + 8l .. +7). A 16-row MFMA fragment
  // would touch 16 separate 64-B segments per load and the per-CU address
  // path (TA), not bandwidth, bounded that version (12.5 us; PMC TA_BUSY).
  // The next row's 7 loads are in flight while this row's dot products and
  // cross-lane reduction run.
  {
    bf16x8 av[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int k = 512 * i + 8 * lane;
      av[i] = k < kFlat ? *reinterpret_cast<const bf16x8*>(A2s + k) : zero8();
    }
    auto ld_row = [&](int o, bf16x8 (&v)[7]) {
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const int k = 512 * i + 8 * lane;
        v[i] = *reinterpret_cast<const bf16x8*>(W.Wh + (size_t)o * kFlat + (k < kFlat ? k : 0));
      }
    };
    bf16x8 vc[7], vn[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) vc[i] = wh0[i];
#pragma unroll 1
    for (int c = 0; c < 8; ++c) {
      if (c + 1 < 8) ld_row(w + 8 * (c + 1), vn);
      // v_dot2_f32_bf16 on the bf16 pairs (no bf16 -> f32 converts) into four
      // independent accumulators: a single fmaf chain of 56 dependent steps
      // per row, plus two converts per product, bounded this phase (PMC:
      // ~7k VALU instructions per wave in the fused step)
      // two K halves, [0, 1536) = loads i < 3 and [1536, 3136) = loads i >= 3,
      // each summed exactly as one half of the paired step sums it (same lane
      // chunks, same accumulator order, one wave_sum each), then (half 0 +
      // half 1) + bias: the solo fallback is bitwise the paired form
      float dq[4] = {0.f, 0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        if (512 * i + 8 * lane < kFlat) {
          float(&q)[4] = i < 3 ? dq : dr;
          q[0] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 0, 1),
                                                 __builtin_shufflevector(vc[i], vc[i], 0, 1), q[0], false);
          q[1] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 2, 3),
                                                 __builtin_shufflevector(vc[i], vc[i], 2, 3), q[1], false);
          q[2] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 4, 5),
                                                 __builtin_shufflevector(vc[i], vc[i], 4, 5), q[2], false);
          q[3] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(av[i], av[i], 6, 7),
                                                 __builtin_shufflevector(vc[i], vc[i], 6, 7), q[3], false);
        }
      }
      float d0 = (dq[0] + dq[1]) + (dq[2] + dq[3]);
      float d1 = (dr[0] + dr[1]) + (dr[2] + dr[3]);
      d0 = wave_sum(d0);
      d1 = wave_sum(d1);
      if (lane == 0) Hs[w + 8 * c] = (d0 + d1) + Bias[kBh + w + 8 * c];
#pragma unroll
      for (int i = 0; i < 7; ++i) vc[i] = vn[i];
    }
  }
  // P5's first 13 dec_fc weight loads, in flight across the barrier and P4
  const __bf16* wp5 = W.Wd + (size_t)(lane & 15) * 32 + 8 * (lane >> 4);
  auto wd5_ld = [&](int i) {
    const int t = w + 8 * i;
    return *reinterpret_cast<const bf16x8*>(wp5 + (size_t)(t < 196 ? t : 0) * 512);
  };
  bf16x8 wd5[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) wd5[i] = wd5_ld(i);
  lds_barrier();

  stamp(a.stamps, 4);
  // ---- P4: reparameterisation (Philox eps) + KLD
  if (tid < 64) {
    float kl = 0.f;
    if (tid < 32) {
      const int c = tid;
      const float mu = Hs[c], lv = Hs[32 + c];
      const unsigned long long stp = (unsigned long long)a.st->step;
      const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(n * 32 + c), a.stream, (uint32_t)(stp & 0xffffffffu),
                                             (uint32_t)(stp >> 32)},
                                       a.hp->seed_lo, a.hp->seed_hi);
      const float ep = normal_from_bits(bits.x, bits.y);
      const float sd = expf(0.5f * lv);
      const float zz = fmaf(ep, sd, mu);
      kl = fmaf(-sd, sd, fmaf(-mu, mu, 1.f + lv));  // explicit: one rounding sequence in both bodies
      Zs[c] = (__bf16)zz;
      reinterpret_cast<float*>(lds + L::Red)[c] = ep;  // the merged step's Q4 (Red is free after P3)
      if (a.train) {
        a.mulv[(size_t)n * 64 + c] = mu;
        a.mulv[(size_t)n * 64 + 32 + c] = lv;
        a.eps[(size_t)n * 32 + c] = ep;
        a.z16[(size_t)n * 32 + c] = (__bf16)zz;
      }
    }
    kl = wave_sum(kl);
    if (tid == 0) Scr[0] = -0.5f * kl;
  }
  lds_barrier();

  stamp(a.stamps, 5);
  // ---- P5: dec_fc (32 -> 3136, MFMA K = 32), ReLU. Wave w: n-tiles w + 8i.
  {
    const bf16x8 av = (lane & 15) == 0 ? *reinterpret_cast<const bf16x8*>(Zs + 8 * (lane >> 4)) : zero8();
    // n-tiles t = w + 8i (i < 25, t < 196): 2 chunks of 13 loads
    stream2_pre<13, 2>(
        wd5, wd5_ld,
        [&](int i, const bf16x8& b) {
          const int t = w + 8 * i;
          if (t < 196) {
            const f32x4 acc = mfma_bf16(av, b, f32x4{0.f, 0.f, 0.f, 0.f});
            if (lane < 16) {
              const int jj = 16 * t + lane;
              const __bf16 o = (__bf16)fmaxf(acc[0] + reinterpret_cast<const float*>(lds + L::Bd)[jj], 0.f);
              *reinterpret_cast<__bf16*>(D0u + img49e(jj >> 6, jj & 63)) = o;
              if (a.train) a.d0[(size_t)n * kFlat + jj] = o;
            }
          }
        });
  }
  w3r.store(W3s);
  lds_barrier();

  stamp(a.stamps, 6);
  // ---- P6: dec1 (convT 64 -> 32, 7x7 -> 14x14, MFMA), ReLU
  {
    float cs[4];
    tconv7to14(D0u, W3s, [&](int, int co) { return Bias[kB3 + co]; }, [&](int pix, int co, float v, float bias) {
      const __bf16 o = (__bf16)fmaxf(v + bias, 0.f);
      D1s[pix * 32 + co] = o;
      if (a.train) a.d1[((size_t)n * 196 + pix) * 32 + co] = o;
      return 0.f;
    }, cs);
  }
  lds_barrier();

  stamp(a.stamps, 7);
  // ---- P7: dec2 (convT 32 -> 1, 14x14 -> 28x28, VALU) + BCE + dlogits
  float loss = 0.f, gsum = 0.f;
  for (int pix = tid; pix < 784; pix += kThreads) {
    const int oy = pix / 28, ox = pix - 28 * (pix / 28);
    const int ca = oy & 1, cb = ox & 1, jy = oy >> 1, jx = ox >> 1;
    // channels 0..15 and 16..31 in two partial sums added last, as the
    // paired step's two halves (conv28_pair.h P7, exchanged in X3)
    float th[2] = {0.f, 0.f};
#pragma unroll 1
    for (int ty = 0; ty < 2; ++ty)
#pragma unroll
      for (int tx = 0; tx < 2; ++tx) {
        const int iy = jy + ca - ty, ix = jx + cb - tx;
        if ((unsigned)iy < 14u && (unsigned)ix < 14u) {
          const int tap = ((1 - ca) + 2 * ty) * 4 + (1 - cb) + 2 * tx;
          const bf16x8* dp = reinterpret_cast<const bf16x8*>(D1s + (iy * 14 + ix) * 32);
          const float4* wp = reinterpret_cast<const float4*>(W4s + tap * 32);
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) {
            const bf16x8 dv = dp[ch];
            const float4 w0 = wp[2 * ch], w1 = wp[2 * ch + 1];
            float& t = th[ch >> 1];
            t = fmaf((float)dv[0], w0.x, t); t = fmaf((float)dv[1], w0.y, t);
            t = fmaf((float)dv[2], w0.z, t); t = fmaf((float)dv[3], w0.w, t);
            t = fmaf((float)dv[4], w1.x, t); t = fmaf((float)dv[5], w1.y, t);
            t = fmaf((float)dv[6], w1.z, t); t = fmaf((float)dv[7], w1.w, t);
          }
        }
      }
    const float t = Bias[kB4] + (th[0] + th[1]);
    const float x = Xs[pix];
    const float p = 1.f / (1.f + expf(-t));
    const float g = p - x;
    const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
    loss += fmaf(x, fminf(sp_pos - t, 100.f), (1.f - x) * fminf(sp_pos, 100.f));  // explicit fma (see kl)
    gsum += g;
    if (a.train) a.dlog[(size_t)n * 784 + pix] = g;
    if constexpr (L::G >= 0) reinterpret_cast<float*>(lds + L::G)[pix] = g;  // the merged step's backward
    if (a.recon) a.recon[(size_t)n * 784 + pix] = p;
  }
  loss = wave_sum(loss);
  gsum = wave_sum(gsum);
  if (lane == 0) {
    Scr[8 + w] = loss;
    Scr[16 + w] = gsum;
  }
  lds_barrier();
  if (tid == 0) {
    float sl = 0.f, sg = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sl += Scr[8 + i];
      sg += Scr[16 + i];
    }
    a.bce_part[n] = sl;
    a.kld_part[n] = Scr[0];
    if (a.db4_part) a.db4_part[n] = sg;
  }
  stamp(a.stamps, 8);
}

template <class L>
__device__ __forceinline__ void fwd_body(const FwdArgs& a, uint8_t* lds, int n) {
  fwd_p01<L>(a, lds, n, [] {});
  lds_barrier();
  fwd_rest<L>(a, lds, n);
}


// ----------------------------------------------------------------- backward
constexpr int kBG = 0;                      // f32 [784] dlogits
constexpr int kBW4 = kBG + 784 * 4;         // f32 [16][32] dec2 weights, tap-major
constexpr int kBGD1 = kBW4 + 512 * 4;       // bf16 img14 [196][32]
constexpr int kBGD0 = kBGD1 + 196 * 64;     // bf16 [3136]
constexpr int kBDM = kBGD0 + kFlat * 2;     // f32 [64] d[mu|lv]
constexpr int kBDZR = kBDM + 64 * 4;        // f32 [2][8][32] dz wave partials (two K halves)
constexpr int kBGA2 = kBDZR + 512 * 4;      // bf16 [3136]
constexpr int kBGA2F = kBGA2 + kFlat * 2;   // f32 [3136] (colsum source)
constexpr int kBCS = kBGA2F + kFlat * 4;    // f32 [8][64] colsum scratch
constexpr int kBW2 = kBCS + 512 * 4;        // 16 x 4 KB enc2 tap images
constexpr int kBCSB = kBW2 + 65536;         // f32 [32][197] dec1-bias column-sum transpose
constexpr int kBLds = kBCSB + 32 * 197 * 4;
static_assert(kBGD1 % 16 == 0 && kBGD0 % 16 == 0 && kBGA2 % 16 == 0 && kBGA2F % 16 == 0 && kBW2 % 16 == 0,
              "LDS alignment");

struct BwdLayout {
  static constexpr int G = kBG, W4 = kBW4, GD1 = kBGD1, GD0 = kBGD0, DM = kBDM, DZR = kBDZR, GA2 = kBGA2;
  static constexpr int GA2F = kBGA2F, CS = kBCS, IMG = kBW2, CSB = kBCSB, LDS = kBLds;
  static constexpr int D1 = -1, D0 = -1, A2 = -1, A1 = -1, H = -1, Red = -1;  // from global memory
};

// MERGED: the backward runs in the forward's workgroup right after it (one
// launch per step) and takes from LDS what the forward left there: the
// dlogits (L::G), dec2 weights (W4), dec1's tap images (IMG; Q2 reads its
// conv-layout B fragments straight out of them), and the ReLU masks d1
// (A1 region), d0 (img49 D0 region) and a2 (A2 region).
template <class L, bool MERGED>
__device__ __forceinline__ void bwd_body(const BwdArgs& a, uint8_t* lds, int n) {
  float* Gs = reinterpret_cast<float*>(lds + L::G);
  float* W4s = reinterpret_cast<float*>(lds + L::W4);
  uint8_t* GD1s = lds + L::GD1;
  __bf16* GD0s = reinterpret_cast<__bf16*>(lds + L::GD0);
  float* DMs = reinterpret_cast<float*>(lds + L::DM);
  float* DZR = reinterpret_cast<float*>(lds + L::DZR);
  uint8_t* GA2u = lds + L::GA2;  // img49 image
  float* GA2F = reinterpret_cast<float*>(lds + L::GA2F);
  float* CS = reinterpret_cast<float*>(lds + L::CS);
  uint8_t* W2s = lds + L::IMG;
  float* CSB = reinterpret_cast<float*>(lds + L::CSB);

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Weights& W = a.w;
  stamp(a.stamps, 0);

  // ---- Q0: dlogits, dec2 weights, dec1 B fragments (conv layout), enc2 tap images
  if constexpr (!MERGED) {
    if (tid < 196) reinterpret_cast<float4*>(Gs)[tid] = reinterpret_cast<const float4*>(a.dlog + (size_t)n * 784)[tid];
    {
      const int c = tid >> 4, t = tid & 15;
      W4s[t * 32 + c] = W.W4f[tid];
    }
    stage_conv_image(W.W3, W2s);  // dec1 weights (conv layout) first; enc2's tap images after Q2
    lds_barrier();
  }

  stamp(a.stamps, 1);
  // ---- Q1: dec2 backward-data (conv 1 -> 32 on the dlogits, 28 -> 14) x dec1 ReLU mask,
  // on exact-f32 MFMA as enc1 in P1 (the paired body's Q1 runs the same per-
  // element MFMA sequence on its own channel tile: pair == solo bitwise).
  {
    const int col = lane & 15, kq = lane >> 4;
    float wa[2][4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wa[mt][ks] = W4s[(4 * ks + kq) * 32 + 16 * mt + col];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nt = w + 8 * j;
      if (nt < 13) {
        const int pix = 16 * nt + col;
        const bool live = pix < 196;
        const int oy = pix / 14, ox = pix - 14 * (pix / 14);
        float gb[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int t = 4 * ks + kq;
          const int iy = 2 * oy - 1 + (t >> 2), ix = 2 * ox - 1 + (t & 3);
          gb[ks] = live && (unsigned)iy < 28u && (unsigned)ix < 28u ? Gs[iy * 28 + ix] : 0.f;
        }
        f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) acc[mt] = mfma16x16x4(wa[mt][ks], gb[ks], acc[mt]);
        if (live) {
          typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
#pragma unroll
          for (int mt = 0; mt < 2; ++mt) {
            const int c0 = 16 * mt + 4 * kq;
            const bf16x4 m = MERGED ? *reinterpret_cast<const bf16x4*>(lds + L::D1 + pix * 64 + c0 * 2)
                                    : *reinterpret_cast<const bf16x4*>(a.d1 + ((size_t)n * 196 + pix) * 32 + c0);
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float v = (float)m[e] > 0.f ? acc[mt][e] : 0.f;
              o[e] = (__bf16)v;
              // dec1 bias partials: transposed through LDS, then 8 lanes per
              // channel sum strided pixels in a fixed order (below)
              CSB[(c0 + e) * 197 + pix] = v;
            }
            *reinterpret_cast<bf16x4*>(GD1s + img14(pix, c0 >> 3) + ((c0 & 7) << 1)) = o;
            *reinterpret_cast<bf16x4*>(a.gd1 + ((size_t)n * 196 + pix) * 32 + c0) = o;
          }
        }
      }
    }
  }
  lds_barrier();
  if (tid < 256) {
    const int c = tid >> 3, part = tid & 7;
    float s = 0.f;
    for (int p = part; p < 196; p += 8) s += CSB[c * 197 + p];
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (part == 0) a.db3_part[(size_t)n * 32 + c] = s;
  }

  stamp(a.stamps, 2);
  // Q3's first 13 weight loads, in flight during the Q2 MFMAs
  auto wd_ld = [&](int it) {
    const int jj = it * 128 + w * 16 + (lane >> 2);
    return *reinterpret_cast<const bf16x8*>(W.Wd + (size_t)(jj < kFlat ? jj : 0) * 32 + 8 * (lane & 3));
  };
  bf16x8 wd0[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) wd0[i] = wd_ld(i);
  // ---- Q2: dec1 backward-data (conv 32 -> 64 with the convT weights, 14 -> 7) x dec_fc ReLU mask
  conv14to7(GD1s,
            [&](int j, int t) {
              if constexpr (MERGED)  // dec1's per-tap image t: row c64 = 16 j + (l & 15), chunk l >> 4
                return *reinterpret_cast<const bf16x8*>(W2s + t * 4096 + timg<32>(16 * j + (lane & 15), lane >> 4));
              else
                return conv_bfrag(W2s, j, t, lane);
            },
            [&](int p, int col) {
              if constexpr (MERGED) return (float)*reinterpret_cast<const __bf16*>(lds + L::D0 + img49e(p, col));
              else return (float)a.d0[(size_t)n * kFlat + p * 64 + col];
            },
            [&](int p, int col, float v, float mask) {
    const size_t e = (size_t)n * kFlat + p * 64 + col;
    const float g = mask > 0.f ? v : 0.f;
    const __bf16 o = (__bf16)g;
    GD0s[p * 64 + col] = o;
    a.gd0[e] = o;
    a.dbd_part[e] = g;
  });
  lds_barrier();

  TapImageRegs w2r;
  w2r.load(W.W2);  // enc2 tap images: in flight during Q3-Q5, written before Q6
  stamp(a.stamps, 3);
  // ---- Q3: dec_fc backward-data dz = g . Wd (VALU over [3136][32] rows) ----
  {
    const int jr = lane >> 2;
    // two K halves (rows [0, 1536) = row groups it < 12, [1536, 3136) = it >= 12),
    // each accumulated and reduced exactly as one half of the paired step
    // (conv28_pair.h Q3); Q4 adds them in the paired order: bitwise the same dz
    float acc[8], acc1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = acc1[e] = 0.f;
    // 25 row groups of 128 (3136 rows): 2 chunks of 13 loads
    stream2_pre<13, 2>(
        wd0, wd_ld,
        [&](int it, const bf16x8& wv) {
          const int jj = it * 128 + w * 16 + jr;
          if (jj < kFlat) {
            const float g = (float)GD0s[jj];
            if (it < 12) {
#pragma unroll
              for (int e = 0; e < 8; ++e) acc[e] = fmaf(g, (float)wv[e], acc[e]);
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e) acc1[e] = fmaf(g, (float)wv[e], acc1[e]);
            }
          }
        });
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = acc[e], u = acc1[e];
      v += __shfl_xor(v, 4, 64);
      u += __shfl_xor(u, 4, 64);
      v += __shfl_xor(v, 8, 64);
      u += __shfl_xor(u, 8, 64);
      v += __shfl_xor(v, 16, 64);
      u += __shfl_xor(u, 16, 64);
      v += __shfl_xor(v, 32, 64);
      u += __shfl_xor(u, 32, 64);
      acc[e] = v;
      acc1[e] = u;
    }
    if (lane < 4) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        DZR[w * 32 + 8 * lane + e] = acc[e];
        DZR[256 + w * 32 + 8 * lane + e] = acc1[e];
      }
    }
  }
  // Q5's first 16 head-weight loads, in flight across the barrier and Q4
  const int k05 = 8 * (tid < kFlat / 8 ? tid : 0);
  auto wh_ld = [&](int o) { return *reinterpret_cast<const bf16x8*>(W.Wh + (size_t)o * kFlat + k05); };
  bf16x8 wh5[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) wh5[i] = wh_ld(i);
  lds_barrier();
  stamp(a.stamps, 4);
  // ---- Q4: reparameterisation backward -> d[mu | logvar]
  if (tid < 32) {
    const int c = tid;
    float dz0 = 0.f, dz1 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) dz0 += DZR[i * 32 + c];
#pragma unroll
    for (int i = 0; i < 8; ++i) dz1 += DZR[256 + i * 32 + c];
    const float dz = dz0 + dz1;  // the paired step's (role-0 part + role-1 part)
    const float beta = a.hp->kl_beta;
    // merged step: mu | logvar and eps from the forward's LDS (H, Red); else from memory
    const float* Hm = reinterpret_cast<const float*>(lds + L::H);
    const float mu = MERGED ? Hm[c] : a.mulv[(size_t)n * 64 + c];
    const float lv = MERGED ? Hm[32 + c] : a.mulv[(size_t)n * 64 + 32 + c];
    const float ep = MERGED ? reinterpret_cast<const float*>(lds + L::Red)[c] : a.eps[(size_t)n * 32 + c];
    const float sd = expf(0.5f * lv);
    const float dm = dz + beta * mu;
    const float dl = 0.5f * dz * ep * sd + 0.5f * beta * (sd * sd - 1.f);
    DMs[c] = dm;
    DMs[32 + c] = dl;
    a.dmulv[(size_t)n * 64 + c] = dm;
    a.dmulv[(size_t)n * 64 + 32 + c] = dl;
    a.dmulv16[(size_t)n * 64 + c] = (__bf16)dm;
    a.dmulv16[(size_t)n * 64 + 32 + c] = (__bf16)dl;
  }
  lds_barrier();

  stamp(a.stamps, 5);
  // ---- Q5: head backward-data g = dmulv . Wh (VALU over 392 chunks of 8) x enc2 ReLU mask
  if (tid < kFlat / 8) {
    const int k0 = 8 * tid;
    float acc[8], acc1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = acc1[e] = 0.f;
    // 64 weight rows: 4 chunks of 16 loads; rows 0..31 and 32..63 in two
    // accumulators added at the end, the paired step's two row groups
    stream2_pre<16, 4>(wh5, wh_ld,
                   [&](int o, const bf16x8& wv) {
                     const float dm = DMs[o];
                     if (o < 32) {
#pragma unroll
                       for (int e = 0; e < 8; ++e) acc[e] = fmaf(dm, (float)wv[e], acc[e]);
                     } else {
#pragma unroll
                       for (int e = 0; e < 8; ++e) acc1[e] = fmaf(dm, (float)wv[e], acc1[e]);
                     }
                   });
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = acc[e] + acc1[e];
    const bf16x8 mk = MERGED ? *reinterpret_cast<const bf16x8*>(lds + L::A2 + 2 * k0)
                             : *reinterpret_cast<const bf16x8*>(a.a2 + (size_t)n * kFlat + k0);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (float)mk[e] > 0.f ? acc[e] : 0.f;
      o[e] = (__bf16)v;
      GA2F[k0 + e] = v;
    }
    *reinterpret_cast<bf16x8*>(GA2u + img49(tid >> 3, tid & 7)) = o;
    *reinterpret_cast<bf16x8*>(a.ga2 + (size_t)n * kFlat + k0) = o;
  }
  w2r.store(W2s);
  lds_barrier();
  if (tid < 64) {  // enc2 bias partials: pixels 0..23 and 24..48 in order, a row per half as the paired step
    float s0 = 0.f, s1 = 0.f;
    for (int p = 0; p < 24; ++p) s0 += GA2F[p * 64 + tid];
    for (int p = 24; p < 49; ++p) s1 += GA2F[p * 64 + tid];
    if (a.db2_m2) {  // [2][M][64]
      a.db2_part[(size_t)n * 64 + tid] = s0;
      a.db2_part[(size_t)(a.db2_m2 + n) * 64 + tid] = s1;
    } else {
      a.db2_part[(size_t)n * 64 + tid] = s0 + s1;
    }
  }

  stamp(a.stamps, 6);
  // ---- Q6: enc2 backward-data (convT 64 -> 32 with the conv weights, 7 -> 14) x enc1 ReLU mask
  {
    float cs[4];
    tconv7to14(GA2u, W2s,
               [&](int pix, int co) {
                 if constexpr (MERGED)  // enc1's output is still in LDS (img14)
                   return (float)*reinterpret_cast<const __bf16*>(lds + L::A1 + img14(pix, co >> 3) + ((co & 7) << 1));
                 else
                   return (float)a.a1[((size_t)n * 196 + pix) * 32 + co];
               },
               [&](int pix, int co, float v, float mask) {
      const size_t e = ((size_t)n * 196 + pix) * 32 + co;
      const float g = mask > 0.f ? v : 0.f;
      a.ga1[e] = (__bf16)g;
      return g;
    }, cs);
    // item sums S[q][mt][col] (col = 16 nj + lane), combined below in the
    // paired step's order: half nj, wave i = (m-tile i & 3, classes i >> 2 and
    // (i >> 2) + 2) -- conv28_pair.h tconv7to14_half + its enc1-bias sum
    if (lane < 16) {
      const int mt = (w >> 1) & 3, col = 16 * (w & 1) + lane;
#pragma unroll
      for (int q = 0; q < 4; ++q) CS[(q * 4 + mt) * 32 + col] = cs[q];
    }
  }
  lds_barrier();
  if (tid < 32) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int mt = i & 3, q = i >> 2;
      s += CS[(q * 4 + mt) * 32 + tid] + CS[((q + 2) * 4 + mt) * 32 + tid];
    }
    a.db1_part[(size_t)n * 32 + tid] = s;
  }
  stamp(a.stamps, 7);
}


// ------------------------------------------------------- merged step (one launch)
// One LDS map for both halves; backward regions alias forward regions that are
// dead by then (noted per line). dec1's tap images stay in IMG from P5 to Q2,
// then enc2's tap images replace them for Q6.
struct StepLayout {
  static constexpr int IMG = 0;                  // 64 KB: W2 conv image (P0-P2), W3 taps (P5-Q2), W2 taps (Q6)
  static constexpr int W1 = IMG + 65536;         // f32 [16][32]
  static constexpr int CS = W1;                  //   bwd colsum scratch (W1 dead after P1)
  static constexpr int W4 = W1 + 512 * 4;        // f32 [16][32], both halves
  static constexpr int X = W4 + 512 * 4;         // f32 [784]
  static constexpr int DM = X;                   //   bwd d[mu|lv] (X dead after P7)
  static constexpr int DZR = X + 64 * 4;         //   bwd dz partials [2][8][32]
  static constexpr int G = X + 784 * 4;          // f32 [784] dlogits (P7 -> Q1)
  static constexpr int A1 = G + 784 * 4;         // bf16 img14: enc1 out (P2 input, Q6 mask)
  static constexpr int A2 = A1 + 196 * 64;       // bf16 [3136] enc2 out (P3 input, Q5 mask)
  static constexpr int D0 = A2 + kFlat * 2;      // bf16 img49 dec_fc out (P6 input, Q2 mask)
  static constexpr int GA2 = D0;                 //   bwd img49 (D0 dead after Q2)
  static constexpr int H = D0 + kFlat * 2;       // f32 [64]
  static constexpr int Z = H + 64 * 4;           // bf16 [32]
  static constexpr int Red = Z + 64;
  static constexpr int Scr = Red + 64 * 4;       // f32 [32]
  static constexpr int Dummy = Scr + 32 * 4;     // 8 KB DMA landing zone
  static constexpr int GD0 = Dummy;              //   bwd bf16 [3136]
  static constexpr int Bd = Dummy + 8192;        // f32 [3136] dec_fc bias (P5 only)
  static constexpr int GD1 = Bd;                 //   bwd bf16 img14
  static constexpr int CSB = Bd + kFlat * 4;     // f32 [32][197]
  static constexpr int D1 = CSB + 32 * 197 * 4;  // bf16 [196][32] dec1 out (P7 input, Q1 mask)
  static constexpr int GA2F = D1;                //   bwd f32 [3136] (D1 dead after Q1)
  static constexpr int Bias = D1 + kFlat * 4;   // f32 [256] small biases (+ a zero chunk at kZero)
  static constexpr int PTab = Bias + 1024;      // u64 [32] pointer table of the paired body (conv28_pair.h)
  static constexpr int LDS = PTab + 256;
  static_assert(W1 % 16 == 0 && X % 16 == 0 && G % 16 == 0 && A1 % 16 == 0 && A2 % 16 == 0 && D0 % 16 == 0 &&
                    Dummy % 16 == 0 && Bd % 16 == 0 && CSB % 16 == 0 && D1 % 16 == 0 && LDS <= 163840,
                "step LDS map");
  static_assert(196 * 64 <= kFlat * 4 && 64 * 4 + 512 * 4 <= 784 * 4 && kFlat * 2 <= 8192, "step LDS aliases");
};


}  // namespace f28
}  // namespace mdt
