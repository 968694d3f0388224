// Fused MLP-VAE training step for MI355X (gfx950).
//
// Model (parity: /root/reference/vae-hpo.py:19-58): fc1 D->H, fc21/fc22 H->Z,
// fc3 Z->H, fc4 H->D, ELBO = BCE(sum) + beta*KLD.  The whole step is seven
// launches (captured in one hipGraph by the runtime):
//
//   F1  h1    = relu(X[rows] W1^T + b1)                       MFMA f32, split-K 4
//   F2  [mu|lv] = h1 W2^T + b2 ; z = mu + eps*exp(lv/2) (Philox) ; KLD partial ;
//       h3 = relu(z W3^T + b3)                                 16 rows / block
//   F3  logits = h3 W4^T + b4 ; dlogits = sigmoid - x ; BCE partial (logit form)
//   B1  dh3 = (dlogits W4) . [h3>0]    ||  dW4 = dlogits^T h3, db4
//   B2  dz = dh3 W3 -> dmu, dlv (reparam + beta-KLD) ; dh1 = ([dmu|dlv] W2) . [h1>0]
//                                      ||  dW3 = dh3^T z, db3
//   B3  dW2 = [dmu|dlv]^T h1, db2      ||  dW1 = dh1^T X[rows], db1
//   (+ bucketed all-reduce on the comm stream, then fused Adam: adam.hip)
//
// Gradients are written (not accumulated) straight into the flat gradient
// arena, so there is no zero_grad and no bucket copy-back. The batch rows are
// gathered by sampler index inside F1/F3/B3 (no host collate, no H2D copy).
// The batch cursor and step counter are device-resident so one captured graph
// replays over an entire epoch.
#include "common.h"
#include "tile_gemm.h"
#include "vae_mlp.h"

namespace mdt {

__device__ __forceinline__ const int* batch_rows(const VaeArgs& a) {
  return a.idx + (size_t)a.st->cursor * a.B;
}

// ------------------------------------------------------------------- F1 ----
struct EpiBiasRelu {
  float* out; const float* bias; int ld, M, N;
  __device__ __forceinline__ float operator()(int i, int j, float v, bool) const {
    if (i < M && j < N) out[(size_t)i * ld + j] = fmaxf(v + bias[j], 0.f);
    return 0.f;
  }
};

__global__ void __launch_bounds__(256) vae_f1(VaeArgs a) {
  __shared__ float lds[4 * 256];
  const int* rows = batch_rows(a);
  ARowGather A{a.X, rows, a.D, a.M, a.D};
  BWeightNT Bw{a.W1, a.D, a.H, a.D};
  EpiBiasRelu epi{a.h1, a.b1, a.H, a.M, a.H};
  gemm_tiles<1>(A, Bw, epi, a.D, (a.M + 15) / 16, (a.H + 15) / 16, -1, blockIdx.x, lds);
}

// ------------------------------------------------------------------- F2 ----
// One block = 16 batch rows. Stage A: [mu|lv](16 x 2Z) = h1 W2^T, split over 4
// waves along k. Stage B: reparameterise + KLD. Stage C: h3 = relu(z W3^T + b3).
// Requires Z <= 32 (2Z <= 64 -> <= 4 n-tiles).
__global__ void __launch_bounds__(256) vae_f2(VaeArgs a) {
  __shared__ float red[4][4][256];   // [wave][ntile][lane*4+r]
  __shared__ float zt[16][36];       // z tile (row-major, k padded)
  __shared__ float scratch[16];
  const int w = wave_id(), lane = lane_id();
  const int i0 = blockIdx.x * 16;
  const int Z2 = 2 * a.Z;
  const int ntj = (Z2 + 15) / 16;
  // Stage A
  {
    ARowMajor A{a.h1, a.H, a.M, a.H};
    BWeightNT Bw{a.W2, a.H, Z2, a.H};
    const int nch = (a.H + 15) / 16;
    const int kc0 = (w * nch) / 4, kc1 = ((w + 1) * nch) / 4;
    for (int tj = 0; tj < 4; ++tj) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (tj < ntj) acc = wave_tile(A, Bw, i0, tj * 16, kc0, kc1);
      float* m = &red[w][tj][lane * 4];
      m[0] = acc[0]; m[1] = acc[1]; m[2] = acc[2]; m[3] = acc[3];
    }
  }
  __syncthreads();
  // Stage B: thread t -> (row r = t / Z, latent c = t % Z), loop over 16*Z.
  float kld = 0.f;
  const uint32_t step_lo = (uint32_t)(a.st->step & 0xffffffffu);
  const uint32_t step_hi = (uint32_t)((uint64_t)a.st->step >> 32);
  for (int e = threadIdx.x; e < 16 * a.Z; e += blockDim.x) {
    const int r = e / a.Z, c = e - r * a.Z;
    const int i = i0 + r;
    // fetch accumulated value of output column col for row r from red[][][]
    auto acc_at = [&](int col) {
      const int tj = col >> 4, cc = col & 15;
      const int l = ((r >> 2) << 4) + cc;  // lane holding (row r, col cc)
      const int rr = r & 3;
      return red[0][tj][l * 4 + rr] + red[1][tj][l * 4 + rr] + red[2][tj][l * 4 + rr] +
             red[3][tj][l * 4 + rr];
    };
    float zz = 0.f;
    if (i < a.M) {
      const float mu = acc_at(c) + a.b2[c];
      const float lv = acc_at(a.Z + c) + a.b2[a.Z + c];
      const float sd = expf(0.5f * lv);
      // counter: (row*Z + c, step) keyed by the trial seed; the sampler row id
      // is deliberately NOT used so replicas of one group draw independent eps
      // only through their seed (parity with per-process randn_like streams).
      const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(i * a.Z + c), a.rng_stream, step_lo, step_hi},
                                       a.hp->seed_lo, a.hp->seed_hi);
      const float ep = normal_from_bits(bits.x, bits.y);
      zz = mu + ep * sd;
      const size_t o = (size_t)i * Z2;
      a.mulv[o + c] = mu;
      a.mulv[o + a.Z + c] = lv;
      a.eps[(size_t)i * a.Z + c] = ep;
      a.z[(size_t)i * a.Z + c] = zz;
      kld += 1.f + lv - mu * mu - sd * sd;
    }
    zt[r][c] = zz;
  }
  // pad k columns of z up to a multiple of 4 with zeros (ARowMajor over LDS)
  for (int e = threadIdx.x; e < 16 * 36; e += blockDim.x) {
    const int r = e / 36, c = e % 36;
    if (c >= a.Z) zt[r][c] = 0.f;
  }
  const float ks = block_sum(kld, scratch);
  if (threadIdx.x == 0) a.partials[kKldPartial + blockIdx.x] = -0.5f * ks;
  __syncthreads();
  // Stage C: h3 tiles; z from LDS (k = Z <= 32 -> two 16-chunks max)
  {
    const int ntiles = (a.H + 15) / 16;
    const int r = lane & 15, q = lane >> 4;
    for (int tj = w; tj < ntiles; tj += 4) {
      const int j = tj * 16 + r;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const float* wrow = j < a.H ? a.W3 + (size_t)j * a.Z : nullptr;
      for (int k0 = 0; k0 < a.Z; k0 += 16) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = k0 + 4 * q + t;
          const float av = (k < a.Z) ? zt[r][k] : 0.f;
          const float bv = (wrow && k < a.Z) ? wrow[k] : 0.f;
          acc = mfma16x16x4(av, bv, acc);
        }
      }
      const int row0 = i0 + 4 * q;
      const int col = j;
      if (col < a.H) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int i = row0 + rr;
          if (i < a.M) a.h3[(size_t)i * a.H + col] = fmaxf(acc[rr] + a.b3[col], 0.f);
        }
      }
    }
  }
}

// ------------------------------------------------------------------- F3 ----
struct EpiBce {
  const float* X; const int* rows; const float* bias; float* dlog; float* recon;
  int D, M, train;
  __device__ __forceinline__ float operator()(int i, int j, float v, bool) const {
    if (i >= M || j >= D) return 0.f;
    const float t = v + bias[j];
    const float x = X[(size_t)rows[i] * D + j];
    const float p = 1.f / (1.f + expf(-t));
    if (train) dlog[(size_t)i * D + j] = p - x;
    if (recon) recon[(size_t)i * D + j] = p;
    // -[x log p + (1-x) log(1-p)] in the overflow-free logit form, with the
    // reference's log clamp at -100 (torch binary_cross_entropy) preserved.
    const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));  // -log(1-p)
    const float sp_neg = sp_pos - t;                                 // -log p
    return x * fminf(sp_neg, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
  }
};

__global__ void __launch_bounds__(256) vae_f3(VaeArgs a) {
  __shared__ float lds[4 * 256];
  __shared__ float scratch[16];
  const int* rows = batch_rows(a);
  ARowMajor A{a.h3, a.H, a.M, a.H};
  BWeightNT Bw{a.W4, a.H, a.D, a.H};
  EpiBce epi{a.X, rows, a.b4, a.dlog, a.recon, a.D, a.M, a.train};
  const float c = gemm_tiles<2>(A, Bw, epi, a.H, (a.M + 15) / 16, (a.D + 15) / 16, -1, blockIdx.x, lds);
  const float s = block_sum(c, scratch);
  if (threadIdx.x == 0) a.partials[kBcePartial + blockIdx.x] = s;
}

// ------------------------------------------------------------------- B1 ----
struct EpiMask {
  float* out; const float* mask; int ld, M, N;
  __device__ __forceinline__ float operator()(int i, int j, float v, bool) const {
    if (i < M && j < N) {
      const size_t o = (size_t)i * ld + j;
      out[o] = mask[o] > 0.f ? v : 0.f;
    }
    return 0.f;
  }
};

struct EpiWGrad {  // weight grad [M=out, N=in] + bias grad [M]
  float* gw; float* gb; int ld, M, N;
  __device__ __forceinline__ float operator()(int i, int j, float v, bool is_bias) const {
    if (i >= M) return 0.f;
    if (is_bias) {
      if (j == 0) gb[i] = v;
    } else if (j < N) {
      gw[(size_t)i * ld + j] = v;
    }
    return 0.f;
  }
};

__global__ void __launch_bounds__(256) vae_b1(VaeArgs a, int nblk_dh3) {
  __shared__ float lds[4 * 256];
  if ((int)blockIdx.x < nblk_dh3) {
    ARowMajor A{a.dlog, a.D, a.M, a.D};
    BRowMajor Bw{a.W4, a.H, a.H, a.D};
    EpiMask epi{a.dh3, a.h3, a.H, a.M, a.H};
    gemm_tiles<1>(A, Bw, epi, a.D, (a.M + 15) / 16, (a.H + 15) / 16, -1, blockIdx.x, lds);
  } else {
    // dW4[D, H] = dlog^T h3, k = batch
    ATrans A{a.dlog, a.D, a.D, a.M};
    BRowMajor Bh{a.h3, a.H, a.H, a.M};
    EpiWGrad epi{a.gW4, a.gb4, a.H, a.D, a.H};
    const int tj = (a.H + 15) / 16;
    gemm_tiles<4>(A, Bh, epi, a.M, (a.D + 15) / 16, tj + 1, tj, blockIdx.x - nblk_dh3, lds);
  }
}

// ------------------------------------------------------------------- B2 ----
// Blocks [0, nrow): 16-row fused dz -> (dmu, dlv) -> dh1.
// Blocks [nrow, ...): dW3 = dh3^T z, db3.
__global__ void __launch_bounds__(256) vae_b2(VaeArgs a, int nrow) {
  __shared__ float red[4][2][256];
  __shared__ float dml[16][68];  // [row][dmu(Z) | dlv(Z)], padded
  if ((int)blockIdx.x >= nrow) {
    float* lds = &red[0][0][0];  // 2048 floats >= 4*256
    ATrans A{a.dh3, a.H, a.H, a.M};
    BRowMajor Bz{a.z, a.Z, a.Z, a.M};
    EpiWGrad epi{a.gW3, a.gb3, a.Z, a.H, a.Z};
    const int tj = (a.Z + 15) / 16;
    gemm_tiles<4>(A, Bz, epi, a.M, (a.H + 15) / 16, tj + 1, tj, blockIdx.x - nrow, lds);
    return;
  }
  const int w = wave_id(), lane = lane_id();
  const int i0 = blockIdx.x * 16;
  const int Z2 = 2 * a.Z;
  // dz (16 x Z) = dh3 (16 x H) W3 (H x Z), split-K over 4 waves
  {
    ARowMajor A{a.dh3, a.H, a.M, a.H};
    BRowMajor Bw{a.W3, a.Z, a.Z, a.H};
    const int nch = (a.H + 15) / 16;
    const int kc0 = (w * nch) / 4, kc1 = ((w + 1) * nch) / 4;
    for (int tj = 0; tj < 2; ++tj) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if (tj * 16 < a.Z) acc = wave_tile(A, Bw, i0, tj * 16, kc0, kc1);
      float* m = &red[w][tj][lane * 4];
      m[0] = acc[0]; m[1] = acc[1]; m[2] = acc[2]; m[3] = acc[3];
    }
  }
  __syncthreads();
  const float beta = a.hp->kl_beta;
  for (int e = threadIdx.x; e < 16 * a.Z; e += blockDim.x) {
    const int r = e / a.Z, c = e - r * a.Z;
    const int i = i0 + r;
    const int tj = c >> 4, cc = c & 15;
    const int l = ((r >> 2) << 4) + cc, rr = r & 3;
    const float dz = red[0][tj][l * 4 + rr] + red[1][tj][l * 4 + rr] + red[2][tj][l * 4 + rr] +
                     red[3][tj][l * 4 + rr];
    float dmu = 0.f, dlv = 0.f;
    if (i < a.M) {
      const float mu = a.mulv[(size_t)i * Z2 + c];
      const float lv = a.mulv[(size_t)i * Z2 + a.Z + c];
      const float ep = a.eps[(size_t)i * a.Z + c];
      const float sd = expf(0.5f * lv);
      // L = BCE + beta * (-0.5 sum(1 + lv - mu^2 - e^lv)), z = mu + eps*sd
      dmu = dz + beta * mu;
      dlv = 0.5f * dz * ep * sd + 0.5f * beta * (sd * sd - 1.f);
      a.dmulv[(size_t)i * Z2 + c] = dmu;
      a.dmulv[(size_t)i * Z2 + a.Z + c] = dlv;
    }
    dml[r][c] = dmu;
    dml[r][a.Z + c] = dlv;
  }
  for (int e = threadIdx.x; e < 16 * 68; e += blockDim.x) {
    const int r = e / 68, c = e % 68;
    if (c >= Z2) dml[r][c] = 0.f;
  }
  __syncthreads();
  // dh1 (16 x H) = dml (16 x 2Z) W2 (2Z x H), masked by h1 > 0
  {
    const int ntiles = (a.H + 15) / 16;
    const int r = lane & 15, q = lane >> 4;
    for (int tj = w; tj < ntiles; tj += 4) {
      const int j = tj * 16 + r;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k0 = 0; k0 < Z2; k0 += 16) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = k0 + 4 * q + t;
          const float av = (k < Z2) ? dml[r][k] : 0.f;
          const float bv = (j < a.H && k < Z2) ? a.W2[(size_t)k * a.H + j] : 0.f;
          acc = mfma16x16x4(av, bv, acc);
        }
      }
      if (j < a.H) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int i = i0 + 4 * q + rr;
          if (i < a.M) {
            const size_t o = (size_t)i * a.H + j;
            a.dh1[o] = a.h1[o] > 0.f ? acc[rr] : 0.f;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------- B3 ----
__global__ void __launch_bounds__(256) vae_b3(VaeArgs a, int nblk_w2) {
  __shared__ float lds[4 * 256];
  const int Z2 = 2 * a.Z;
  if ((int)blockIdx.x < nblk_w2) {
    ATrans A{a.dmulv, Z2, Z2, a.M};
    BRowMajor Bh{a.h1, a.H, a.H, a.M};
    EpiWGrad epi{a.gW2, a.gb2, a.H, Z2, a.H};
    const int tj = (a.H + 15) / 16;
    gemm_tiles<4>(A, Bh, epi, a.M, (Z2 + 15) / 16, tj + 1, tj, blockIdx.x, lds);
  } else {
    const int* rows = batch_rows(a);
    ATrans A{a.dh1, a.H, a.H, a.M};
    BRowGather Bx{a.X, rows, a.D, a.D, a.M};
    EpiWGrad epi{a.gW1, a.gb1, a.D, a.H, a.D};
    const int tj = (a.D + 15) / 16;
    gemm_tiles<4>(A, Bx, epi, a.M, (a.H + 15) / 16, tj + 1, tj, blockIdx.x - nblk_w2, lds);
  }
}

// --------------------------------------------------------------- decode ----
// Sampling path (/root/reference/vae-hpo.py:163-170): x = sigmoid(fc4(relu(fc3(z)))).
struct EpiSigmoid {
  float* out; const float* bias; int ld, M, N;
  __device__ __forceinline__ float operator()(int i, int j, float v, bool) const {
    if (i < M && j < N) out[(size_t)i * ld + j] = 1.f / (1.f + expf(-(v + bias[j])));
    return 0.f;
  }
};

__global__ void __launch_bounds__(256) vae_dec1(VaeArgs a, const float* zin) {
  __shared__ float lds[4 * 256];
  ARowMajor A{zin, a.Z, a.M, a.Z};
  BWeightNT Bw{a.W3, a.Z, a.H, a.Z};
  EpiBiasRelu epi{a.h3, a.b3, a.H, a.M, a.H};
  gemm_tiles<4>(A, Bw, epi, a.Z, (a.M + 15) / 16, (a.H + 15) / 16, -1, blockIdx.x, lds);
}

__global__ void __launch_bounds__(256) vae_dec2(VaeArgs a) {
  __shared__ float lds[4 * 256];
  ARowMajor A{a.h3, a.H, a.M, a.H};
  BWeightNT Bw{a.W4, a.H, a.D, a.H};
  EpiSigmoid epi{a.recon, a.b4, a.D, a.M, a.D};
  gemm_tiles<2>(A, Bw, epi, a.H, (a.M + 15) / 16, (a.D + 15) / 16, -1, blockIdx.x, lds);
}

// -------------------------------------------------------------- host side ----
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

VaeGrid vae_grid(int M, int D, int H, int Z) {
  VaeGrid g;
  const int ti = cdiv(M, 16);
  g.f1 = ti * cdiv(H, 16);
  g.f2 = ti;
  g.f3 = cdiv(ti * cdiv(D, 16), 2);
  g.b1_dh3 = ti * cdiv(H, 16);
  g.b1 = g.b1_dh3 + cdiv(cdiv(D, 16) * (cdiv(H, 16) + 1), 4);
  g.b2_rows = ti;
  g.b2 = g.b2_rows + cdiv(cdiv(H, 16) * (cdiv(Z, 16) + 1), 4);
  g.b3_w2 = cdiv(cdiv(2 * Z, 16) * (cdiv(H, 16) + 1), 4);
  g.b3 = g.b3_w2 + cdiv(cdiv(H, 16) * (cdiv(D, 16) + 1), 4);
  return g;
}

}  // namespace mdt

using namespace mdt;

extern "C" int mdt_vae_check(const VaeArgs* a) {
  if (a->M <= 0 || a->M > a->B || a->B > kMaxBatch) return 1;
  if (a->Z > 32 || a->Z <= 0) return 2;
  if ((a->D & 3) || (a->H & 3)) return 3;  // float4 alignment of row-major operands
  const VaeGrid g = vae_grid(a->M, a->D, a->H, a->Z);
  if (g.f2 > kBcePartial - kKldPartial) return 4;
  if (g.f3 > kPartials - kBcePartial) return 5;
  return 0;
}

extern "C" int mdt_vae_forward(const VaeArgs* a, hipStream_t s) {
  const int rc = mdt_vae_check(a);
  if (rc) return rc;
  const VaeGrid g = vae_grid(a->M, a->D, a->H, a->Z);
  hipLaunchKernelGGL(vae_f1, dim3(g.f1), dim3(256), 0, s, *a);
  hipLaunchKernelGGL(vae_f2, dim3(g.f2), dim3(256), 0, s, *a);
  hipLaunchKernelGGL(vae_f3, dim3(g.f3), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}

extern "C" int mdt_vae_backward(const VaeArgs* a, hipStream_t s, int part) {
  const int rc = mdt_vae_check(a);
  if (rc) return rc;
  const VaeGrid g = vae_grid(a->M, a->D, a->H, a->Z);
  if (part == 0 || part == 1) hipLaunchKernelGGL(vae_b1, dim3(g.b1), dim3(256), 0, s, *a, g.b1_dh3);
  if (part == 0 || part == 2) hipLaunchKernelGGL(vae_b2, dim3(g.b2), dim3(256), 0, s, *a, g.b2_rows);
  if (part == 0 || part == 3) hipLaunchKernelGGL(vae_b3, dim3(g.b3), dim3(256), 0, s, *a, g.b3_w2);
  return (int)hipGetLastError();
}

extern "C" int mdt_vae_decode(const VaeArgs* a, const float* zin, hipStream_t s) {
  if (a->M <= 0 || a->M > a->B || !a->recon) return 1;
  const int ti = (a->M + 15) / 16;
  hipLaunchKernelGGL(vae_dec1, dim3((ti * ((a->H + 15) / 16) + 3) / 4), dim3(256), 0, s, *a, zin);
  hipLaunchKernelGGL(vae_dec2, dim3((ti * ((a->D + 15) / 16) + 1) / 2), dim3(256), 0, s, *a);
  return (int)hipGetLastError();
}
