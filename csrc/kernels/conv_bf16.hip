// Conv-VAE step kernels around the implicit-GEMM layers (conv_igemm.hip):
// batch gather, reparameterisation (+KLD) and its backward, logit-form BCE
// (+dlogits, +bias-gradient partials), loss ring update, and the optimizer
// tail: gradient finalisation (deterministic partial-slab reduction) with a
// fused Adam + bf16 cast, and the LDS-tiled parity-ordered weight transpose.
#include "common.h"
#include "vae_mlp.h"
#include "adam_common.h"
#include "conv_igemm.h"
#include "conv_small.h"

namespace mdt {

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

// dz (f32 [B, Z], from the decoder Linear's backward-data) -> d[mu|lv].
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

// logits f32 [B*P] vs target rows: BCE (logit form, -100 log clamp) partials,
// dlogits (bf16) for the decoder and, for single-channel images, the partial
// sums of dlogits = the last layer's bias gradient.
__global__ void __launch_bounds__(256) bce_logits_k(const float* logits, const float* X, const int* rows, int B,
                                                    int P, __bf16* dlog, float* recon, float* part, float* gpart) {
  __shared__ float scratch[16];
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float loss = 0.f, g = 0.f;
  if (e < (long long)B * P) {
    const int i = (int)(e / P), j = (int)(e - (long long)i * P);
    const float t = logits[e];
    const float x = X[(size_t)(rows ? rows[i] : i) * P + j];
    const float p = 1.f / (1.f + expf(-t));
    g = p - x;
    if (dlog) dlog[e] = (__bf16)g;
    if (recon) recon[e] = p;
    const float sp_pos = fmaxf(t, 0.f) + log1pf(expf(-fabsf(t)));
    loss = x * fminf(sp_pos - t, 100.f) + (1.f - x) * fminf(sp_pos, 100.f);
  }
  const float s = block_sum(loss, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
  if (gpart) {
    __syncthreads();
    const float gs = block_sum(g, scratch);
    if (threadIdx.x == 0) gpart[blockIdx.x] = gs;
  }
}

// Sum loss partials -> loss ring; advance step (optionally cursor).
__global__ void __launch_bounds__(256) conv_loss_finalize_k(LossArgs la) {
  __shared__ float scratch[16];
  loss_finalize_body(la, scratch);
}

// step++ and the Adam beta^t running products (first launch of a step).
__global__ void step_begin_k(TrainState* st, const HParams* hp) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st->step = st->step + 1;
    st->b1pow *= hp->beta1_d;
    st->b2pow *= hp->beta2_d;
  }
}

// ------------------------------------------------ optimizer tail ----
// Adam (optional) + bf16 cast over every segment; used for the initial cast,
// after checkpoint loads and after a DDP all-reduce.
__global__ void __launch_bounds__(256) adam_cast_k(float* P, const float* G, float* Mo, float* Vo, __bf16* w16,
                                                   const GradSeg* segs, int nseg, const TrainState* st,
                                                   const HParams* hp, int do_adam) {
  __shared__ AdamC cs;
  const AdamC c = adam_consts_block(st, hp, &cs);
  for (int s = 0; s < nseg; ++s) {
    const GradSeg sg = segs[s];
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < sg.numel;
         i += (long long)gridDim.x * blockDim.x) {
      const long long o = sg.off + i;
      float p = P[o];
      if (do_adam) {
        float m = Mo[o], v = Vo[o];
        adam_update(p, m, v, G[o], c);
        P[o] = p; Mo[o] = m; Vo[o] = v;
      }
      w16[o] = (__bf16)p;
    }
  }
}

// One unit = `count` consecutive elements of one segment. Threads t = rl*count
// + col sum partial rows rl, rl+rp, ... (rp = 512/count) of column col, then
// row lane 0 adds the rp sums in order: a fixed reduction tree, so results are
// bitwise reproducible (unlike f32 atomics). With do_adam the same thread
// applies Adam to the parameter and re-emits its bf16 copy.
__global__ void __launch_bounds__(512) grad_finalize_k(float* P, float* G, float* Mo, float* Vo, __bf16* w16,
                                                       const GradSeg* segs, const GradUnit* units,
                                                       const TrainState* st, const HParams* hp, int do_adam) {
  __shared__ float red[512];
  __shared__ AdamC cs;
  AdamC c{};
  if (do_adam) c = adam_consts_block(st, hp, &cs);
  const GradUnit u = units[blockIdx.x];
  const GradSeg sg = segs[u.seg];
  const int t = threadIdx.x, cnt = u.count, rp = 512 / cnt;
  const int col = t % cnt, rl = t / cnt;
  float acc = 0.f;
  if (sg.slab && rl < rp) {
    const float* p = sg.slab + u.start + col;
    const long long n = sg.numel;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = rl;
    for (; s + 3 * rp < sg.nsplit; s += 4 * rp) {
      a0 += p[(long long)s * n];
      a1 += p[(long long)(s + rp) * n];
      a2 += p[(long long)(s + 2 * rp) * n];
      a3 += p[(long long)(s + 3 * rp) * n];
    }
    for (; s < sg.nsplit; s += rp) a0 += p[(long long)s * n];
    acc = (a0 + a1) + (a2 + a3);
  }
  red[t] = acc;
  __syncthreads();
  if (rl == 0) {
    const long long o = sg.off + u.start + col;
    float g;
    if (sg.slab) {
      g = 0.f;
      for (int r = 0; r < rp; ++r) g += red[r * cnt + col];
      if (!do_adam) G[o] = g;  // the fused-Adam path consumes g in registers only
    } else {
      g = G[o];
    }
    if (do_adam) {
      float p = P[o], m = Mo[o], v = Vo[o];
      adam_update(p, m, v, g, c);
      P[o] = p; Mo[o] = m; Vo[o] = v;
      w16[o] = (__bf16)p;
    }
  }
}

// bf16 weights [CO][k][k][CI] -> parity-ordered transpose [s][s][CI][k/s][k/s][CO]
// (class (a, b) holds taps ky = a + s*ty, kx = b + s*tx) for the kModeTconv
// GEMM. One 64x64 (co, ci) tile of one tap per block, staged through LDS so
// both the read (ci-contiguous) and the write (co-contiguous) are coalesced.
__global__ void __launch_bounds__(256) wtrans_k(const __bf16* w16, __bf16* w16t, const GradSeg* segs,
                                                const TrUnit* units) {
  __shared__ unsigned short tile[64][66];
  const TrUnit u = units[blockIdx.x];
  const GradSeg sg = segs[u.seg];
  const int k = sg.k, s = sg.s, CI = sg.ci, CO = sg.co, T = k / s;
  const int ky = u.tap / k, kx = u.tap - ky * k;
  const int a = ky % s, ty = ky / s, b = kx % s, tx = kx / s;
  const unsigned short* src = reinterpret_cast<const unsigned short*>(w16) + sg.off;
  unsigned short* dst = reinterpret_cast<unsigned short*>(w16t) + sg.toff;
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int r = idx >> 6, c = idx & 63;
    const int co = u.co0 + r, ci = u.ci0 + c;
    if (co < CO && ci < CI) tile[r][c] = src[((long long)(co * k + ky) * k + kx) * CI + ci];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * 64; idx += 256) {
    const int r = idx >> 6, c = idx & 63;
    const int ci = u.ci0 + r, co = u.co0 + c;
    if (co < CO && ci < CI) dst[((((long long)(a * s + b) * CI + ci) * T + ty) * T + tx) * CO + co] = tile[c][r];
  }
}

}  // namespace mdt

using namespace mdt;

// ------------------------------------------------------------ host API ----
static inline int cdivh(long long a, long long b) { return (int)((a + b - 1) / b); }

extern "C" {

int mdt_reparam(const float* mulv, float* eps, void* z16, float* z32, int B, int Z, const void* st, const void* hp,
                unsigned stream, float* kld_part, hipStream_t s) {
  hipLaunchKernelGGL(reparam_k, dim3(cdivh((long long)B * Z, 256)), dim3(256), 0, s, mulv, eps,
                     reinterpret_cast<__bf16*>(z16), z32, B, Z, reinterpret_cast<const TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp), (uint32_t)stream, kld_part);
  return (int)hipGetLastError();
}

int mdt_reparam_bwd(const float* dz, const float* mulv, const float* eps, float* dmulv, void* dmulv16, int B, int Z,
                    const void* hp, hipStream_t s) {
  hipLaunchKernelGGL(reparam_bwd_k, dim3(cdivh((long long)B * Z, 256)), dim3(256), 0, s, dz, mulv, eps, dmulv,
                     reinterpret_cast<__bf16*>(dmulv16), B, Z, reinterpret_cast<const HParams*>(hp));
  return (int)hipGetLastError();
}

int mdt_gather_rows(const float* X, const int* idx, const void* st, int B, int M, int P, float* xb, hipStream_t s) {
  if (P % 4) return 1;
  int blocks = cdivh((long long)M * (P / 4), 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(gather_rows_k, dim3(blocks), dim3(256), 0, s, X, idx, reinterpret_cast<const TrainState*>(st),
                     B, M, P, xb);
  return (int)hipGetLastError();
}

int mdt_bce_logits(const float* logits, const float* X, const int* rows, int B, int P, void* dlog16, float* recon,
                   float* part, float* gpart, hipStream_t s) {
  hipLaunchKernelGGL(bce_logits_k, dim3(cdivh((long long)B * P, 256)), dim3(256), 0, s, logits, X, rows, B, P,
                     reinterpret_cast<__bf16*>(dlog16), recon, part, gpart);
  return (int)hipGetLastError();
}

int mdt_conv_loss_finalize(const float* bce_part, int nb, const float* kld_part, int nk, void* st, const void* hp,
                           int advance_cursor, hipStream_t s) {
  const LossArgs la{bce_part, nb, kld_part, nk, reinterpret_cast<TrainState*>(st), reinterpret_cast<const HParams*>(hp),
                    advance_cursor};
  hipLaunchKernelGGL(conv_loss_finalize_k, dim3(1), dim3(256), 0, s, la);
  return (int)hipGetLastError();
}

int mdt_step_begin(void* st, const void* hp, hipStream_t s) {
  hipLaunchKernelGGL(step_begin_k, dim3(1), dim3(64), 0, s, reinterpret_cast<TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp));
  return (int)hipGetLastError();
}

int mdt_adam_cast(float* P, const float* G, float* Mo, float* Vo, void* w16, const void* segs, int nseg,
                  long long total, const void* st, const void* hp, int do_adam, hipStream_t s) {
  int blocks = cdivh(total, 256 * 4);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_cast_k, dim3(blocks), dim3(256), 0, s, P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16),
                     reinterpret_cast<const GradSeg*>(segs), nseg, reinterpret_cast<const TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp), do_adam);
  return (int)hipGetLastError();
}

int mdt_grad_finalize(float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs, const void* units,
                      int nunits, const void* st, const void* hp, int do_adam, hipStream_t s) {
  if (nunits <= 0) return 0;
  hipLaunchKernelGGL(grad_finalize_k, dim3(nunits), dim3(512), 0, s, P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16),
                     reinterpret_cast<const GradSeg*>(segs), reinterpret_cast<const GradUnit*>(units),
                     reinterpret_cast<const TrainState*>(st), reinterpret_cast<const HParams*>(hp), do_adam);
  return (int)hipGetLastError();
}

int mdt_wtrans(const void* w16, void* w16t, const void* segs, const void* units, int nunits, hipStream_t s) {
  if (nunits <= 0) return 0;
  hipLaunchKernelGGL(wtrans_k, dim3(nunits), dim3(256), 0, s, reinterpret_cast<const __bf16*>(w16),
                     reinterpret_cast<__bf16*>(w16t), reinterpret_cast<const GradSeg*>(segs),
                     reinterpret_cast<const TrUnit*>(units));
  return (int)hipGetLastError();
}

}  // extern "C"
