#include <stdlib.h>
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
__global__ void __launch_bounds__(256) conv_loss_finalize_k(LossArgs la, int advance_step) {
  __shared__ float scratch[16];
  if (advance_step)
    loss_step_body(la, scratch);  // the fused 28x28 forward's eval batches (its forward reads the step first)
  else
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
// Adam (optional) + bf16 cast over the whole flat arena; used for the initial
// cast, after checkpoint loads and after a stream-side DDP all-reduce. One
// 16-B stream over [0, total): the 64-element padding between segments is
// zero in P, G, m and v and stays zero under Adam (m = v = 0, p = 0 - 0), so
// no per-segment loop is needed (the per-segment form was 15 us for the 28x28
// model's 0.37 M parameters: one dependent pass per segment).
__global__ void __launch_bounds__(256) adam_cast_k(float* P, const float* G, float* Mo, float* Vo, __bf16* w16,
                                                   long long total, const TrainState* st, const HParams* hp,
                                                   int do_adam) {
  __shared__ AdamC cs;
  AdamC c{};
  if (do_adam) c = adam_consts_block(st, hp, &cs);
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const long long n4 = total >> 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    f32x4 p = reinterpret_cast<const f32x4*>(P)[i];
    if (do_adam) {
      const f32x4 g = reinterpret_cast<const f32x4*>(G)[i];
      f32x4 m = reinterpret_cast<const f32x4*>(Mo)[i], v = reinterpret_cast<const f32x4*>(Vo)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_update(pj, mj, vj, g[j], c);
        p[j] = pj; m[j] = mj; v[j] = vj;
      }
      reinterpret_cast<f32x4*>(P)[i] = p;
      reinterpret_cast<f32x4*>(Mo)[i] = m;
      reinterpret_cast<f32x4*>(Vo)[i] = v;
    }
    bf16x4 h;
#pragma unroll
    for (int j = 0; j < 4; ++j) h[j] = (__bf16)p[j];
    reinterpret_cast<bf16x4*>(w16)[i] = h;
  }
}

template <bool FENCE>
__global__ void __launch_bounds__(kFinalizeThreads) grad_finalize_k(FinalizeArgs fa, BatchGather bg) {
  __shared__ float red[kFinalizeThreads];
  __shared__ AdamC cs;
  // next-batch gather blocks first (only when bg.xn is set): their dependent
  // cursor -> index -> row chain then overlaps the finalize units instead of
  // trailing the grid
  const int gb = bg.xn ? gather_blocks(bg.B) : 0;
  if ((int)blockIdx.x < gb) {
    batch_gather_body(bg, (int)blockIdx.x);
    return;
  }
  grad_finalize_body(fa, red, &cs, (int)blockIdx.x - gb);
  // diagnostic (MDT_FIN_FENCE=1): an explicit agent-scope release of the
  // parameter / bf16 stores before the kernel-end release
  if constexpr (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

__global__ void __launch_bounds__(256) wtrans_k(WtransArgs wa) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWtransLds];
  wtrans_body(wa, lds, blockIdx.x);
}

__global__ void __launch_bounds__(256) combine_reparam_k(CombineReparamArgs a) {
  __shared__ __attribute__((aligned(16))) float red[1024 + 16];
  if (combine_rows_ok(a.Z)) combine_reparam_rows_body(a, red, blockIdx.x);
  else combine_reparam_body(a, red, blockIdx.x);
}

__global__ void __launch_bounds__(256) combine_reparam_bwd_k(CombineReparamBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float red[1024];
  if (combine_rows_ok(a.Z)) combine_reparam_bwd_rows_body(a, red, blockIdx.x);
  else combine_reparam_bwd_body(a, red, blockIdx.x);
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
  // advance_cursor: bit 0 = advance the batch cursor, bit 1 = also advance the step (loss_step_body)
  const LossArgs la{bce_part, nb, kld_part, nk, reinterpret_cast<TrainState*>(st), reinterpret_cast<const HParams*>(hp),
                    advance_cursor & 1};
  hipLaunchKernelGGL(conv_loss_finalize_k, dim3(1), dim3(256), 0, s, la, (advance_cursor >> 1) & 1);
  return (int)hipGetLastError();
}

int mdt_step_begin(void* st, const void* hp, hipStream_t s) {
  hipLaunchKernelGGL(step_begin_k, dim3(1), dim3(64), 0, s, reinterpret_cast<TrainState*>(st),
                     reinterpret_cast<const HParams*>(hp));
  return (int)hipGetLastError();
}

int mdt_adam_cast(float* P, const float* G, float* Mo, float* Vo, void* w16, const void* segs, int nseg,
                  long long total, const void* st, const void* hp, int do_adam, hipStream_t s) {
  (void)segs;
  (void)nseg;
  if (total % 4 || ((uintptr_t)P | (uintptr_t)G | (uintptr_t)Mo | (uintptr_t)Vo) % 16 || (uintptr_t)w16 % 8) return 1;
  int blocks = cdivh(total / 4, 256);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_cast_k, dim3(blocks), dim3(256), 0, s, P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16), total,
                     reinterpret_cast<const TrainState*>(st), reinterpret_cast<const HParams*>(hp), do_adam);
  return (int)hipGetLastError();
}

int mdt_grad_finalize(float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs, const void* units,
                      int nunits, const void* st, const void* hp, int do_adam, const float* gX, const int* gidx,
                      float* xn, unsigned* xtag, int gB, hipStream_t s) {
  if (nunits <= 0) return 0;
  const FinalizeArgs fa{P, G, Mo, Vo, reinterpret_cast<__bf16*>(w16), reinterpret_cast<const GradSeg*>(segs),
                        reinterpret_cast<const GradUnit*>(units), reinterpret_cast<const TrainState*>(st),
                        reinterpret_cast<const HParams*>(hp), do_adam};
  const bool gather = xn && xtag && gX && gidx && gB > 0;
  const BatchGather bg{gX, gidx, reinterpret_cast<const TrainState*>(st), gather ? xn : nullptr, xtag, gB, nunits};
  const int grid = nunits + (gather ? gather_blocks(gB) : 0);
  static const bool fence = [] {
    const char* e = getenv("MDT_FIN_FENCE");
    return e && e[0] == '1';
  }();
  if (fence)
    hipLaunchKernelGGL(grad_finalize_k<true>, dim3(grid), dim3(kFinalizeThreads), 0, s, fa, bg);
  else
    hipLaunchKernelGGL(grad_finalize_k<false>, dim3(grid), dim3(kFinalizeThreads), 0, s, fa, bg);
  return (int)hipGetLastError();
}

int mdt_wtrans(const void* w16, void* w16t, const void* segs, const void* units, int nunits, hipStream_t s) {
  if (nunits <= 0) return 0;
  const WtransArgs wa{reinterpret_cast<const __bf16*>(w16), reinterpret_cast<__bf16*>(w16t),
                      reinterpret_cast<const GradSeg*>(segs), reinterpret_cast<const TrUnit*>(units)};
  hipLaunchKernelGGL(wtrans_k, dim3(nunits), dim3(256), 0, s, wa);
  return (int)hipGetLastError();
}

int mdt_combine_reparam(const float* slab, int ks, const float* bias, float* mulv, float* eps, void* z16, float* z32,
                        int B, int Z, const void* st, const void* hp, unsigned stream, float* kld_part, hipStream_t s) {
  const CombineReparamArgs a{slab, ks, splitk_rp(ks), bias, mulv, eps, reinterpret_cast<__bf16*>(z16), z32, B, Z,
                             reinterpret_cast<const TrainState*>(st), reinterpret_cast<const HParams*>(hp),
                             (uint32_t)stream, kld_part};
  hipLaunchKernelGGL(combine_reparam_k, dim3(combine_reparam_blocks(ks, B, Z)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int mdt_combine_reparam_bwd(const float* slab, int ks, const float* mulv, const float* eps, float* dmulv,
                            void* dmulv16, float* dz, int B, int Z, const void* hp, hipStream_t s) {
  const CombineReparamBwdArgs a{slab, ks, splitk_rp(ks), mulv, eps, dmulv, reinterpret_cast<__bf16*>(dmulv16), dz, B,
                                Z, reinterpret_cast<const HParams*>(hp)};
  hipLaunchKernelGGL(combine_reparam_bwd_k, dim3(combine_reparam_blocks(ks, B, Z)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int mdt_combine_reparam_blocks(int ks, int B, int Z) { return combine_reparam_blocks(ks, B, Z); }

}  // extern "C"
