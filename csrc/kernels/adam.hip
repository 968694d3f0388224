// Single-launch fused Adam over a flat parameter arena (MI355X, gfx950).
//
// Replaces torch's foreach Adam (~8-10 multi-tensor launches per step over 10
// tensors, /root/reference/vae-hpo.py:131,74) with one memory-bound pass:
// per element 4 reads (p, g, m, v) + 3 writes, float4-vectorised, grid-stride.
// Numerics follow torch.optim.Adam (non-amsgrad, L2 weight decay) operation
// for operation: m.lerp_(g, 1-b1); v = b2*v + (1-b2)*g*g;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
//
// The kernel also closes the training step without an extra launch: the last
// workgroup to arrive (relaxed agent-scope ticket) reduces the loss partials
// written by the forward kernels into the device loss ring, and advances the
// device step counter and batch cursor that the next replay of the captured
// step graph reads. Every block reads `step` before it takes its ticket, so
// the increment by the last arriver cannot race a reader.
#include "common.h"
#include "vae_mlp.h"

namespace mdt {

struct AdamArgs {
  float* p; const float* g; float* m; float* v;
  long long n4;            // number of float4 groups
  const HParams* hp;
  TrainState* st;
  const float* partials;   // may be null (no loss finalize)
  int nkld, nbce;
  int advance;             // bit 0: step++, bit 1: cursor++ (training: 3)
  int decoupled_wd;        // 1: AdamW
};

__device__ void finalize_step(const AdamArgs& a, long long step, float* scratch) {
  float s_b = 0.f, s_k = 0.f;
  if (a.partials) {
    for (int i = threadIdx.x; i < a.nbce; i += blockDim.x) s_b += a.partials[kBcePartial + i];
    for (int i = threadIdx.x; i < a.nkld; i += blockDim.x) s_k += a.partials[kKldPartial + i];
  }
  const float bce = block_sum(s_b, scratch);
  __syncthreads();
  const float kld = block_sum(s_k, scratch);
  if (threadIdx.x == 0) {
    TrainState* st = a.st;
    if (a.partials) {
      const float loss = bce + a.hp->kl_beta * kld;
      st->loss_hist[step % kLossHist] = loss;
      st->epoch_loss += (double)loss;
      st->epoch_count += 1.0;
    }
    if (a.advance & 1) st->step = step + 1;
    if (a.advance & 2) {
      int c = st->cursor + 1;
      if (st->nbatches > 0 && c >= st->nbatches) c = 0;
      st->cursor = c;
    }
    st->ticket = 0;
  }
}

__global__ void __launch_bounds__(256) adam_flat(AdamArgs a) {
  __shared__ double sh[4];
  __shared__ float scratch[16];
  __shared__ int last;
  if (threadIdx.x == 0) {
    const long long t = a.st->step + 1;
    const double b1 = a.hp->beta1, b2 = a.hp->beta2;
    const double bc1 = 1.0 - pow(b1, (double)t);
    const double bc2 = 1.0 - pow(b2, (double)t);
    sh[0] = (double)a.hp->lr / bc1;  // step_size
    sh[1] = sqrt(bc2);               // bias_correction2_sqrt
    sh[2] = (double)t;
  }
  __syncthreads();
  const float step_size = (float)sh[0];
  const float bc2s = (float)sh[1];
  const long long step = (long long)sh[2] - 1;
  const float b1 = a.hp->beta1, b2 = a.hp->beta2, eps = a.hp->eps;
  const float wd = a.hp->weight_decay, gs = a.hp->grad_scale, lr = a.hp->lr;
  float4* P = reinterpret_cast<float4*>(a.p);
  const float4* G = reinterpret_cast<const float4*>(a.g);
  float4* Mv = reinterpret_cast<float4*>(a.m);
  float4* Vv = reinterpret_cast<float4*>(a.v);
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < a.n4; i += stride) {
    float4 p = P[i], g = G[i], m = Mv[i], v = Vv[i];
    float* pp = &p.x; float* gg = &g.x; float* mm = &m.x; float* vv = &v.x;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float gr = gg[c] * gs;
      if (wd != 0.f) {
        if (a.decoupled_wd) pp[c] *= (1.f - lr * wd);
        else gr = fmaf(wd, pp[c], gr);
      }
      mm[c] = fmaf(1.f - b1, gr - mm[c], mm[c]);         // lerp
      vv[c] = fmaf(1.f - b2, gr * gr, vv[c] * b2);        // mul_ + addcmul_
      const float denom = sqrtf(vv[c]) / bc2s + eps;
      pp[c] = pp[c] - step_size * (mm[c] / denom);        // addcdiv_
    }
    P[i] = p; Mv[i] = m; Vv[i] = v;
  }
  // ---- last-arriver finalize (loss ring, step/cursor advance) ----
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned tk = __hip_atomic_fetch_add(&a.st->ticket, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    last = (tk == gridDim.x - 1);
  }
  __syncthreads();
  if (last) finalize_step(a, step, scratch);
}

// Loss-only finalize for eval batches (no optimizer): one block.
__global__ void __launch_bounds__(256) loss_finalize(AdamArgs a) {
  __shared__ float scratch[16];
  finalize_step(a, a.st->step, scratch);
}

}  // namespace mdt

using namespace mdt;

extern "C" int mdt_adam_step(float* p, const float* g, float* m, float* v, long long n,
                             const HParams* hp, TrainState* st, const float* partials,
                             int nkld, int nbce, int advance, int decoupled_wd, int max_blocks,
                             hipStream_t s) {
  if (n % 4) return 1;
  AdamArgs a{p, g, m, v, n / 4, hp, st, partials, nkld, nbce, advance, decoupled_wd};
  long long blocks = (a.n4 + 255) / 256;
  // Enough blocks to fill 256 CUs several times over, grid-stride beyond that.
  const long long cap = max_blocks > 0 ? max_blocks : 2048;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_flat, dim3((unsigned)blocks), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int mdt_loss_finalize(const HParams* hp, TrainState* st, const float* partials,
                                 int nkld, int nbce, int advance, hipStream_t s) {
  AdamArgs a{nullptr, nullptr, nullptr, nullptr, 0, hp, st, partials, nkld, nbce, advance, 0};
  hipLaunchKernelGGL(loss_finalize, dim3(1), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
