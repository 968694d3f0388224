// Single-launch fused Adam over a flat parameter arena (MI355X, gfx950).
//
// Replaces torch's foreach Adam (~8-10 multi-tensor launches per step over 10
// tensors, /root/reference/vae-hpo.py:131,74) with one memory-bound pass:
// per element 4 reads (p, g, m, v) + 3 writes, float4-vectorised. Used when
// the gradients must be all-reduced before the update (intra-group DDP);
// otherwise the MLP-VAE step applies Adam inside its weight-gradient GEMM
// epilogues (vae_mlp.hip, B3). Numerics: adam_common.h (torch.optim.Adam).
//
// Also hosts the eval-path loss reduction (one block).
#include "common.h"
#include "vae_mlp.h"
#include "adam_common.h"

namespace mdt {

struct AdamArgs {
  float* p; const float* g; float* m; float* v;
  long long n4;            // number of float4 groups
  const HParams* hp;
  TrainState* st;
};

__global__ void __launch_bounds__(512) adam_flat(AdamArgs a) {
  __shared__ AdamC cs;
  const AdamC c = adam_consts_block(a.st, a.hp, &cs);
  adam_stream(a.p, a.g, a.m, a.v, 0, a.n4 * 4, blockIdx.x, gridDim.x, c);
}

// loss = sum(BCE partials) + beta * sum(KLD partials) -> loss ring of `st`.
__global__ void __launch_bounds__(256) loss_finalize(const HParams* hp, TrainState* st,
                                                     const float* partials, int nkld, int nbce) {
  __shared__ float scratch[16];
  float sb = 0.f, sk = 0.f;
  for (int i = threadIdx.x; i < nbce; i += blockDim.x) sb += partials[kBcePartial + i];
  for (int i = threadIdx.x; i < nkld; i += blockDim.x) sk += partials[kKldPartial + i];
  const float bce = block_sum(sb, scratch);
  __syncthreads();
  const float kld = block_sum(sk, scratch);
  if (threadIdx.x == 0) {
    const float loss = bce + hp->kl_beta * kld;
    st->loss_hist[(st->step - 1) % kLossHist] = loss;
    st->epoch_loss += (double)loss;
    st->epoch_count += 1.0;
  }
}

}  // namespace mdt

using namespace mdt;

extern "C" int mdt_adam_step(float* p, const float* g, float* m, float* v, long long n,
                             const HParams* hp, TrainState* st, hipStream_t s) {
  if (n % 4) return 1;
  AdamArgs a{p, g, m, v, n / 4, hp, st};
  long long blocks = (a.n4 + 511) / 512;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(adam_flat, dim3((unsigned)blocks), dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

extern "C" int mdt_loss_finalize(const HParams* hp, TrainState* st, const float* partials,
                                 int nkld, int nbce, hipStream_t s) {
  hipLaunchKernelGGL(loss_finalize, dim3(1), dim3(256), 0, s, hp, st, partials, nkld, nbce);
  return (int)hipGetLastError();
}
