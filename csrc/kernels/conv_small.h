// Device bodies of the small conv-VAE step kernels that also run as jobs of
// the horizontally fused launches (conv_igemm.hip, "job kernels").
#pragma once
#include "common.h"
#include "vae_mlp.h"

namespace mdt {

struct LossArgs {
  const float* bce_part;
  int nb;
  const float* kld_part;
  int nk;
  TrainState* st;
  const HParams* hp;
  int advance_cursor;
};

// One block: sum the loss partials -> loss ring, epoch sums; optionally
// advance the batch cursor. `scratch` >= 16 floats.
__device__ __forceinline__ void loss_finalize_body(const LossArgs& la, float* scratch) {
  float sb = 0.f, sk = 0.f;
  for (int i = threadIdx.x; i < la.nb; i += blockDim.x) sb += la.bce_part[i];
  for (int i = threadIdx.x; i < la.nk; i += blockDim.x) sk += la.kld_part[i];
  const float bce = block_sum(sb, scratch);
  __syncthreads();
  const float kld = block_sum(sk, scratch);
  if (threadIdx.x == 0) {
    TrainState* st = la.st;
    const float loss = bce + la.hp->kl_beta * kld;
    st->loss_hist[(st->step - 1) % kLossHist] = loss;
    st->epoch_loss += (double)loss;
    st->epoch_count += 1.0;
    if (la.advance_cursor) {
      int c = st->cursor + 1;
      if (st->nbatches > 0 && c >= st->nbatches) c = 0;
      st->cursor = c;
    }
  }
}

}  // namespace mdt
