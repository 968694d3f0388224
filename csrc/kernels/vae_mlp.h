// Host/device-shared structures of the fused MLP-VAE step (see vae_mlp.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace mdt {

constexpr int kMaxBatch = 4096;
constexpr int kKldPartial = 0;      // F2 blocks write [0, 256)
constexpr int kBcePartial = 256;    // F3 blocks write [256, kPartials)
constexpr int kPartials = 256 + 8192;
constexpr int kLossHist = 4096;     // per-step loss ring (host reads at log points)

// Device-resident training state of one trial (64-byte aligned, memset to 0).
struct TrainState {
  int64_t step;        // optimizer steps taken (Adam t = step + 1; RNG counter)
  int32_t cursor;      // batch index within the epoch's index list
  int32_t nbatches;    // cursor wraps at this value
  uint32_t ticket;     // arrival counter for the optimizer's last-block finalize
  int32_t nparts_kld;  // partial slots written by the last forward (F2 blocks)
  int32_t nparts_bce;  // partial slots written by the last forward (F3 blocks)
  int32_t pad0;
  double epoch_loss;   // running sum of per-batch losses since the host reset it
  double epoch_count;  // batches accumulated in epoch_loss
  float loss_hist[kLossHist];
};

// Per-trial hyper-parameters, device-resident so a captured graph picks up
// lr/beta changes (schedules, HPO perturbation) without re-capture.
struct HParams {
  float lr, beta1, beta2, eps, weight_decay, kl_beta, grad_scale, pad;
  uint32_t seed_lo, seed_hi;
  uint32_t pad2[6];
};

struct VaeArgs {
  int M, B, D, H, Z;
  uint32_t rng_stream;   // distinguishes replicas / eval draws
  int train;             // 1: write backward intermediates
  int pad;
  const float* X;        // dataset [N, D]
  const int* idx;        // epoch index list [nbatches * B] (+ tail)
  const float *W1, *b1, *W2, *b2, *W3, *b3, *W4, *b4;
  float *gW1, *gb1, *gW2, *gb2, *gW3, *gb3, *gW4, *gb4;
  float *h1, *mulv, *eps, *z, *h3, *dlog, *dh3, *dmulv, *dh1;
  float* recon;          // optional sigmoid output [M, D] (eval / images)
  float* partials;       // [kPartials]
  TrainState* st;
  const HParams* hp;
};

struct VaeGrid {
  int f1, f2, f3, b1, b1_dh3, b2, b2_rows, b3, b3_w2;
};

VaeGrid vae_grid(int M, int D, int H, int Z);

}  // namespace mdt

extern "C" {
int mdt_vae_check(const mdt::VaeArgs* a);
int mdt_vae_forward(const mdt::VaeArgs* a, hipStream_t s);
int mdt_vae_backward(const mdt::VaeArgs* a, hipStream_t s, int part);
int mdt_vae_decode(const mdt::VaeArgs* a, const float* zin, hipStream_t s);
}
