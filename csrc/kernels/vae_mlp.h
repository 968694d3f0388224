// Host/device-shared structures of the fused MLP-VAE step (see vae_mlp.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace mdt {

constexpr int kMaxBatch = 4096;
constexpr int kKldPartial = 0;      // F2 waves write [0, 2048)  (8 per block)
constexpr int kBcePartial = 2048;   // F3 waves write [2048, kPartials) (8 per block)
constexpr int kPartials = 2048 + 65536;
constexpr int kLossHist = 4096;     // per-step loss ring (host reads at log points)

// Device-resident training state of one trial (memset to 0 at creation).
//
// Advance protocol (no atomics, no extra launch): within one step
//   F1 block 0 increments `step`   (F1 never reads step),
//   F2 block 0 advances `cursor`   (F2 never reads cursor; F1 already copied
//                                    the batch rows into the xb buffer that
//                                    F3/B3 read).
// So `step` counts steps started: the RNG counter of the running step is
// step-1 and Adam's 1-based t is step.
struct TrainState {
  int64_t step;
  int32_t cursor;      // batch index within the epoch's index list
  int32_t nbatches;    // cursor wraps at this value
  double b1pow, b2pow; // beta1^step, beta2^step (Adam bias corrections; F1 advances them)
  double epoch_loss;   // running sum of per-batch losses since the host reset it
  double epoch_count;  // batches accumulated in epoch_loss
  float loss_hist[kLossHist];
};

// Per-trial hyper-parameters, device-resident so a captured graph picks up
// lr/beta changes (schedules, HPO perturbation) without re-capture.
struct HParams {
  float lr, beta1, beta2, eps, weight_decay, kl_beta, grad_scale;
  int32_t decoupled_wd;
  uint32_t seed_lo, seed_hi;
  double lr_d, beta1_d, beta2_d;  // double copies: torch computes lr/bc1 in double
};

struct VaeArgs {
  int M, B, D, H, Z;
  uint32_t rng_stream;   // distinguishes replicas / eval draws
  int train;             // 1: write backward intermediates
  int fuse_adam;         // 1: B3 applies Adam in its epilogues (+ streams the rest)
  const float* X;        // dataset [N, D]
  const int* idx;        // epoch index list [nbatches * B] (+ tail)
  const float *W1, *b1, *W2, *b2, *W3, *b3, *W4, *b4;
  float *gW1, *gb1, *gW2, *gb2, *gW3, *gb3, *gW4, *gb4;
  float *h1, *mulv, *eps, *z, *h3, *dlog, *dh3, *dmulv, *dh1, *xb;
  // split-K partial slabs handed from F1 -> F2 ([mu|lv] over 16-wide h1 slices)
  // and B1 -> B2 (dz over 16-wide dh3 slices): [row tile][H/16][16][width]
  float *slab_mv, *slab_dz;
  float* recon;          // optional sigmoid output [M, D] (eval / images)
  float* partials;       // [kPartials]
  TrainState* st;
  const HParams* hp;
  // optimizer arenas (fused Adam): param / grad / exp_avg / exp_avg_sq base
  float *P, *G, *Mo, *Vo;
  long long oW1, ob1, oW2, ob2;   // arena offsets of the epilogue-updated tensors
  long long s_beg, s_end;         // arena range Adam-streamed by B3 (fc3, fc4)
  unsigned long long* stamps;     // optional phase timestamps (profiling builds of a run)
};

// stamps[((kernel*kStampBlocks + block)*8 + wave)*8 + slot] = s_memrealtime (100 MHz)
constexpr int kStampBlocks = 512;
constexpr int kStampKernels = 6;

struct VaeGrid {
  int f1, f2, f3, b1, b1_dh3, b2, b2_rows, b3, b3_w2, b3_w1, b3_stream;
  int th, ntm, sw, ntz, swz, groups;  // slab geometry (see vae_mlp.hip)
};

VaeGrid vae_grid(const VaeArgs& a);

}  // namespace mdt

extern "C" {
int mdt_vae_check(const mdt::VaeArgs* a);
int mdt_vae_forward(const mdt::VaeArgs* a, hipStream_t s);
int mdt_vae_backward(const mdt::VaeArgs* a, hipStream_t s, int part);
int mdt_vae_decode(const mdt::VaeArgs* a, const float* zin, hipStream_t s);
}
