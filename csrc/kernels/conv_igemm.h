// Shared host/device definitions of the conv-VAE implicit-GEMM kernels
// (csrc/kernels/conv_igemm.hip) and their C++ bindings (csrc/runtime/conv_ops.cpp).
// Plain structs only: included by hipcc and g++ alike.
#pragma once
#include <stdint.h>

namespace mdt {

// Convolution geometry, always in "conv view": input (N,H,W,C) NHWC,
// output (N,OH,OW,CO), weight [CO][KH][KW][C]. A transposed conv is the
// conv whose backward-data is its forward (input = convT output).
struct ConvDesc {
  int N, H, W, C;
  int OH, OW, CO;
  int KH, KW, S, P;
};

// Unsigned division by a runtime constant with one mul-hi + add + shift
// (valid for numerators < 2^31): replaces the ~40-instruction integer divide
// in the per-chunk im2col address math.
struct FastDiv {
  uint32_t d, mul, shr;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  f.shr = 0;
  while ((1u << f.shr) < d) ++f.shr;
  const uint64_t one = 1;
  f.mul = (uint32_t)(((one << 32) * ((one << f.shr) - d)) / d + 1);
  return f;
}

// Row-space GEMM kinds of the forward-type kernel.
enum IgemmMode : int {
  kModeConv = 0,   // rows = conv output pixels, k = (ky, kx, ci): conv fwd / convT bwd-data
  kModeTconv = 1,  // rows = conv INPUT pixels of one stride-parity class, k = (ty, tx, co):
                   // conv bwd-data / convT fwd, without the zero-insertion taps
};

// Launch plan of one forward-type GEMM (computed on the host, deterministic
// in the geometry so the trainer can size the partial-sum buffers up front).
struct FwdPlan {
  int cfg;          // tile configuration index (see conv_igemm.hip)
  int BM, BN;
  int classes;      // 1, or S*S parity classes (kModeTconv)
  int M;            // GEMM rows per class
  int Ncols, K;     // GEMM columns / depth (per class)
  int mtiles, ntiles, ktiles;
  int ksplit, kt_per_split;
  int colsum_rows;  // rows of the per-block column-sum partials (classes * mtiles)
  int thin;         // 1: per-element im2col gather (channel count not a multiple of 8)
  int direct;       // > 0: patch-resident direct kernel configuration + 1 (conv_direct.h)
};

// Weight-gradient GEMM plan: dW[CO][KH*KW*C] = sum_m G[m][co] * im2col(X)[m][k'].
struct WgradPlan {
  int cfg;
  int BM, BN;       // co tile x k' tile
  int M, K2;
  int cotiles, ktiles, mtiles;  // m-tiles of 64
  int nsplit, mt_per_split;
  int thin;
};

// Gradient finalisation: per arena segment, g = sum over `nsplit` partial rows
// of width `numel` (deterministic order), then either stored to the gradient
// arena or consumed by a fused Adam + bf16 cast (+ parity-ordered transpose).
// Optional A-operand prologue: the producing layer ran split-K without a
// combine pass; A(row, k) = act(bias[c] + sum_s slab[s][off]) is formed while
// staging (c = off % cin) and written once to `out16` (the producer's output,
// needed later by the backward), saving the combine launch in between.
struct APro {
  const float* slab;  // [ks][A elements] partial sums of the producer (null: plain A)
  const float* bias;
  void* out16;        // bf16
  int ks, relu, cin;
  long long stride;   // elements per slab
};

struct GradSeg {
  long long off, numel;
  const float* slab;  // nullptr: the gradient arena already holds g
  int nsplit;
  int co, k, s, ci;   // weight geometry of the transposed copy ([CO][k][k][ci])
  long long toff;     // offset of the transposed copy in w16t, -1 if none
};

struct GradUnit {
  int seg, start, count;
};

// One 64(co) x 64(ci) tile of one tap of a weight segment for the transpose
// into the parity-ordered copy.
struct TrUnit {
  int seg, tap, co0, ci0;
};

// One job of a horizontally fused launch (conv_jobs.hip): an independent
// piece of work (a GEMM, a weight gradient, a column sum, ...) that runs on
// its own range of workgroups of a shared launch. `args` holds the job's
// kernel-argument struct; `kind` names the device body that interprets it.
constexpr int kJobArgBytes = 256;
struct JobBlob {
  int kind;       // 0 = none / not fusable
  int nblk;       // workgroups of this job (256 threads each)
  int aux[6];     // per-kind geometry (e.g. GEMM tiles per plane, k-splits)
  alignas(16) unsigned char args[kJobArgBytes];
};

// Job kind ids (see conv_jobs.hip for the instantiated combinations).
enum JobKindBase : int {
  kJobIgemm = 1000,      // + mode*100 + cfg  (bf16, vector gathers)
  kJobWgrad = 2000,      // + cfg              (bf16, vector gathers)
  kJobWgradThin = 2050,  // + 20*f32 + cfg     (per-element gathers)
  kJobThinWgM = 2100,    // + f32               (MFMA single-channel weight gradient, conv_thin_wg.h)
  kJobThinConv = 3000,   // + CO + 100*f32
  kJobThinTconv = 4000,  // + CO
  kJobColsum = 5000,
  kJobLoss = 5001,
  kJobCombine = 5002,
  kJobFinalize = 5003,
  kJobWtrans = 5004,
  kJobLossStep = 5005,   // loss reduction + step advance (fused 28x28 step)
  kJobComm = 5006,       // fused xGMI all-reduce + Adam over finalize units (comm_jobs.h)
  kJobGather = 5007,     // next-batch row gather behind the loss job (dependent multi-job launch)
  kJobDconv = 6000,      // + direct cfg       (patch-resident direct conv, conv_direct.h)
};

// Up to kMaxMultiJobs jobs of any kind of the multi-job kernel (jobs_multi_k).
constexpr int kMaxMultiJobs = 16;

}  // namespace mdt
