// Device bodies of the small conv-VAE step kernels that also run as jobs of
// the horizontally fused launches (conv_igemm.hip, "job kernels").
#pragma once
#include "adam_common.h"
#include "common.h"
#include "conv_igemm.h"
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

// Loss reduction that also ADVANCES the step (the fused 28x28 step,
// conv28_fused.hip): its forward reads `step` as the running step's RNG
// counter, so the increment happens here, after the forward and backward
// launches and before the finalize launch reads beta^t for Adam. Same state
// layout and the same loss ring slot (step - 1 after the increment) as
// loss_finalize_body after a step_begin.
__device__ __forceinline__ void loss_step_body(const LossArgs& la, float* scratch) {
  float sb = 0.f, sk = 0.f;
  for (int i = threadIdx.x; i < la.nb; i += blockDim.x) sb += la.bce_part[i];
  for (int i = threadIdx.x; i < la.nk; i += blockDim.x) sk += la.kld_part[i];
  const float bce = block_sum(sb, scratch);
  __syncthreads();
  const float kld = block_sum(sk, scratch);
  if (threadIdx.x == 0) {
    TrainState* st = la.st;
    st->step = st->step + 1;
    st->b1pow *= la.hp->beta1_d;
    st->b2pow *= la.hp->beta2_d;
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

// Split-K combines fused with the reparameterisation (forward) and its
// backward. A block owns cnt = 256/rp consecutive latent elements e = i*Z + c;
// rp threads per element sum the interleaved k-slices z = r, r+rp, ... (loads
// in flight in parallel), and the element's lane adds the rp partials in order
// (deterministic, same tree as splitk_combine_body).
__host__ __device__ inline int splitk_rp(int ks) {
  int rp = 1;
  while (rp < 64 && rp * 4 < ks) rp *= 2;
  return rp;
}
// Row form (the default where it applies: Z a power of two in [8, 512]): one
// block per sample row. Its 2Z (forward) / Z (backward) slab columns are read
// as float4s by Z/2 (Z/4) lanes per k-slice row -- every wave-instruction
// covers whole 256-B+ row pieces -- with 256/lanes k-slices in flight, then a
// fixed-order LDS combine. The element-strided form above reads 16 B of each
// 64-B segment per wave-instruction (4x the slab bytes fetched: 16.6 MB for a
// 4 MB slab at the 128x128 decoder Linear) and stays for other Z.
__host__ __device__ inline bool combine_rows_ok(int Z) { return Z >= 8 && Z <= 512 && (Z & (Z - 1)) == 0; }
__host__ __device__ inline int combine_reparam_blocks(int ks, int B, int Z) {
  if (combine_rows_ok(Z)) return B;
  const int cnt = 256 / splitk_rp(ks);
  return (B * Z + cnt - 1) / cnt;
}

// sum_z slab[z][row0 + 4q .. +3] over k-slices z = rg, rg + RG, ... (RG =
// 256 / LW row groups of LW float4 lanes) -> red[rg][4q .. 4q+3]; `W` = row
// width in floats (4 LW), `MN` = slab row pitch in floats.
__device__ __forceinline__ void combine_rows_partial(const float* slab, int ks, long long MN, long long row0, int W,
                                                     float* red) {
  const int LW = W >> 2, RG = 256 / LW;
  const int t = threadIdx.x, q = t % LW, rg = t / LW;
  float4 s = {0.f, 0.f, 0.f, 0.f};
  const float4* p = reinterpret_cast<const float4*>(slab + row0) + q;
  const long long pitch4 = MN >> 2;
  auto add = [&](const float4& v) {
    s.x += v.x;
    s.y += v.y;
    s.z += v.z;
    s.w += v.w;
  };
  // 16 loads in flight per lane (64 KB per workgroup): the slab was written by
  // the previous launch, so every load is a fabric round trip
  int z = rg;
  for (; z + 15 * RG < ks; z += 16 * RG) {
    float4 v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = p[(long long)(z + u * RG) * pitch4];
#pragma unroll
    for (int u = 0; u < 16; ++u) add(v[u]);
  }
  for (; z < ks; z += RG) add(p[(long long)z * pitch4]);
  reinterpret_cast<float4*>(red)[rg * LW + q] = s;
}

// Encoder head: mulv = sum_z slab[z] + bias (f32 [B][2Z]); eps ~ N(0,1)
// (Philox, keyed like the MLP kernels); z = mu + eps * exp(lv/2) -> bf16
// (+f32); one KLD partial per block (combine_reparam_blocks of them).
struct CombineReparamArgs {
  const float* slab;
  int ks, rp;
  const float* bias;
  float* mulv;
  float* eps;
  __bf16* z16;
  float* z32;
  int B, Z;
  const TrainState* st;
  const HParams* hp;
  uint32_t stream;
  float* kld_part;
};

// `red` >= 1024 + 16 floats (16-B aligned)
__device__ __forceinline__ void combine_reparam_rows_body(const CombineReparamArgs& a, float* red, int i) {
  const int Z = a.Z, W = 2 * Z, RG = 1024 / W, t = threadIdx.x;
  const bool own = t < Z;
  // the step, seeds and bias before the slab sum: loaded after it they were a
  // second dependent round trip at the kernel's end
  const long long stp = a.st->step - 1;
  const uint32_t seed_lo = a.hp->seed_lo, seed_hi = a.hp->seed_hi;
  float bm = 0.f, bl = 0.f;
  if (own && a.bias) {
    bm = a.bias[t];
    bl = a.bias[Z + t];
  }
  combine_rows_partial(a.slab, a.ks, (long long)a.B * W, (long long)i * W, W, red);
  __syncthreads();
  float kl = 0.f, mu = 0.f, lv = 0.f, ep = 0.f, zz = 0.f;
  if (own) {
    const int c = t;
    for (int r = 0; r < RG; ++r) {
      mu += red[r * W + c];
      lv += red[r * W + Z + c];
    }
    if (a.bias) {
      mu += bm;
      lv += bl;
    }
    const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(i * Z + c), a.stream, (uint32_t)((unsigned long long)stp & 0xffffffffu),
                                           (uint32_t)((unsigned long long)stp >> 32)},
                                     seed_lo, seed_hi);
    ep = normal_from_bits(bits.x, bits.y);
    const float sd = expf(0.5f * lv);
    zz = mu + ep * sd;
    kl = 1.f + lv - mu * mu - sd * sd;
  }
  // the KLD block sum before the stores (see below)
  const float s = block_sum(kl, red + 1024);
  if (own) {
    const int c = t, e = i * Z + c;
    a.mulv[(size_t)i * W + c] = mu;
    a.mulv[(size_t)i * W + Z + c] = lv;
    a.eps[e] = ep;
    a.z16[e] = (__bf16)zz;
    if (a.z32) a.z32[e] = zz;
  }
  if (t == 0) a.kld_part[i] = -0.5f * s;
}

// `red` >= 2*256 + 16 floats
__device__ __forceinline__ void combine_reparam_body(const CombineReparamArgs& a, float* red, int bid) {
  const int t = threadIdx.x, cnt = 256 / a.rp, col = t % cnt, rl = t / cnt;
  const int e = bid * cnt + col;
  const bool live = e < a.B * a.Z;
  const int i = live ? e / a.Z : 0, c = live ? e - i * a.Z : 0;
  const long long MN = (long long)a.B * 2 * a.Z;
  const long long em = (long long)i * 2 * a.Z + c, el = em + a.Z;
  float vm = 0.f, vl = 0.f;
  if (live) {
    for (int z = rl; z < a.ks; z += a.rp) {
      vm += a.slab[(size_t)z * MN + em];
      vl += a.slab[(size_t)z * MN + el];
    }
  }
  red[t] = vm;
  red[256 + t] = vl;
  __syncthreads();
  float kl = 0.f, mu = 0.f, lv = 0.f, ep = 0.f, zz = 0.f;
  if (rl == 0 && live) {
    for (int r = 0; r < a.rp; ++r) {
      mu += red[r * cnt + col];
      lv += red[256 + r * cnt + col];
    }
    if (a.bias) {
      mu += a.bias[c];
      lv += a.bias[a.Z + c];
    }
    const long long stp = a.st->step - 1;
    const u32x4 bits = philox4x32_10(u32x4{(uint32_t)(i * a.Z + c), a.stream, (uint32_t)((unsigned long long)stp & 0xffffffffu),
                                           (uint32_t)((unsigned long long)stp >> 32)},
                                     a.hp->seed_lo, a.hp->seed_hi);
    ep = normal_from_bits(bits.x, bits.y);
    const float sd = expf(0.5f * lv);
    zz = mu + ep * sd;
    kl = 1.f + lv - mu * mu - sd * sd;
  }
  // the KLD block sum before the stores: its barriers would otherwise wait
  // for their acknowledgements (vmcnt counts stores on CDNA)
  const float s = block_sum(kl, red + 512);
  if (rl == 0 && live) {
    a.mulv[em] = mu;
    a.mulv[el] = lv;
    a.eps[e] = ep;
    a.z16[e] = (__bf16)zz;
    if (a.z32) a.z32[e] = zz;
  }
  if (threadIdx.x == 0) a.kld_part[bid] = -0.5f * s;
}

// Decoder Linear backward-data: dz = sum_z slab[z] -> d[mu|lv] (+bf16 copy).
struct CombineReparamBwdArgs {
  const float* slab;
  int ks, rp;
  const float* mulv;
  const float* eps;
  float* dmulv;
  __bf16* dmulv16;
  float* dz;
  int B, Z;
  const HParams* hp;
};

// `red` >= 1024 floats (16-B aligned)
__device__ __forceinline__ void combine_reparam_bwd_rows_body(const CombineReparamBwdArgs& a, float* red, int i) {
  const int Z = a.Z, RG = 1024 / Z, t = threadIdx.x;
  // this lane's mu / logvar / eps and beta before the slab sum (one round trip
  // fewer at the kernel's end)
  const int c = t < Z ? t : 0, e = i * Z + c;
  const float beta = a.hp->kl_beta;
  const float mu = a.mulv[(size_t)i * 2 * Z + c], lv = a.mulv[(size_t)i * 2 * Z + Z + c], ee = a.eps[e];
  combine_rows_partial(a.slab, a.ks, (long long)a.B * Z, (long long)i * Z, Z, red);
  __syncthreads();
  if (t >= Z) return;
  float g = 0.f;
  for (int r = 0; r < RG; ++r) g += red[r * Z + c];
  if (a.dz) a.dz[e] = g;
  const float sd = expf(0.5f * lv);
  const float dm = g + beta * mu;
  const float dl = 0.5f * g * ee * sd + 0.5f * beta * (sd * sd - 1.f);
  a.dmulv[(size_t)i * 2 * Z + c] = dm;
  a.dmulv[(size_t)i * 2 * Z + Z + c] = dl;
  if (a.dmulv16) {
    a.dmulv16[(size_t)i * 2 * Z + c] = (__bf16)dm;
    a.dmulv16[(size_t)i * 2 * Z + Z + c] = (__bf16)dl;
  }
}

// `red` >= 256 floats
__device__ __forceinline__ void combine_reparam_bwd_body(const CombineReparamBwdArgs& a, float* red, int bid) {
  const int t = threadIdx.x, cnt = 256 / a.rp, col = t % cnt, rl = t / cnt;
  const int e = bid * cnt + col;
  const bool live = e < a.B * a.Z;
  const long long MN = (long long)a.B * a.Z;
  float v = 0.f;
  if (live)
    for (int z = rl; z < a.ks; z += a.rp) v += a.slab[(size_t)z * MN + e];
  red[t] = v;
  __syncthreads();
  if (rl != 0 || !live) return;
  float g = 0.f;
  for (int r = 0; r < a.rp; ++r) g += red[r * cnt + col];
  const int i = e / a.Z, c = e - i * a.Z;
  if (a.dz) a.dz[e] = g;
  const float beta = a.hp->kl_beta;
  const float mu = a.mulv[(size_t)i * 2 * a.Z + c], lv = a.mulv[(size_t)i * 2 * a.Z + a.Z + c];
  const float sd = expf(0.5f * lv);
  const float dm = g + beta * mu;
  const float dl = 0.5f * g * a.eps[e] * sd + 0.5f * beta * (sd * sd - 1.f);
  a.dmulv[(size_t)i * 2 * a.Z + c] = dm;
  a.dmulv[(size_t)i * 2 * a.Z + a.Z + c] = dl;
  if (a.dmulv16) {
    a.dmulv16[(size_t)i * 2 * a.Z + c] = (__bf16)dm;
    a.dmulv16[(size_t)i * 2 * a.Z + a.Z + c] = (__bf16)dl;
  }
}

// Gradient finalisation (256-thread blocks). One unit = `count` consecutive
// elements of one segment. Threads t = rl*count + col sum partial rows rl,
// rl+rp, ... (rp = 256/count) of column col, then row lane 0 adds the rp sums
// in order: a fixed reduction tree, so results are bitwise reproducible
// (unlike f32 atomics). With do_adam the same thread applies Adam to the
// parameter and re-emits its bf16 copy.
struct FinalizeArgs {
  float *P, *G, *Mo, *Vo;
  __bf16* w16;
  const GradSeg* segs;
  const GradUnit* units;
  const TrainState* st;
  const HParams* hp;
  int do_adam;
  // 1: the slabs and the step state were written IN THIS LAUNCH by other
  // workgroups (a dependent jobs_multi_k launch, conv_jobs.hip JobDeps): every
  // load of them is an sc1 vector load (past this CU's L1, never the scalar
  // cache), behind the counter poll that published them
  int dep;
};

constexpr int kFinalizeThreads = 256;

// Next-batch gather riding in the 28x28 step's finalize launch (blocks ahead
// of the finalize units): by then the loss job has advanced the cursor and the
// step, so rows idx[cursor * B + n] are the NEXT step's batch; they go to xn
// with xtag[n] = step, which the step kernel's P0 checks before taking its
// row from xn in one round trip (conv28_fused.h fwd_p01). Same launch, so
// the kernel boundary publishes both to the next step.
struct BatchGather {
  const float* X;      // dataset [rows][784]
  const int* idx;      // epoch index list (whole batches of B)
  const TrainState* st;
  float* xn;           // [B][784], null = off
  unsigned* xtag;      // [B]
  int B, nunits;       // blocks [0, gather_blocks(B)) gather, the finalize units follow
};
__host__ __device__ constexpr int gather_blocks(int B) { return (B * 196 + kFinalizeThreads - 1) / kFinalizeThreads; }

__device__ __forceinline__ void batch_gather_body(const BatchGather& g, int b) {
  const int e = b * kFinalizeThreads + (int)threadIdx.x;  // float4 index over [B][196]
  const int n = e / 196, c = e - 196 * (e / 196);
  if (n < g.B) {
    const int row = g.idx[(size_t)g.st->cursor * g.B + n];
    reinterpret_cast<float4*>(g.xn + (size_t)n * 784)[c] = reinterpret_cast<const float4*>(g.X + (size_t)row * 784)[c];
    if (c == 0) g.xtag[n] = (unsigned)g.st->step;
  }
}

// The same gather as a job of a dependent jobs_multi_k launch (kJobGather),
// after the loss job advanced cursor and step in that launch: both are read
// with sc1 vector loads behind the poll of the loss job's counter.
__device__ __forceinline__ void batch_gather_dep_body(const BatchGather& g, int b) {
  const int e = b * kFinalizeThreads + (int)threadIdx.x;
  const int n = e / 196, c = e - 196 * (e / 196);
  if (n < g.B) {
    using gi32 = __attribute__((address_space(1))) int;  // global, never flat
    using gu64 = __attribute__((address_space(1))) unsigned long long;
    TrainState* st = const_cast<TrainState*>(g.st);
    const int cur = __hip_atomic_load((gi32*)&st->cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int row = g.idx[(size_t)cur * g.B + n];
    reinterpret_cast<float4*>(g.xn + (size_t)n * 784)[c] = reinterpret_cast<const float4*>(g.X + (size_t)row * 784)[c];
    if (c == 0)
      g.xtag[n] = (unsigned)__hip_atomic_load((gu64*)&st->step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Partial-slab sums shared by the finalize bodies here and the fused
// all-reduce jobs (comm_jobs.h): one summation order everywhere, so a
// gradient finalized on its own and one finalized inside a collective job
// carry the same bits. `ld(i)` loads element (or 4 elements at) index i of
// the slab: plain loads (SlabPlain) or, for slabs written earlier in the same
// launch, sc1 buffer loads (SlabSc1).
struct SlabPlain {
  const float* p;
  __device__ __forceinline__ f32x4 v4(long long i) const { return *reinterpret_cast<const f32x4*>(p + i); }
  __device__ __forceinline__ float v1(long long i) const { return p[i]; }
};
struct SlabSc1 {
  __amdgpu_buffer_rsrc_t rs;  // whole slab (uniform base), byte offsets < 4 GB
  __device__ __forceinline__ SlabSc1(const float* slab, long long elems)
      : rs(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(slab), 0, (int)(elems * 4), 0x00020000)) {}
  __device__ __forceinline__ f32x4 v4(long long i) const {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 4), 0, 16 /* sc1 */));
  }
  __device__ __forceinline__ float v1(long long i) const {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(i * 4), 0, 16 /* sc1 */));
  }
};
// 4 consecutive elements at e (vec4 units): 4 interleaved accumulators over the slabs
template <class L>
__device__ __forceinline__ f32x4 slab_sum4_l(const L& ld, long long e, long long n, int nsplit) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 a0 = z, a1 = z, a2 = z, a3 = z;
  int s = 0;
  for (; s + 3 < nsplit; s += 4) {
    a0 += ld.v4(e + (long long)s * n);
    a1 += ld.v4(e + (long long)(s + 1) * n);
    a2 += ld.v4(e + (long long)(s + 2) * n);
    a3 += ld.v4(e + (long long)(s + 3) * n);
  }
  for (; s < nsplit; ++s) a0 += ld.v4(e + (long long)s * n);
  return z + ((a0 + a1) + (a2 + a3));
}
// one element (tail of a vec4 unit), same order as one lane of slab_sum4
template <class L>
__device__ __forceinline__ float slab_sum1_l(const L& ld, long long e, long long n, int nsplit) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 3 < nsplit; s += 4) {
    a0 += ld.v1(e + (long long)s * n);
    a1 += ld.v1(e + (long long)(s + 1) * n);
    a2 += ld.v1(e + (long long)(s + 2) * n);
    a3 += ld.v1(e + (long long)(s + 3) * n);
  }
  for (; s < nsplit; ++s) a0 += ld.v1(e + (long long)s * n);
  return 0.f + ((a0 + a1) + (a2 + a3));
}
// scalar units: slabs rl, rl + rp, ... of column e (row lane rl of rp)
template <class L>
__device__ __forceinline__ float slab_partial_l(const L& ld, long long e, long long n, int nsplit, int rl, int rp) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = rl;
  for (; s + 3 * rp < nsplit; s += 4 * rp) {
    a0 += ld.v1(e + (long long)s * n);
    a1 += ld.v1(e + (long long)(s + rp) * n);
    a2 += ld.v1(e + (long long)(s + 2 * rp) * n);
    a3 += ld.v1(e + (long long)(s + 3 * rp) * n);
  }
  for (; s < nsplit; s += rp) a0 += ld.v1(e + (long long)s * n);
  return (a0 + a1) + (a2 + a3);
}
__device__ __forceinline__ f32x4 slab_sum4(const float* p, long long n, int nsplit) {
  return slab_sum4_l(SlabPlain{p}, 0, n, nsplit);
}
__device__ __forceinline__ float slab_sum1(const float* p, long long n, int nsplit) {
  return slab_sum1_l(SlabPlain{p}, 0, n, nsplit);
}
__device__ __forceinline__ float slab_partial(const float* p, long long n, int nsplit, int rl, int rp) {
  return slab_partial_l(SlabPlain{p}, 0, n, nsplit, rl, rp);
}

// Units of more than 256 elements (planned when a segment has <= 16 partial
// slabs and 16-B aligned rows): each thread finalizes 4 consecutive elements
// with 16-B loads/stores -- same per-element summation order as the scalar
// path (4 interleaved accumulators over the slabs), so results are unchanged.
// The optimizer tail streams P, m, v (+ slabs) once: 16-B accesses keep
// 4x the bytes in flight per wave-instruction of the 4-B path.
template <bool DEP>
__device__ __forceinline__ void grad_finalize_vec4(const FinalizeArgs& a, const AdamC& c, const GradUnit& u,
                                                   const GradSeg& sg) {
  const int e0 = u.start + 4 * (int)threadIdx.x;
  const int left = u.start + u.count - e0;
  if (left <= 0) return;
  const long long o = sg.off + e0;
  const long long n = sg.numel;
  if (left >= 4) {
    f32x4 g;
    if (sg.slab) {
      if constexpr (DEP) g = slab_sum4_l(SlabSc1(sg.slab, n * sg.nsplit), e0, n, sg.nsplit);
      else g = slab_sum4(sg.slab + e0, n, sg.nsplit);
      if (!a.do_adam) *reinterpret_cast<f32x4*>(a.G + o) = g;
    } else {
      g = *reinterpret_cast<const f32x4*>(a.G + o);
    }
    if (a.do_adam) {
      f32x4 p = *reinterpret_cast<const f32x4*>(a.P + o);
      f32x4 m = *reinterpret_cast<const f32x4*>(a.Mo + o);
      f32x4 v = *reinterpret_cast<const f32x4*>(a.Vo + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_update(pj, mj, vj, g[j], c);
        p[j] = pj; m[j] = mj; v[j] = vj;
      }
      *reinterpret_cast<f32x4*>(a.P + o) = p;
      *reinterpret_cast<f32x4*>(a.Mo + o) = m;
      *reinterpret_cast<f32x4*>(a.Vo + o) = v;
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 w;
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = (__bf16)p[j];
      *reinterpret_cast<bf16x4*>(a.w16 + o) = w;
    }
    return;
  }
  for (int j = 0; j < left; ++j) {  // segment tail (< 4 elements)
    float g;
    if (sg.slab) {
      if constexpr (DEP) g = slab_sum1_l(SlabSc1(sg.slab, n * sg.nsplit), e0 + j, n, sg.nsplit);
      else g = slab_sum1(sg.slab + e0 + j, n, sg.nsplit);
      if (!a.do_adam) a.G[o + j] = g;
    } else {
      g = a.G[o + j];
    }
    if (a.do_adam) {
      float p = a.P[o + j], m = a.Mo[o + j], v = a.Vo[o + j];
      adam_update(p, m, v, g, c);
      a.P[o + j] = p; a.Mo[o + j] = m; a.Vo[o + j] = v;
      a.w16[o + j] = (__bf16)p;
    }
  }
}

template <bool DEP>
__device__ __forceinline__ void grad_finalize_body_t(const FinalizeArgs& a, float* red, AdamC* cs, int bid) {
  AdamC c{};
  if (a.do_adam) c = DEP ? adam_consts_block_sc1(a.st, a.hp, cs) : adam_consts_block(a.st, a.hp, cs);
  const GradUnit u = a.units[bid];
  const GradSeg sg = a.segs[u.seg];
  if (u.count > kFinalizeThreads) {
    grad_finalize_vec4<DEP>(a, c, u, sg);
    return;
  }
  const int t = threadIdx.x, cnt = u.count, rp = kFinalizeThreads / cnt;
  const int col = t % cnt, rl = t / cnt;
  float part = 0.f;
  if (sg.slab && rl < rp) {
    if constexpr (DEP)
      part = slab_partial_l(SlabSc1(sg.slab, sg.numel * sg.nsplit), u.start + col, sg.numel, sg.nsplit, rl, rp);
    else
      part = slab_partial(sg.slab + u.start + col, sg.numel, sg.nsplit, rl, rp);
  }
  red[t] = part;
  __syncthreads();
  if (rl == 0) {
    const long long o = sg.off + u.start + col;
    float g;
    if (sg.slab) {
      g = 0.f;
      for (int r = 0; r < rp; ++r) g += red[r * cnt + col];
      if (!a.do_adam) a.G[o] = g;  // the fused-Adam path consumes g in registers only
    } else {
      g = a.G[o];
    }
    if (a.do_adam) {
      float p = a.P[o], m = a.Mo[o], v = a.Vo[o];
      adam_update(p, m, v, g, c);
      a.P[o] = p; a.Mo[o] = m; a.Vo[o] = v;
      a.w16[o] = (__bf16)p;
    }
  }
}
// stand-alone finalize launch and the 3-job combos: nothing in the launch
// writes the slabs or the step state (FinalizeArgs.dep is 0 there)
__device__ __forceinline__ void grad_finalize_body(const FinalizeArgs& a, float* red, AdamC* cs, int bid) {
  grad_finalize_body_t<false>(a, red, cs, bid);
}

// bf16 weights [CO][k][k][CI] -> parity-ordered transpose [s][s][CI][k/s][k/s][CO]
// (class (a, b) holds taps ky = a + s*ty, kx = b + s*tx) for the kModeTconv
// GEMM. One 64x64 (co, ci) tile of one tap per block, staged through LDS so
// both the read (ci-contiguous) and the write (co-contiguous) are coalesced.
struct WtransArgs {
  const __bf16* w16;
  __bf16* w16t;
  const GradSeg* segs;
  const TrUnit* units;
};

constexpr int kWtransPitch = 72;                 // 16-B form: row pitch in bf16 (16-B aligned rows)
constexpr int kWtransLds = 64 * kWtransPitch * 2;  // >= the scalar form's 64 x 66

__device__ __forceinline__ void wtrans_body(const WtransArgs& wa, uint8_t* lds, int bid) {
  const TrUnit u = wa.units[bid];
  const GradSeg sg = wa.segs[u.seg];
  const int k = sg.k, s = sg.s, CI = sg.ci, CO = sg.co, T = k / s;
  const int ky = u.tap / k, kx = u.tap - ky * k;
  const int a = ky % s, ty = ky / s, b = kx % s, tx = kx / s;
  const unsigned short* src = reinterpret_cast<const unsigned short*>(wa.w16) + sg.off;
  unsigned short* dst = reinterpret_cast<unsigned short*>(wa.w16t) + sg.toff;
  if (CI % 8 == 0 && CO % 8 == 0 && sg.off % 8 == 0 && sg.toff % 8 == 0) {
    // 16-B form: 8 channels per global access on both sides (the 2-B form
    // below issued 32 global instructions per thread; 13.4 us for the
    // 128x128 model's 3 M weights, profiles/r4_pmc_conv128). Chunk q of tile
    // row r sits at slot q ^ (r >> 3), so the column reads of the transposed
    // side spread over 8 bank groups.
    typedef unsigned short us8 __attribute__((ext_vector_type(8)));
    unsigned short (*tile)[kWtransPitch] = reinterpret_cast<unsigned short (*)[kWtransPitch]>(lds);
    for (int ch = threadIdx.x; ch < 64 * 8; ch += blockDim.x) {
      const int r = ch >> 3, q = ch & 7;  // tile row = co, chunk = 8 ci
      const int co = u.co0 + r, ci = u.ci0 + 8 * q;
      if (co < CO && ci < CI)
        *reinterpret_cast<us8*>(&tile[r][8 * (q ^ (r >> 3))]) =
            *reinterpret_cast<const us8*>(src + ((long long)(co * k + ky) * k + kx) * CI + ci);
    }
    __syncthreads();
    for (int ch = threadIdx.x; ch < 64 * 8; ch += blockDim.x) {
      const int r = ch >> 3, q = ch & 7;  // output row = ci, chunk = 8 co
      const int ci = u.ci0 + r, co = u.co0 + 8 * q;
      if (co < CO && ci < CI) {
        us8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = tile[8 * q + j][8 * ((r >> 3) ^ q) + (r & 7)];
        *reinterpret_cast<us8*>(dst + ((((long long)(a * s + b) * CI + ci) * T + ty) * T + tx) * CO + co) = v;
      }
    }
    return;
  }
  unsigned short (*tile)[66] = reinterpret_cast<unsigned short (*)[66]>(lds);
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
