// torch.optim.Adam arithmetic, shared by the streaming Adam kernel (adam.hip)
// and the weight-gradient epilogues that apply Adam in place (vae_mlp.hip).
#pragma once
#include "common.h"
#include "vae_mlp.h"

namespace mdt {

struct AdamC {
  float step_size, bc2s, b1, b2, eps, wd, gs, lr;
  int decoupled;
};

// Compute once per block (thread 0, double precision like torch's Python-side
// scalars) and broadcast through LDS. beta^t comes from the running products
// F1 keeps in TrainState (t = st->step, 1-based), so no pow() on the device.
__device__ __forceinline__ AdamC adam_consts_block(const TrainState* st, const HParams* hp, AdamC* sh) {
  if (threadIdx.x == 0) {
    const double bc1 = 1.0 - st->b1pow;
    const double bc2 = 1.0 - st->b2pow;
    AdamC c;
    c.step_size = (float)(hp->lr_d / bc1);
    c.bc2s = (float)sqrt(bc2);
    c.b1 = hp->beta1; c.b2 = hp->beta2; c.eps = hp->eps; c.wd = hp->weight_decay;
    c.gs = hp->grad_scale; c.lr = hp->lr; c.decoupled = hp->decoupled_wd;
    *sh = c;
  }
  __syncthreads();
  return *sh;
}

// Same constants when the step state was advanced earlier IN THIS LAUNCH by
// another workgroup (dependent jobs_multi_k launch): beta^t through sc1 vector
// loads, so neither this CU's L1 nor the scalar cache can serve an old copy.
__device__ __forceinline__ AdamC adam_consts_block_sc1(const TrainState* st, const HParams* hp, AdamC* sh) {
  if (threadIdx.x == 0) {
    using gu64 = __attribute__((address_space(1))) unsigned long long;  // global, never flat
    TrainState* s = const_cast<TrainState*>(st);
    const double b1pow =
        __builtin_bit_cast(double, __hip_atomic_load((gu64*)&s->b1pow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const double b2pow =
        __builtin_bit_cast(double, __hip_atomic_load((gu64*)&s->b2pow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    AdamC c;
    c.step_size = (float)(hp->lr_d / (1.0 - b1pow));
    c.bc2s = (float)sqrt(1.0 - b2pow);
    c.b1 = hp->beta1; c.b2 = hp->beta2; c.eps = hp->eps; c.wd = hp->weight_decay;
    c.gs = hp->grad_scale; c.lr = hp->lr; c.decoupled = hp->decoupled_wd;
    *sh = c;
  }
  __syncthreads();
  return *sh;
}

__device__ __forceinline__ void adam_update(float& p, float& m, float& v, float g, const AdamC& c) {
  float gr = g * c.gs;
  if (c.wd != 0.f) {
    if (c.decoupled) p *= (1.f - c.lr * c.wd);
    else gr = fmaf(c.wd, p, gr);
  }
  m = fmaf(1.f - c.b1, gr - m, m);          // exp_avg.lerp_(g, 1-b1)
  v = fmaf(1.f - c.b2, gr * gr, v * c.b2);  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = sqrtf(v) / c.bc2s + c.eps;
  p = p - c.step_size * (m / denom);        // param.addcdiv_(m, denom, -step_size)
}

// Grid-stride streaming Adam over arena range [beg, end) (multiples of 4),
// executed by `nblk` blocks whose local index is `blk`.
__device__ __forceinline__ void adam_stream(float* P, const float* G, float* Mo, float* Vo, long long beg,
                                            long long end, int blk, int nblk, const AdamC& c) {
  const long long n4 = (end - beg) >> 2;
  float4* p4 = reinterpret_cast<float4*>(P + beg);
  const float4* g4 = reinterpret_cast<const float4*>(G + beg);
  float4* m4 = reinterpret_cast<float4*>(Mo + beg);
  float4* v4 = reinterpret_cast<float4*>(Vo + beg);
  for (long long i = (long long)blk * blockDim.x + threadIdx.x; i < n4; i += (long long)nblk * blockDim.x) {
    float4 p = p4[i], g = g4[i], m = m4[i], v = v4[i];
    adam_update(p.x, m.x, v.x, g.x, c);
    adam_update(p.y, m.y, v.y, g.y, c);
    adam_update(p.z, m.z, v.z, g.z, c);
    adam_update(p.w, m.w, v.w, g.w, c);
    p4[i] = p; m4[i] = m; v4[i] = v;
  }
}

}  // namespace mdt
