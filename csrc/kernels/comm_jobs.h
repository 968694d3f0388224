// Gradient all-reduce over xGMI fused into the backward's job launches (gfx950).
//
// Reference counterpart: torch DDP's Reducer, which launches a bucket's
// all-reduce from the autograd hooks while backward continues, waits, copies
// the averaged bucket back into .grad, after which foreach-Adam runs
// (/root/reference/vae-hpo.py:72-74, :130). On this stack every one of those
// hand-offs between streams costs 5-12 us inside a replayed step graph
// (profiles/r3_rccl_graph/step_sequence.txt: a cross-queue dependency is a
// barrier packet + completion-signal round trip, and RCCL kernel nodes add
// their own gaps), which doubled the 64 us 28x28 step. So here the collective
// is not a kernel on a second stream: it is a JOB of the launches the backward
// issues anyway, one stream, no events.
//
// A job works on the finalize units of the weight-gradient plan (GradUnit:
// `count` consecutive elements of one segment), one 256-thread workgroup per
// unit, in three modes:
//   push         finalize the unit (sum its split-K partial slabs, the same
//                order as grad_finalize: slab_sum4 / slab_partial), keep it in
//                the local gradient arena, store it straight into every peer's
//                receive region (remote stores through the hipIpc mapping, one
//                xGMI hop, all s-1 links of the group at once), then publish
//                one flag per (source rank, unit) in every peer;
//   reduce       wait for the unit's flag from every peer (bounded), sum the s
//                contributions IN RANK ORDER (bitwise the same on every
//                replica), scale (1/s), then Adam + the bf16 weight copy in
//                the same thread;
//   push+reduce  both in one workgroup, the own contribution kept in registers.
// The 28x28 DDP step (models/conv_vae.py::_step28) puts the decoder units'
// push into the launch that computes the encoder weight gradients -- the
// decoder bucket's transfer runs on the xGMI links while those workgroups
// compute -- and ends with ONE launch of push+reduce (encoder) || reduce
// (decoder), which also applies Adam. On one rank (s = 1) the jobs degenerate
// to finalize + scale + Adam: the same step structure with nothing to move,
// which is how its cost is measured on a one-GPU box.
//
// Memory: the receive region and flags live in ONE uncached device
// allocation per rank (hipDeviceMallocUncached; exported with hipIpc by
// XgmiP2PReducer, csrc/runtime/p2p_comm.cpp), indexed by ARENA OFFSET, so any
// unit decomposition works without re-sizing the shared region:
//   recv  [2 parity][s src][numel] f32      flags [s src][numel] u32
//   (a flag is stored at its unit's first element only)
// Epoch: ONE per step for every unit, e = TrainState.step + ep_base. Every job
// of a step runs after the launch that advanced `step` (f28: the loss/step job
// of the first job launch; layer path: the forward's first launch), so all
// units of a step -- whatever the batch size M made of the unit
// decomposition -- agree on e and on the receive parity e & 1 (the per-unit
// epochs of round 4 gave full and tail steps different parities for the same
// elements). Parity double-buffers the receive slots: a peer can
// run at most one step ahead (its step k+2 push needs its step k+1 reduce,
// which needs this rank's step k+1 pushes, which follow this rank's step k
// reduce on the same stream). A flag only ever grows while `step` grows;
// ``rebase_epochs`` keeps e increasing when the host moves `step` backwards.
// Publication: every storing wave waits for its stores (s_waitcnt vmcnt(0)
// after the release fence, MI355X_MICROARCH.md "Compiler hazard"), then a
// workgroup barrier, then one lane per peer does a system-scope release store
// of the flag; the consumer polls with system-scope acquire loads, then a
// barrier. A wait longer than `timeout_ticks` sets `status` (1 + 1000000 +
// unit offset, never 0) and leaves the unit's parameters unchanged: a lost peer
// never hangs the GPU. Once `status` is set, or the host raised the abort word
// (host-mapped, XgmiP2PReducer.abort(): the runner's _abort on a lost peer),
// a wait gives up at its first unsuccessful poll, so the steps still queued
// behind a failure drain in microseconds each instead of one timeout each.
#pragma once
#include "conv_small.h"
#include "p2p_allreduce.h"

namespace mdt {

struct CommJobArgs {
  FinalizeArgs fa;      // P, G, m, v, w16, segs, units (this job's slice), state, hparams, do_adam
  const CommCtx* ctx;   // device memory (built by the reducer)
  int mode;             // kCommPush | kCommReduce | kCommPushReduce
};

constexpr int kCommLds = kFinalizeThreads * 4 + 64 + 16;

// Publication of a unit's stores to every peer: each storing wave waits for
// its stores (release fence + vmcnt(0)), a workgroup barrier, then lane p
// stores `val` into peer p's flag of (this rank, unit) at system scope.
__device__ __forceinline__ void comm_publish(const CommCtx* cx, long long o0, unsigned val, int t) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < cx->s && t != cx->me)
    __hip_atomic_store(cx->peer_flags[t] + (long long)cx->me * cx->numel + o0, val, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait until every peer's flag of the unit reaches `target` (bounded; gives up
// at once after a recorded failure or a host abort: *s_ok = 0), then barrier +
// acquire. Lane p of wave 0 polls peer p's flag in local memory.
__device__ __forceinline__ void comm_wait(const CommCtx* cx, long long o0, unsigned target, int t, int* s_ok) {
  if (t < 64 && *s_ok) {
    const int me = cx->me;
    const bool mine = t < cx->s && t != me;
    const unsigned* f = cx->peer_flags[me] + (long long)(mine ? t : 0) * cx->numel + o0;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned it = 0;; ++it) {
      const bool ready =
          !mine || (int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - target) >= 0;
      if (__all(ready)) break;
      // a failure already recorded (this or an earlier step) or a host abort: give up now
      if ((it & 63u) == 0 && p2p_wait_abandoned(cx->status, cx->abort_flag, t)) {
        if (t == 0) {
          atomicCAS(cx->status, 0, kCommAborted);
          *s_ok = 0;
        }
        break;
      }
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > cx->timeout_ticks) {
        if (t == 0) {
          atomicCAS(cx->status, 0, (int)(1 + 1000000 + (o0 < 2000000000LL ? o0 : 2000000000LL)));
          *s_ok = 0;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

__device__ __forceinline__ void comm_unit_body(const CommJobArgs& a, uint8_t* lds, int b) {
  float* red = reinterpret_cast<float*>(lds);
  AdamC* cs = reinterpret_cast<AdamC*>(lds + kFinalizeThreads * 4);
  unsigned* s_ep = reinterpret_cast<unsigned*>(lds + kFinalizeThreads * 4 + 64);
  int* s_ok = reinterpret_cast<int*>(s_ep + 1);
  const FinalizeArgs& fa = a.fa;
  const CommCtx* cx = a.ctx;
  const bool push = (a.mode & kCommPush) != 0, reduce = (a.mode & kCommReduce) != 0;
  const bool adam = reduce && fa.do_adam;
  AdamC c{};
  if (adam) c = adam_consts_block(fa.st, fa.hp, cs);
  const GradUnit u = fa.units[b];
  const GradSeg sg = fa.segs[u.seg];
  const long long o0 = sg.off + u.start;  // the unit's first arena element: its flag / epoch slot
  const int S = cx->s, me = cx->me;
  if (threadIdx.x == 0) {
    *s_ep = (unsigned)(fa.st->step + cx->ep_base);
    *s_ok = 1;
  }
  __syncthreads();
  const unsigned e = *s_ep;
  const long long rs = cx->numel;
  const int par = (int)(e & 1u);

  // this thread's elements: [o, o + nel), nel in 0..4
  const int t = threadIdx.x;
  const bool v4 = u.count > kFinalizeThreads;
  long long o = 0;
  int nel = 0;
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  if (v4) {
    const int e0 = u.start + 4 * t;
    const int left = u.start + u.count - e0;
    nel = left <= 0 ? 0 : (left < 4 ? left : 4);
    o = sg.off + e0;
    if (push && nel == 4 && sg.slab) {
      const f32x4 s4 = slab_sum4(sg.slab + e0, sg.numel, sg.nsplit);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = s4[j];
    } else if (push && sg.slab) {
      for (int j = 0; j < nel; ++j) g[j] = slab_sum1(sg.slab + e0 + j, sg.numel, sg.nsplit);
    } else if (nel == 4) {
      const f32x4 s4 = *reinterpret_cast<const f32x4*>(fa.G + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) g[j] = s4[j];
    } else {
      for (int j = 0; j < nel; ++j) g[j] = fa.G[o + j];
    }
  } else {
    const int cnt = u.count, rp = kFinalizeThreads / cnt;
    const int col = t % cnt, rl = t / cnt;
    if (push && sg.slab) {
      red[t] = rl < rp ? slab_partial(sg.slab + u.start + col, sg.numel, sg.nsplit, rl, rp) : 0.f;
      __syncthreads();
      if (rl == 0) {
        float s1 = 0.f;
        for (int r = 0; r < rp; ++r) s1 += red[r * cnt + col];
        g[0] = s1;
      }
    }
    if (rl == 0) {
      nel = 1;
      o = sg.off + u.start + col;
      if (!(push && sg.slab)) g[0] = fa.G[o];
    }
  }

  // two-shot (groups >= 3, CommCtx.two_shot): the unit is cut into S chunks of
  // `chunk` elements (a multiple of 4 from the unit start, so a thread's elements
  // never straddle two chunks); chunk q is owned by rank q
  const bool two = cx->two_shot && S > 2;
  const int chunk = two ? ((u.count + S - 1) / S + 3) / 4 * 4 : u.count;
  const int owner = two ? (int)((o - o0) / chunk) : me;

  if (push) {
    // own contribution into the local arena, then into the receive slot [par][me]
    // of every peer (one-shot) or of the chunk's owner only (two-shot)
    if (nel == 4) {
      const f32x4 s4 = {g[0], g[1], g[2], g[3]};
      *reinterpret_cast<f32x4*>(fa.G + o) = s4;
      for (int p = 0; p < S; ++p)
        if (p != me && (!two || p == owner))
          *reinterpret_cast<f32x4*>(cx->peer_recv[p] + ((long long)par * S + me) * rs + o) = s4;
    } else {
      for (int j = 0; j < nel; ++j) {
        fa.G[o + j] = g[j];
        for (int p = 0; p < S; ++p)
          if (p != me && (!two || p == owner)) cx->peer_recv[p][((long long)par * S + me) * rs + o + j] = g[j];
      }
    }
    if (S > 1) comm_publish(cx, o0, 2u * e - 1u, t);
  }

  if (reduce) {
    if (S > 1) comm_wait(cx, o0, 2u * e - 1u, t, s_ok);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const float* my_recv = cx->peer_recv[me];
    if (*s_ok && nel > 0 && owner == me) {
      // rank-order sum: identical bits on every replica (and two-shot == one-shot)
      for (int p = 0; p < S; ++p) {
        if (p == me) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = p == 0 ? g[j] : acc[j] + g[j];
        } else {
          const float* src = my_recv + ((long long)par * S + p) * rs + o;
          if (nel == 4) {
            const f32x4 r4 = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = p == 0 ? r4[j] : acc[j] + r4[j];
          } else {
            for (int j = 0; j < nel; ++j) acc[j] = p == 0 ? src[j] : acc[j] + src[j];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] *= cx->scale;
      if (two) {
        // all-gather: the reduced chunk into every peer's slot [par][me] (its
        // elements there are never a reduce-scatter target: those are the
        // peer's own chunk)
        for (int p = 0; p < S; ++p) {
          if (p == me) continue;
          float* dst = cx->peer_recv[p] + ((long long)par * S + me) * rs + o;
          if (nel == 4) {
            *reinterpret_cast<f32x4*>(dst) = f32x4{acc[0], acc[1], acc[2], acc[3]};
          } else {
            for (int j = 0; j < nel; ++j) dst[j] = acc[j];
          }
        }
      }
    }
    if (two) {
      // a failed reduce-scatter wait publishes nothing: the peers then fail
      // their own wait (status) instead of reading a chunk that never came
      if (*s_ok) comm_publish(cx, o0, 2u * e, t);
      comm_wait(cx, o0, 2u * e, t, s_ok);
      if (*s_ok && nel > 0 && owner != me) {  // the owner's reduced, scaled chunk
        const float* src = my_recv + ((long long)par * S + owner) * rs + o;
        if (nel == 4) {
          const f32x4 r4 = *reinterpret_cast<const f32x4*>(src);
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j] = r4[j];
        } else {
          for (int j = 0; j < nel; ++j) acc[j] = src[j];
        }
      }
    }
    if (*s_ok && nel > 0) {
      if (!adam) {
        if (nel == 4) {
          const f32x4 s4 = {acc[0], acc[1], acc[2], acc[3]};
          *reinterpret_cast<f32x4*>(fa.G + o) = s4;
        } else {
          for (int j = 0; j < nel; ++j) fa.G[o + j] = acc[j];
        }
      } else if (nel == 4) {
        f32x4 p4 = *reinterpret_cast<const f32x4*>(fa.P + o);
        f32x4 m4 = *reinterpret_cast<const f32x4*>(fa.Mo + o);
        f32x4 w4 = *reinterpret_cast<const f32x4*>(fa.Vo + o);
        typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
        bf16x4 h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float pj = p4[j], mj = m4[j], vj = w4[j];
          adam_update(pj, mj, vj, acc[j], c);
          p4[j] = pj; m4[j] = mj; w4[j] = vj;
          h[j] = (__bf16)pj;
        }
        *reinterpret_cast<f32x4*>(fa.P + o) = p4;
        *reinterpret_cast<f32x4*>(fa.Mo + o) = m4;
        *reinterpret_cast<f32x4*>(fa.Vo + o) = w4;
        *reinterpret_cast<bf16x4*>(fa.w16 + o) = h;
      } else {
        for (int j = 0; j < nel; ++j) {
          float pj = fa.P[o + j], mj = fa.Mo[o + j], vj = fa.Vo[o + j];
          adam_update(pj, mj, vj, acc[j], c);
          fa.P[o + j] = pj; fa.Mo[o + j] = mj; fa.Vo[o + j] = vj;
          fa.w16[o + j] = (__bf16)pj;
        }
      }
    }
  }
}

}  // namespace mdt
