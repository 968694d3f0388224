// Peer-to-peer all-reduce over xGMI, one-shot and two-shot (host/device shared declarations).
//
// Included by the HIP kernel (p2p_allreduce.hip) and by the host reducer
// (csrc/runtime/p2p_comm.cpp); plain data only.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace mdt {

constexpr int kP2PMaxRanks = 8;  // one xGMI hop: a group never spans more than one node

struct P2PArgs {
  float* data;                          // this rank's bucket, reduced in place
  long long n;                          // bucket elements
  float* peer_recv[kP2PMaxRanks];       // every rank's receive region base (device VA in this process)
  unsigned* peer_flags[kP2PMaxRanks];   // every rank's flag region base
  float* my_recv;                       // == peer_recv[me]
  unsigned* my_flags;                   // == peer_flags[me]
  unsigned* ep;                         // per-block epoch counters of this bucket (local only)
  int* status;                          // 0 = ok, 1 + bucket = a wait timed out
  long long recv_off;                   // this bucket's receive slab: [2 parity][s src][n]
                                        // (two-shot: RS [2 parity][s src][chunk] then AG, same shape)
  long long flag_off;                   // this bucket's flags: [2 phase][s src][grid]
  int me, s, bucket;
  int two_shot;                         // 1: reduce-scatter by chunk owner + all-gather
  float scale;                          // 1/s for averaging
  long long timeout_ticks;              // s_memrealtime ticks (100 MHz)
  const int* abort_flag;                // host-mapped word the host sets to abandon every wait (may be null)
};

// Device descriptor of the all-reduce JOBS (comm_jobs.h) over a gradient
// arena of `numel` elements; built by XgmiP2PReducer.comm_ctx().
struct CommCtx {
  float* peer_recv[kP2PMaxRanks];      // every rank's receive region (device VA in this process)
  unsigned* peer_flags[kP2PMaxRanks];  // every rank's flag array
  int* status;                         // 0 ok; else 1 + 1000000 + arena offset of a unit whose wait timed out,
                                       // or kCommAborted once a wait saw the host's abort word
  const int* abort_flag;               // host-mapped word: nonzero = abandon every wait (runner's _abort)
  long long numel;                     // gradient arena elements (receive stride)
  long long ep_base;                   // epoch of a step = TrainState.step + ep_base (rebase_epochs)
  int me, s;
  int two_shot;                        // 1 (groups >= 3): reduce-scatter to chunk owners + all-gather per unit
  float scale;                         // 1/s (averaging) or a test pre-multiplier
  long long timeout_ticks;             // s_memrealtime ticks (100 MHz)
};

enum : int { kCommPush = 1, kCommReduce = 2, kCommPushReduce = 3 };
constexpr int kCommAborted = 999999;  // status after an abort (distinct from 1 + bucket / 1000001 + offset)

}  // namespace mdt

extern "C" int mdt_p2p_allreduce(const mdt::P2PArgs* a, int grid, hipStream_t stream);
extern "C" int mdt_selftest_fill(float* g, long long n, int q, hipStream_t stream);
extern "C" int mdt_selftest_check(const float* g, long long n, int s, float scale, int* bad, hipStream_t stream);
