// Bucketed gradient all-reduce over a flat gradient arena (native DDP reducer).
//
// Replaces torch DDP's C++ Reducer as used by /root/reference/vae-hpo.py:130
// (25 MiB buckets, per-param copy into bucket storage, copy-back into .grad).
// Here gradients already live in one contiguous arena, so a bucket is a plain
// [begin, end) view: no pack, no copy-back. Buckets are launched
//  * explicitly (`launch(b)`) by the fused MLP-VAE step, which knows exactly
//    after which backward kernel a bucket's gradients are final, or
//  * by readiness counting (`mark_ready(param)`) from autograd post-accumulate
//    hooks for generic modules (conv-VAE).
// Collectives go through the c10d ProcessGroup handed in from Python: RCCL
// (ProcessGroupNCCL, its own comm stream, fenced against the compute stream,
// graph-capturable) on MI355X, gloo on CPU for the multi-process tests.
#pragma once
#include <torch/extension.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <vector>

namespace mdt {

class BucketReducer {
 public:
  BucketReducer(c10::intrusive_ptr<c10d::ProcessGroup> pg, at::Tensor flat,
                std::vector<int64_t> bounds, bool average);

  int64_t num_buckets() const { return (int64_t)bounds_.size() - 1; }
  std::vector<int64_t> bounds() const { return bounds_; }
  void launch(int64_t b);
  void wait(int64_t b);
  void wait_all();
  void launch_all();

  // readiness mode
  void set_param_map(std::vector<int64_t> param_bucket);
  void mark_ready(int64_t param_index);
  void reset_iteration();
  int64_t pending() const;
  int64_t launched_count() const { return launched_total_; }

 private:
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  at::Tensor flat_;
  std::vector<int64_t> bounds_;
  bool average_;
  bool use_avg_op_;
  int world_;
  std::vector<c10::intrusive_ptr<c10d::Work>> work_;
  std::vector<int64_t> param_bucket_, need_, have_;
  int64_t launched_total_ = 0;
};

}  // namespace mdt
