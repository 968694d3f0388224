#include "reducer.h"

#include <stdexcept>

namespace mdt {

BucketReducer::BucketReducer(c10::intrusive_ptr<c10d::ProcessGroup> pg, at::Tensor flat,
                             std::vector<int64_t> bounds, bool average)
    : pg_(std::move(pg)), flat_(std::move(flat)), bounds_(std::move(bounds)), average_(average) {
  TORCH_CHECK(pg_, "BucketReducer needs a process group (got None)");
  TORCH_CHECK(flat_.dim() == 1 && flat_.is_contiguous(), "flat gradient arena must be 1-D contiguous");
  TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() == flat_.numel(),
              "bucket bounds must start at 0 and end at numel");
  for (size_t i = 1; i < bounds_.size(); ++i)
    TORCH_CHECK(bounds_[i] > bounds_[i - 1], "bucket bounds must be increasing");
  world_ = pg_->getSize();
  // RCCL/NCCL implement AVG natively (pre-mul-sum); gloo does not (also not on GPU tensors).
  use_avg_op_ = average_ && flat_.is_cuda() && pg_->getBackendName() != "gloo";
  work_.resize(bounds_.size() - 1);
}

void BucketReducer::launch(int64_t b) {
  TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
  if (world_ == 1) return;  // size-1 trial group: nothing to reduce
  TORCH_CHECK(!work_[b], "bucket ", b, " launched twice in one iteration");
  std::vector<at::Tensor> t{flat_.narrow(0, bounds_[b], bounds_[b + 1] - bounds_[b])};
  c10d::AllreduceOptions opts;
  opts.reduceOp = use_avg_op_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
  work_[b] = pg_->allreduce(t, opts);
  ++launched_total_;
}

void BucketReducer::wait(int64_t b) {
  TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
  if (!work_[b]) return;
  work_[b]->wait();
  work_[b].reset();
  if (average_ && !use_avg_op_)
    flat_.narrow(0, bounds_[b], bounds_[b + 1] - bounds_[b]).div_((double)world_);
}

void BucketReducer::launch_all() {
  for (int64_t b = 0; b < num_buckets(); ++b)
    if (!work_[b]) launch(b);
}

void BucketReducer::wait_all() {
  for (int64_t b = 0; b < num_buckets(); ++b) wait(b);
}

void BucketReducer::set_param_map(std::vector<int64_t> param_bucket) {
  param_bucket_ = std::move(param_bucket);
  need_.assign(num_buckets(), 0);
  for (auto b : param_bucket_) {
    TORCH_CHECK(b >= 0 && b < num_buckets(), "param bucket out of range");
    need_[b] += 1;
  }
  have_.assign(num_buckets(), 0);
}

void BucketReducer::mark_ready(int64_t p) {
  TORCH_CHECK(p >= 0 && p < (int64_t)param_bucket_.size(), "param index out of range");
  const int64_t b = param_bucket_[p];
  if (++have_[b] == need_[b]) launch(b);
}

void BucketReducer::reset_iteration() {
  std::fill(have_.begin(), have_.end(), 0);
}

int64_t BucketReducer::pending() const {
  int64_t n = 0;
  for (auto& w : work_) n += w ? 1 : 0;
  return n;
}

}  // namespace mdt
