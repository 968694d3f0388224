// Stream/event bookkeeping shared by the device-side bucket reducers
// (RcclBucketReducer, XgmiP2PReducer).
//
// A bucket is a [begin, end) view of a flat gradient arena. `launch(b)` records
// "gradients of b are final" on the caller's current stream, makes the reducer's
// own highest-priority stream wait for it, issues the collective there and
// records completion; `wait(b)` joins the caller's stream on that completion.
// Everything is device-side (events only, no host waits), so the whole exchange
// can be captured into a hipGraph together with the compute it overlaps.
// Buckets are launched explicitly by fused model steps or by readiness
// counting (`mark_ready(param)`) from autograd hooks.
#pragma once
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <vector>

namespace mdt {

#define MDT_HIP_CHECK(x)                                                         \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    TORCH_CHECK(e_ == hipSuccess, "mdt: ", #x, ": ", hipGetErrorString(e_));     \
  } while (0)

struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

class StreamBuckets {
 public:
  StreamBuckets(at::Tensor flat, std::vector<int64_t> bounds) : flat_(std::move(flat)), bounds_(std::move(bounds)) {
    TORCH_CHECK(flat_.is_cuda() && flat_.dim() == 1 && flat_.is_contiguous(), "flat arena must be 1-D contiguous CUDA");
    TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() == flat_.numel(),
                "bucket bounds must start at 0 and end at numel");
    for (size_t i = 1; i < bounds_.size(); ++i) TORCH_CHECK(bounds_[i] > bounds_[i - 1], "bounds must increase");
    device_ = flat_.device().index();
    DeviceGuard g(device_);
    int least = 0, greatest = 0;
    MDT_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    MDT_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest));
    const size_t nb = bounds_.size() - 1;
    ready_.resize(nb);
    done_.resize(nb);
    for (size_t b = 0; b < nb; ++b) {
      MDT_HIP_CHECK(hipEventCreateWithFlags(&ready_[b], hipEventDisableTiming));
      MDT_HIP_CHECK(hipEventCreateWithFlags(&done_[b], hipEventDisableTiming));
    }
    inflight_.assign(nb, 0);
  }
  virtual ~StreamBuckets() {
    for (auto e : ready_) (void)hipEventDestroy(e);
    for (auto e : done_) (void)hipEventDestroy(e);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  StreamBuckets(const StreamBuckets&) = delete;
  StreamBuckets& operator=(const StreamBuckets&) = delete;

  int64_t num_buckets() const { return (int64_t)bounds_.size() - 1; }
  std::vector<int64_t> bounds() const { return bounds_; }

  // inline mode: collectives go on the CALLER's stream, in issue order, with
  // no events -- no cross-queue dependency inside a replayed graph (each costs
  // 5-12 us on this stack, profiles/r3_rccl_graph); wait() is then a no-op.
  void set_inline(bool v) { inline_ = v; }
  bool is_inline() const { return inline_; }

  void launch(int64_t b) {
    TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
    TORCH_CHECK(!inflight_[b], "bucket ", b, " launched twice in one iteration");
    DeviceGuard g(device_);
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    if (inline_) {
      issue(b, cur);
      ++launched_total_;
      return;
    }
    MDT_HIP_CHECK(hipEventRecord(ready_[b], cur));  // gradients of bucket b are final
    MDT_HIP_CHECK(hipStreamWaitEvent(stream_, ready_[b], 0));
    issue(b, stream_);
    MDT_HIP_CHECK(hipEventRecord(done_[b], stream_));
    inflight_[b] = 1;
    ++launched_total_;
  }
  void wait(int64_t b) {
    TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
    if (!inflight_[b]) return;
    DeviceGuard g(device_);
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    MDT_HIP_CHECK(hipStreamWaitEvent(cur, done_[b], 0));  // device-side join, no host sync
    inflight_[b] = 0;
  }
  void launch_all() {
    for (int64_t b = 0; b < num_buckets(); ++b)
      if (!inflight_[b]) launch(b);
  }
  void wait_all() {
    for (int64_t b = 0; b < num_buckets(); ++b) wait(b);
  }

  void set_param_map(std::vector<int64_t> param_bucket) {
    param_bucket_ = std::move(param_bucket);
    need_.assign(num_buckets(), 0);
    for (auto b : param_bucket_) {
      TORCH_CHECK(b >= 0 && b < num_buckets(), "param bucket out of range");
      need_[b] += 1;
    }
    have_.assign(num_buckets(), 0);
  }
  void mark_ready(int64_t p) {
    TORCH_CHECK(p >= 0 && p < (int64_t)param_bucket_.size(), "param index out of range");
    const int64_t b = param_bucket_[p];
    if (++have_[b] == need_[b]) launch(b);
  }
  void reset_iteration() { std::fill(have_.begin(), have_.end(), 0); }
  int64_t pending() const {
    int64_t n = 0;
    for (auto v : inflight_) n += v;
    return n;
  }
  int64_t launched_count() const { return launched_total_; }

 protected:
  // enqueue bucket b's collective on `s` (the reducer's own stream)
  virtual void issue(int64_t b, hipStream_t s) = 0;

  at::Tensor flat_;
  std::vector<int64_t> bounds_;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  bool inline_ = false;

 private:
  std::vector<hipEvent_t> ready_, done_;
  std::vector<int> inflight_;
  std::vector<int64_t> param_bucket_, need_, have_;
  int64_t launched_total_ = 0;
};

// pybind11: the common bucket API on a concrete reducer class
template <class Cls>
void def_bucket_api(Cls& c) {
  namespace py = pybind11;
  using T = typename Cls::type;
  c.def("num_buckets", &T::num_buckets)
      .def("bounds", &T::bounds)
      .def("launch", &T::launch)
      .def("wait", &T::wait)
      .def("launch_all", &T::launch_all)
      .def("wait_all", &T::wait_all)
      .def("set_param_map", &T::set_param_map)
      .def("mark_ready", &T::mark_ready)
      .def("reset_iteration", &T::reset_iteration)
      .def("pending", &T::pending)
      .def("launched_count", &T::launched_count)
      .def("set_inline", &T::set_inline)
      .def("is_inline", &T::is_inline);
}

}  // namespace mdt
