// Native gradient-bucket all-reduce directly on RCCL (xGMI data plane).
//
// The reference relies on torch DDP's Reducer -> ProcessGroupNCCL (pre-divide
// kernel + allreduce + copy-back per bucket, /root/reference/vae-hpo.py:130).
// This reducer reuses the communicator torch already created for the trial
// group (ProcessGroupNCCL._comm_ptr(), so only one RCCL runtime and one
// communicator exist per group) and issues the collectives itself:
//  * averaging is fused into the collective with ncclRedOpCreatePreMulSum(1/s)
//    (no separate scale kernel, no c10d Work objects, no watchdog bookkeeping);
//  * collectives run on a dedicated highest-priority HIP stream, fenced
//    against the compute stream with events in both directions, so a bucket
//    all-reduce overlaps the remaining backward kernels on the xGMI links and
//    the whole exchange stays capturable in a hipGraph (no host waits);
//  * buckets are [begin, end) views of the flat gradient arena: no packing.
// Same Python API as BucketReducer (explicit launch or readiness counting).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <vector>

namespace mdt {

#define MDT_HIP(x)                                                                         \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    TORCH_CHECK(e_ == hipSuccess, "mdt rccl reducer: ", #x, ": ", hipGetErrorString(e_)); \
  } while (0)
#define MDT_NCCL(x)                                                                           \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    TORCH_CHECK(r_ == ncclSuccess, "mdt rccl reducer: ", #x, ": ", ncclGetErrorString(r_)); \
  } while (0)

class RcclBucketReducer {
 public:
  RcclBucketReducer(int64_t comm_ptr, int64_t group_size, at::Tensor flat, std::vector<int64_t> bounds,
                    bool average, double scale)
      : comm_(reinterpret_cast<ncclComm_t>((uintptr_t)comm_ptr)),
        size_((int)group_size),
        flat_(std::move(flat)),
        bounds_(std::move(bounds)) {
    TORCH_CHECK(comm_ != nullptr, "RcclBucketReducer: null communicator");
    TORCH_CHECK(flat_.is_cuda() && flat_.dim() == 1 && flat_.is_contiguous(), "flat arena must be 1-D contiguous CUDA");
    TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() == flat_.numel(),
                "bucket bounds must start at 0 and end at numel");
    for (size_t i = 1; i < bounds_.size(); ++i) TORCH_CHECK(bounds_[i] > bounds_[i - 1], "bounds must increase");
    int nranks = 0;
    MDT_NCCL(ncclCommCount(comm_, &nranks));
    TORCH_CHECK(nranks == size_, "communicator has ", nranks, " ranks, group size is ", size_);
    device_ = flat_.device().index();
    HIPGuard g(device_);
    switch (flat_.scalar_type()) {
      case torch::kFloat32: dtype_ = ncclFloat32; break;
      case torch::kBFloat16: dtype_ = ncclBfloat16; break;
      default: TORCH_CHECK(false, "RcclBucketReducer: arena dtype must be f32 or bf16");
    }
    // pre-multiplier (1/s for averaging) fused into the reduction
    scale_ = (float)(scale > 0 ? scale : (average ? 1.0 / size_ : 1.0));
    if (scale_ != 1.0f) {
      MDT_NCCL(ncclRedOpCreatePreMulSum(&op_, &scale_, ncclFloat32, ncclScalarHostImmediate, comm_));
      custom_op_ = true;
    } else {
      op_ = ncclSum;
    }
    TORCH_CHECK(dtype_ == ncclFloat32 || !custom_op_, "PreMulSum scalar is f32: use an f32 arena");
    int least = 0, greatest = 0;
    MDT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    MDT_HIP(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest));
    const size_t nb = bounds_.size() - 1;
    ready_.resize(nb);
    done_.resize(nb);
    for (size_t b = 0; b < nb; ++b) {
      MDT_HIP(hipEventCreateWithFlags(&ready_[b], hipEventDisableTiming));
      MDT_HIP(hipEventCreateWithFlags(&done_[b], hipEventDisableTiming));
    }
    inflight_.assign(nb, 0);
  }

  ~RcclBucketReducer() {
    // The communicator (and any redop attached to it) belongs to torch's
    // ProcessGroupNCCL and is released with it; only our own objects go here.
    for (auto e : ready_) (void)hipEventDestroy(e);
    for (auto e : done_) (void)hipEventDestroy(e);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  int64_t num_buckets() const { return (int64_t)bounds_.size() - 1; }
  std::vector<int64_t> bounds() const { return bounds_; }
  double scale() const { return scale_; }

  void launch(int64_t b) {
    TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
    TORCH_CHECK(!inflight_[b], "bucket ", b, " launched twice in one iteration");
    HIPGuard g(device_);
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    MDT_HIP(hipEventRecord(ready_[b], cur));          // gradients of bucket b are final
    MDT_HIP(hipStreamWaitEvent(stream_, ready_[b], 0));
    void* p = (char*)flat_.data_ptr() + bounds_[b] * flat_.element_size();
    const size_t count = (size_t)(bounds_[b + 1] - bounds_[b]);
    if (size_ > 1 || custom_op_) {
      MDT_NCCL(ncclAllReduce(p, p, count, dtype_, op_, comm_, stream_));
    }
    MDT_HIP(hipEventRecord(done_[b], stream_));
    inflight_[b] = 1;
    ++launched_total_;
  }

  void wait(int64_t b) {
    TORCH_CHECK(b >= 0 && b < num_buckets(), "bucket index out of range");
    if (!inflight_[b]) return;
    HIPGuard g(device_);
    hipStream_t cur = c10::hip::getCurrentHIPStream(device_).stream();
    MDT_HIP(hipStreamWaitEvent(cur, done_[b], 0));  // device-side join, no host sync
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

 private:
  struct HIPGuard {
    int prev = 0;
    explicit HIPGuard(int dev) {
      (void)hipGetDevice(&prev);
      if (prev != dev) (void)hipSetDevice(dev);
    }
    ~HIPGuard() { (void)hipSetDevice(prev); }
  };

  ncclComm_t comm_;
  int size_;
  at::Tensor flat_;
  std::vector<int64_t> bounds_;
  int device_ = 0;
  ncclDataType_t dtype_ = ncclFloat32;
  ncclRedOp_t op_ = ncclSum;
  bool custom_op_ = false;
  float scale_ = 1.0f;
  hipStream_t stream_ = nullptr;
  std::vector<hipEvent_t> ready_, done_;
  std::vector<int> inflight_;
  std::vector<int64_t> param_bucket_, need_, have_;
  int64_t launched_total_ = 0;
};

int64_t rccl_version() {
  int v = 0;
  MDT_NCCL(ncclGetVersion(&v));
  return v;
}

void bind_rccl(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<RcclBucketReducer>(m, "RcclBucketReducer")
      .def(py::init<int64_t, int64_t, at::Tensor, std::vector<int64_t>, bool, double>(), py::arg("comm_ptr"),
           py::arg("group_size"), py::arg("flat"), py::arg("bounds"), py::arg("average") = true,
           py::arg("scale") = 0.0)
      .def("num_buckets", &RcclBucketReducer::num_buckets)
      .def("bounds", &RcclBucketReducer::bounds)
      .def("scale", &RcclBucketReducer::scale)
      .def("launch", &RcclBucketReducer::launch)
      .def("wait", &RcclBucketReducer::wait)
      .def("launch_all", &RcclBucketReducer::launch_all)
      .def("wait_all", &RcclBucketReducer::wait_all)
      .def("set_param_map", &RcclBucketReducer::set_param_map)
      .def("mark_ready", &RcclBucketReducer::mark_ready)
      .def("reset_iteration", &RcclBucketReducer::reset_iteration)
      .def("pending", &RcclBucketReducer::pending)
      .def("launched_count", &RcclBucketReducer::launched_count);
  m.def("rccl_version", &rccl_version);
}

}  // namespace mdt
