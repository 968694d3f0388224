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
#include <rccl/rccl.h>

#include "runtime/stream_buckets.h"

namespace mdt {

#define MDT_NCCL(x)                                                                           \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    TORCH_CHECK(r_ == ncclSuccess, "mdt rccl reducer: ", #x, ": ", ncclGetErrorString(r_)); \
  } while (0)

class RcclBucketReducer : public StreamBuckets {
 public:
  RcclBucketReducer(int64_t comm_ptr, int64_t group_size, at::Tensor flat, std::vector<int64_t> bounds,
                    bool average, double scale)
      : StreamBuckets(std::move(flat), std::move(bounds)),
        comm_(reinterpret_cast<ncclComm_t>((uintptr_t)comm_ptr)),
        size_((int)group_size) {
    TORCH_CHECK(comm_ != nullptr, "RcclBucketReducer: null communicator");
    int nranks = 0;
    MDT_NCCL(ncclCommCount(comm_, &nranks));
    TORCH_CHECK(nranks == size_, "communicator has ", nranks, " ranks, group size is ", size_);
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
  }
  // The communicator (and any redop attached to it) belongs to torch's
  // ProcessGroupNCCL and is released with it; events/stream: ~StreamBuckets.

  double scale() const { return scale_; }

 protected:
  void issue(int64_t b, hipStream_t s) override {
    void* p = (char*)flat_.data_ptr() + bounds_[b] * flat_.element_size();
    const size_t count = (size_t)(bounds_[b + 1] - bounds_[b]);
    if (size_ > 1 || custom_op_) MDT_NCCL(ncclAllReduce(p, p, count, dtype_, op_, comm_, s));
  }

 private:
  ncclComm_t comm_;
  int size_;
  ncclDataType_t dtype_ = ncclFloat32;
  ncclRedOp_t op_ = ncclSum;
  bool custom_op_ = false;
  float scale_ = 1.0f;
};

int64_t rccl_version() {
  int v = 0;
  MDT_NCCL(ncclGetVersion(&v));
  return v;
}

void bind_rccl(pybind11::module& m) {
  namespace py = pybind11;
  auto c = py::class_<RcclBucketReducer>(m, "RcclBucketReducer")
               .def(py::init<int64_t, int64_t, at::Tensor, std::vector<int64_t>, bool, double>(),
                    py::arg("comm_ptr"), py::arg("group_size"), py::arg("flat"), py::arg("bounds"),
                    py::arg("average") = true, py::arg("scale") = 0.0)
               .def("scale", &RcclBucketReducer::scale);
  def_bucket_api(c);
  m.def("rccl_version", &rccl_version);
}

}  // namespace mdt
