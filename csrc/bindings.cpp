// Python bindings of the native runtime (multidisttorch_amd._C).
#include <torch/extension.h>

#include "runtime/reducer.h"
#include "runtime/vae_engine.h"

namespace py = pybind11;

namespace mdt {
void probe_clock(at::Tensor out, int64_t iters);
void probe_latency(at::Tensor idx, int64_t hops, at::Tensor out);
void probe_empty(int64_t blocks, int64_t threads);
void probe_lds_poison(int64_t pattern, int64_t blocks);
void probe_cu_ids(at::Tensor out);
void bind_conv(pybind11::module& m);
void bind_rccl(pybind11::module& m);
void bind_p2p(pybind11::module& m);
void bind_cpu(pybind11::module& m);
}  // namespace mdt

PYBIND11_MODULE(_C, m) {
  m.doc() = "multidisttorch_amd native runtime: HIP/CDNA4 kernels + C++ reducer";
  m.attr("ARCH") = "gfx950";
  m.def("probe_clock", &mdt::probe_clock);
  m.def("probe_latency", &mdt::probe_latency);
  m.def("probe_empty", &mdt::probe_empty);
  m.def("probe_cu_ids", &mdt::probe_cu_ids);
  m.def("probe_lds_poison", &mdt::probe_lds_poison, py::arg("pattern"), py::arg("blocks") = 1024);
  mdt::bind_conv(m);
  mdt::bind_rccl(m);
  mdt::bind_p2p(m);
  mdt::bind_cpu(m);

  py::class_<mdt::MlpVaeEngine>(m, "MlpVaeEngine")
      .def(py::init<int64_t, int64_t, int64_t, int64_t, int64_t>(), py::arg("batch"),
           py::arg("D"), py::arg("H"), py::arg("Z"), py::arg("device_index"))
      .def("layout", &mdt::MlpVaeEngine::layout)
      .def("numel", &mdt::MlpVaeEngine::numel)
      .def("bucket_split", &mdt::MlpVaeEngine::bucket_split)
      .def("set_hparams", &mdt::MlpVaeEngine::set_hparams, py::arg("lr"), py::arg("beta1"),
           py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("kl_beta"),
           py::arg("grad_scale"), py::arg("seed"), py::arg("decoupled_wd") = false)
      .def("set_cursor", &mdt::MlpVaeEngine::set_cursor)
      .def("set_step", &mdt::MlpVaeEngine::set_step)
      .def("reset_loss", &mdt::MlpVaeEngine::reset_loss)
      .def("read_state", &mdt::MlpVaeEngine::read_state)
      .def("loss_history", &mdt::MlpVaeEngine::loss_history)
      .def("forward", &mdt::MlpVaeEngine::forward, py::arg("X"), py::arg("idx"), py::arg("M"),
           py::arg("train"), py::arg("eval"), py::arg("rng_stream"), py::arg("want_recon"))
      .def("backward", &mdt::MlpVaeEngine::backward, py::arg("X"), py::arg("idx"), py::arg("M"),
           py::arg("part") = 0, py::arg("fuse_adam") = false)
      .def("adam", &mdt::MlpVaeEngine::adam)
      .def("loss_finalize", &mdt::MlpVaeEngine::loss_finalize, py::arg("eval"))
      .def("act", &mdt::MlpVaeEngine::act)
      .def("decode", &mdt::MlpVaeEngine::decode)
      .def("set_stamps", &mdt::MlpVaeEngine::set_stamps)
      .def_readonly("params", &mdt::MlpVaeEngine::params)
      .def_readonly("grads", &mdt::MlpVaeEngine::grads)
      .def_readonly("exp_avg", &mdt::MlpVaeEngine::exp_avg)
      .def_readonly("exp_avg_sq", &mdt::MlpVaeEngine::exp_avg_sq)
      .def_readonly("partials", &mdt::MlpVaeEngine::partials)
      .def_readonly("train_state", &mdt::MlpVaeEngine::train_state)
      .def_readonly("eval_state", &mdt::MlpVaeEngine::eval_state)
      .def_readonly("hparams", &mdt::MlpVaeEngine::hparams);

  py::class_<mdt::BucketReducer>(m, "BucketReducer")
      .def(py::init<c10::intrusive_ptr<c10d::ProcessGroup>, at::Tensor, std::vector<int64_t>, bool>(),
           py::arg("pg"), py::arg("flat"), py::arg("bounds"), py::arg("average"))
      .def("num_buckets", &mdt::BucketReducer::num_buckets)
      .def("bounds", &mdt::BucketReducer::bounds)
      .def("launch", &mdt::BucketReducer::launch, py::call_guard<py::gil_scoped_release>())
      .def("wait", &mdt::BucketReducer::wait, py::call_guard<py::gil_scoped_release>())
      .def("launch_all", &mdt::BucketReducer::launch_all, py::call_guard<py::gil_scoped_release>())
      .def("wait_all", &mdt::BucketReducer::wait_all, py::call_guard<py::gil_scoped_release>())
      .def("set_param_map", &mdt::BucketReducer::set_param_map)
      .def("mark_ready", &mdt::BucketReducer::mark_ready, py::call_guard<py::gil_scoped_release>())
      .def("reset_iteration", &mdt::BucketReducer::reset_iteration)
      .def("pending", &mdt::BucketReducer::pending)
      .def("launched_count", &mdt::BucketReducer::launched_count);
}
