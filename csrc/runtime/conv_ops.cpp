// Torch bindings of the conv-VAE kernels (csrc/kernels/conv_bf16.hip) and a
// device-resident trial state (same TrainState / HParams structs as the MLP
// engine) for generic trainers.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <cmath>
#include <cstring>
#include <tuple>
#include <vector>

#include "../kernels/vae_mlp.h"

namespace mdt {
struct ConvDesc {
  int N, H, W, C;
  int OH, OW, CO;
  int KH, KW, S, P;
};
struct AdamSeg {
  long long off, numel;
  int co, taps, ci;
  long long toff;
};
}  // namespace mdt

extern "C" {
int mdt_conv_fwd(const void* X, int x_is_f32, const int* rows, const void* W16, mdt::ConvDesc d, const float* bias,
                 int relu, void* y16, float* y32, const void* omask, hipStream_t s);
int mdt_conv_dgrad(const void* G16, const void* mask16, const void* Wt16, mdt::ConvDesc d, const float* bias, int relu,
                   void* y16, float* y32, const void* omask, hipStream_t s);
int mdt_gather_rows(const float* X, const int* idx, const void* st, int B, int M, int P, float* xb, hipStream_t s);
int mdt_conv_wgrad(const void* G16, const void* mask16, const void* X, int x_is_f32, const int* rows, mdt::ConvDesc d,
                   float* dW, float* db, hipStream_t s);
int mdt_chan_sum(const void* G16, int M, int C, float* db, hipStream_t s);
int mdt_reparam(const float* mulv, float* eps, void* z16, float* z32, int B, int Z, const void* st, const void* hp,
                unsigned stream, float* kld_part, hipStream_t s);
int mdt_reparam_bwd(const float* dz, const float* mulv, const float* eps, float* dmulv, void* dmulv16, int B, int Z,
                    const void* hp, hipStream_t s);
int mdt_bce_logits(const float* logits, const float* X, const int* rows, int B, int P, void* dlog16, float* recon,
                   float* part, hipStream_t s);
int mdt_conv_loss_finalize(const float* bce_part, int nb, const float* kld_part, int nk, void* st, const void* hp,
                           int advance_cursor, hipStream_t s);
int mdt_step_begin(void* st, const void* hp, hipStream_t s);
int mdt_adam_cast(float* P, const float* G, float* Mo, float* Vo, void* w16, void* w16t, const void* segs, int nseg,
                  long long total, const void* st, const void* hp, int do_adam, hipStream_t s);
}

namespace mdt {

static hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }
static void rc(int r, const char* w) { TORCH_CHECK(r == 0, "mdt: ", w, " failed (", r, ")"); }
static const void* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

static ConvDesc desc(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 11, "conv desc needs 11 ints (N,H,W,C,OH,OW,CO,KH,KW,S,P)");
  return ConvDesc{(int)v[0], (int)v[1], (int)v[2], (int)v[3], (int)v[4], (int)v[5],
                  (int)v[6], (int)v[7], (int)v[8], (int)v[9], (int)v[10]};
}

static void check_bf16(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16 && t.is_contiguous(), n,
              " must be a contiguous CUDA bfloat16 tensor");
}

void conv_fwd(const at::Tensor& X, const c10::optional<at::Tensor>& rows, const at::Tensor& W16,
              const std::vector<int64_t>& dv, const c10::optional<at::Tensor>& bias, bool relu,
              const c10::optional<at::Tensor>& y16, const c10::optional<at::Tensor>& y32,
              const c10::optional<at::Tensor>& omask) {
  const ConvDesc d = desc(dv);
  TORCH_CHECK(X.is_cuda() && X.is_contiguous(), "X must be contiguous CUDA");
  const bool f32 = X.scalar_type() == torch::kFloat32;
  TORCH_CHECK(f32 || X.scalar_type() == torch::kBFloat16, "X must be f32 or bf16");
  check_bf16(W16, "W16");
  TORCH_CHECK(W16.numel() == (int64_t)d.CO * d.KH * d.KW * d.C, "W16 size mismatch");
  rc(mdt_conv_fwd(X.data_ptr(), f32, (const int*)opt_ptr(rows), W16.data_ptr(), d, (const float*)opt_ptr(bias),
                  relu, const_cast<void*>(opt_ptr(y16)), (float*)opt_ptr(y32), opt_ptr(omask), cur()),
     "conv_fwd");
}

void conv_dgrad(const at::Tensor& G16, const c10::optional<at::Tensor>& mask, const at::Tensor& Wt16,
                const std::vector<int64_t>& dv, const c10::optional<at::Tensor>& bias, bool relu,
                const c10::optional<at::Tensor>& y16, const c10::optional<at::Tensor>& y32,
                const c10::optional<at::Tensor>& omask) {
  const ConvDesc d = desc(dv);
  check_bf16(G16, "G16");
  check_bf16(Wt16, "Wt16");
  TORCH_CHECK(G16.numel() >= (int64_t)d.N * d.OH * d.OW * d.CO, "G16 too small");
  rc(mdt_conv_dgrad(G16.data_ptr(), opt_ptr(mask), Wt16.data_ptr(), d, (const float*)opt_ptr(bias), relu,
                    const_cast<void*>(opt_ptr(y16)), (float*)opt_ptr(y32), opt_ptr(omask), cur()),
     "conv_dgrad");
}

void conv_wgrad(const at::Tensor& G16, const c10::optional<at::Tensor>& mask, const at::Tensor& X,
                const c10::optional<at::Tensor>& rows, const std::vector<int64_t>& dv, at::Tensor dW,
                const c10::optional<at::Tensor>& db) {
  const ConvDesc d = desc(dv);
  check_bf16(G16, "G16");
  const bool f32 = X.scalar_type() == torch::kFloat32;
  TORCH_CHECK(dW.scalar_type() == torch::kFloat32 && dW.numel() == (int64_t)d.CO * d.KH * d.KW * d.C,
              "dW must be f32 [CO*KH*KW*C]");
  rc(mdt_conv_wgrad(G16.data_ptr(), opt_ptr(mask), X.data_ptr(), f32, (const int*)opt_ptr(rows), d,
                    dW.data_ptr<float>(), (float*)opt_ptr(db), cur()),
     "conv_wgrad");
}

void chan_sum(const at::Tensor& G16, int64_t M, int64_t C, at::Tensor db) {
  check_bf16(G16, "G16");
  rc(mdt_chan_sum(G16.data_ptr(), (int)M, (int)C, db.data_ptr<float>(), cur()), "chan_sum");
}

void reparam(const at::Tensor& mulv, at::Tensor eps, at::Tensor z16, const c10::optional<at::Tensor>& z32, int64_t B,
             int64_t Z, const at::Tensor& state, const at::Tensor& hparams, int64_t stream, at::Tensor kld_part) {
  rc(mdt_reparam(mulv.data_ptr<float>(), eps.data_ptr<float>(), z16.data_ptr(), (float*)opt_ptr(z32), (int)B, (int)Z,
                 state.data_ptr(), hparams.data_ptr(), (unsigned)stream, kld_part.data_ptr<float>(), cur()),
     "reparam");
}

void reparam_bwd(const at::Tensor& dz, const at::Tensor& mulv, const at::Tensor& eps, at::Tensor dmulv,
                 const c10::optional<at::Tensor>& dmulv16, int64_t B, int64_t Z, const at::Tensor& hparams) {
  rc(mdt_reparam_bwd(dz.data_ptr<float>(), mulv.data_ptr<float>(), eps.data_ptr<float>(), dmulv.data_ptr<float>(),
                     const_cast<void*>(opt_ptr(dmulv16)), (int)B, (int)Z, hparams.data_ptr(), cur()),
     "reparam_bwd");
}

void gather_rows(const at::Tensor& X, const at::Tensor& idx, const at::Tensor& state, int64_t B, int64_t M,
                 at::Tensor xb) {
  TORCH_CHECK(X.scalar_type() == torch::kFloat32 && idx.scalar_type() == torch::kInt32, "gather_rows dtypes");
  rc(mdt_gather_rows(X.data_ptr<float>(), idx.data_ptr<int32_t>(), state.data_ptr(), (int)B, (int)M,
                     (int)X.size(1), xb.data_ptr<float>(), cur()),
     "gather_rows");
}

void bce_logits(const at::Tensor& logits, const at::Tensor& X, const c10::optional<at::Tensor>& rows, int64_t B,
                int64_t P, const c10::optional<at::Tensor>& dlog16, const c10::optional<at::Tensor>& recon,
                at::Tensor part) {
  rc(mdt_bce_logits(logits.data_ptr<float>(), X.data_ptr<float>(), (const int*)opt_ptr(rows), (int)B, (int)P,
                    const_cast<void*>(opt_ptr(dlog16)), (float*)opt_ptr(recon), part.data_ptr<float>(), cur()),
     "bce_logits");
}

void loss_finalize2(const at::Tensor& bce_part, int64_t nb, const at::Tensor& kld_part, int64_t nk, at::Tensor state,
                    const at::Tensor& hparams, bool advance_cursor) {
  rc(mdt_conv_loss_finalize(bce_part.data_ptr<float>(), (int)nb, kld_part.data_ptr<float>(), (int)nk,
                            state.data_ptr(), hparams.data_ptr(), advance_cursor ? 1 : 0, cur()),
     "loss_finalize");
}

void step_begin(at::Tensor state, const at::Tensor& hparams) {
  rc(mdt_step_begin(state.data_ptr(), hparams.data_ptr(), cur()), "step_begin");
}

at::Tensor make_adam_segs(const std::vector<std::vector<int64_t>>& segs, int64_t device_index) {
  std::vector<AdamSeg> v;
  for (auto& s : segs) {
    TORCH_CHECK(s.size() == 6, "segment = (off, numel, co, taps, ci, toff)");
    v.push_back(AdamSeg{s[0], s[1], (int)s[2], (int)s[3], (int)s[4], s[5]});
  }
  auto cpu = torch::empty({(int64_t)(v.size() * sizeof(AdamSeg))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), v.data(), v.size() * sizeof(AdamSeg));
  return cpu.to(torch::Device(torch::kCUDA, device_index));
}

void adam_cast(at::Tensor P, const at::Tensor& G, at::Tensor M, at::Tensor V, at::Tensor w16, at::Tensor w16t,
               const at::Tensor& segs, int64_t nseg, const at::Tensor& state, const at::Tensor& hparams,
               bool do_adam) {
  rc(mdt_adam_cast(P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(),
                   w16.data_ptr(), w16t.data_ptr(), segs.data_ptr(), (int)nseg, P.numel(), state.data_ptr(),
                   hparams.data_ptr(), do_adam ? 1 : 0, cur()),
     "adam_cast");
}

// ------------------------------------------------------------------ state ----
class TrialStateBuf {
 public:
  TrialStateBuf(int64_t device_index) : dev_(device_index) {
    auto bopt = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, device_index);
    train_state = torch::zeros({(int64_t)((sizeof(TrainState) + 63) / 64 * 64)}, bopt);
    eval_state = torch::zeros_like(train_state);
    hparams = torch::zeros({(int64_t)((sizeof(HParams) + 63) / 64 * 64)}, bopt);
    set_hparams(1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, 1.0, 0, false);
  }
  void set_hparams(double lr, double b1, double b2, double eps, double wd, double kl_beta, double gs, int64_t seed,
                   bool decoupled) {
    HParams h;
    std::memset(&h, 0, sizeof(h));
    h.lr = (float)lr; h.beta1 = (float)b1; h.beta2 = (float)b2; h.eps = (float)eps; h.weight_decay = (float)wd;
    h.kl_beta = (float)kl_beta; h.grad_scale = (float)gs; h.decoupled_wd = decoupled ? 1 : 0;
    h.seed_lo = (uint32_t)((uint64_t)seed & 0xffffffffu); h.seed_hi = (uint32_t)((uint64_t)seed >> 32);
    h.lr_d = lr; h.beta1_d = b1; h.beta2_d = b2;
    const bool changed = b1 != b1_ || b2 != b2_;
    b1_ = b1; b2_ = b2;
    auto cpu = torch::empty({(int64_t)sizeof(HParams)}, torch::kUInt8);
    std::memcpy(cpu.data_ptr(), &h, sizeof(h));
    hparams.narrow(0, 0, sizeof(HParams)).copy_(cpu);
    if (changed) {
      pows(train_state, (int64_t)read_state(false)[0]);
      pows(eval_state, (int64_t)read_state(true)[0]);
    }
  }
  void set_cursor(bool eval, int64_t cursor, int64_t nbatches) {
    int32_t v[2] = {(int32_t)cursor, (int32_t)nbatches};
    auto cpu = torch::empty({8}, torch::kUInt8);
    std::memcpy(cpu.data_ptr(), v, 8);
    (eval ? eval_state : train_state).narrow(0, offsetof(TrainState, cursor), 8).copy_(cpu);
  }
  void set_step(bool eval, int64_t step) {
    auto cpu = torch::empty({8}, torch::kUInt8);
    std::memcpy(cpu.data_ptr(), &step, 8);
    at::Tensor& s = eval ? eval_state : train_state;
    s.narrow(0, offsetof(TrainState, step), 8).copy_(cpu);
    pows(s, step);
  }
  void reset_loss(bool eval) { (eval ? eval_state : train_state).narrow(0, offsetof(TrainState, epoch_loss), 16).zero_(); }
  std::vector<double> read_state(bool eval) {
    auto cpu = (eval ? eval_state : train_state).narrow(0, 0, offsetof(TrainState, loss_hist)).to(torch::kCPU);
    TrainState h;
    std::memcpy(&h, cpu.data_ptr(), offsetof(TrainState, loss_hist));
    return {(double)h.step, (double)h.cursor, (double)h.nbatches, h.epoch_loss, h.epoch_count};
  }
  at::Tensor loss_history(bool eval) {
    return (eval ? eval_state : train_state)
        .narrow(0, offsetof(TrainState, loss_hist), sizeof(float) * kLossHist)
        .to(torch::kCPU)
        .view(torch::kFloat32);
  }
  at::Tensor train_state, eval_state, hparams;

 private:
  void pows(at::Tensor& s, int64_t step) {
    double v[2] = {std::pow(b1_, (double)step), std::pow(b2_, (double)step)};
    auto cpu = torch::empty({16}, torch::kUInt8);
    std::memcpy(cpu.data_ptr(), v, 16);
    s.narrow(0, offsetof(TrainState, b1pow), 16).copy_(cpu);
  }
  int64_t dev_;
  double b1_ = -1, b2_ = -1;
};

void bind_conv(pybind11::module& m) {
  namespace py = pybind11;
  m.def("conv_fwd", &conv_fwd, py::arg("X"), py::arg("rows"), py::arg("W16"), py::arg("desc"), py::arg("bias"),
        py::arg("relu"), py::arg("y16"), py::arg("y32"), py::arg("omask") = py::none());
  m.def("conv_dgrad", &conv_dgrad, py::arg("G16"), py::arg("mask"), py::arg("Wt16"), py::arg("desc"),
        py::arg("bias"), py::arg("relu"), py::arg("y16"), py::arg("y32"), py::arg("omask") = py::none());
  m.def("gather_rows", &gather_rows);
  m.def("conv_wgrad", &conv_wgrad, py::arg("G16"), py::arg("mask"), py::arg("X"), py::arg("rows"), py::arg("desc"),
        py::arg("dW"), py::arg("db"));
  m.def("chan_sum", &chan_sum);
  m.def("reparam", &reparam);
  m.def("reparam_bwd", &reparam_bwd);
  m.def("bce_logits", &bce_logits);
  m.def("loss_finalize2", &loss_finalize2);
  m.def("step_begin", &step_begin);
  m.def("make_adam_segs", &make_adam_segs);
  m.def("adam_cast", &adam_cast);
  py::class_<TrialStateBuf>(m, "TrialState")
      .def(py::init<int64_t>())
      .def("set_hparams", &TrialStateBuf::set_hparams)
      .def("set_cursor", &TrialStateBuf::set_cursor)
      .def("set_step", &TrialStateBuf::set_step)
      .def("reset_loss", &TrialStateBuf::reset_loss)
      .def("read_state", &TrialStateBuf::read_state)
      .def("loss_history", &TrialStateBuf::loss_history)
      .def_readonly("train_state", &TrialStateBuf::train_state)
      .def_readonly("eval_state", &TrialStateBuf::eval_state)
      .def_readonly("hparams", &TrialStateBuf::hparams);
}

}  // namespace mdt
