// Native CPU training step of the reference MLP-VAE (BASELINE config #1:
// world 2 on CPU/gloo, two trials of one rank each).
//
// The reference's step (/root/reference/vae-hpo.py:67-74) is eager torch:
// nn.Linear forward, autograd backward, F.binary_cross_entropy, foreach Adam
// -- ~60 ATen calls per step, a dozen full passes over the 128x784 logits and
// seven over the 652,824-parameter arena in Adam. Here the GEMMs stay on
// torch's BLAS (at::addmm_out / at::mm_out into preallocated buffers and
// straight into the flat gradient arena's views), and everything between them
// is fused into one parallel loop per stage on torch's intra-op thread pool:
//   gather rows -> [GEMM fc1 + bias] -> ReLU | [GEMM fc21|fc22] ->
//   reparam (Philox eps, exp, KLD) -> [GEMM fc3] -> ReLU | [GEMM fc4] ->
//   BCE-with-logits (the reference's -100 log clamp) + dlogits in ONE pass |
//   backward GEMMs with the ReLU masks and bias column sums fused |
//   Adam over the whole arena in ONE pass (torch.optim.Adam arithmetic).
// The noise is the same counter-based Philox4x32-10 draw as the GPU kernels
// (csrc/kernels/common.h) and ops/philox.py, keyed by (seed, stream, step).
#include <torch/extension.h>
#include <ATen/Parallel.h>

#include <cmath>
#include <cstdint>
#include <vector>

namespace mdt {

// cpu_mlp_bce.cpp: BCE-with-logits (clamped) sum of one row; t <- sigmoid(t) - x
float bce_dlogits_row(float* t, const float* x, int64_t n);

namespace {

struct Ph { uint32_t x, y, z, w; };

inline Ph philox10(Ph c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32), lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = Ph{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

inline float normal_bits(uint32_t a, uint32_t b) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;
  const float u2 = (float)b * 2.3283064365386963e-10f;
  return std::sqrt(-2.0f * std::log(u1)) * std::cos(6.283185307179586f * u2);
}


}  // namespace

class MlpCpuStep {
 public:
  MlpCpuStep(int64_t B, int64_t D, int64_t H, int64_t Z) : B_(B), D_(D), H_(H), Z_(Z) {
    auto f = torch::TensorOptions().dtype(torch::kFloat32);
    x_ = torch::empty({B, D}, f);
    h1_ = torch::empty({B, H}, f);
    mulv_ = torch::empty({B, 2 * Z}, f);
    eps_ = torch::empty({B, Z}, f);
    z_ = torch::empty({B, Z}, f);
    h3_ = torch::empty({B, H}, f);
    t_ = torch::empty({B, D}, f);
    dh3_ = torch::empty({B, H}, f);
    dz_ = torch::empty({B, Z}, f);
    dmulv_ = torch::empty({B, 2 * Z}, f);
    dh1_ = torch::empty({B, H}, f);
    b2_ = torch::empty({2 * Z}, f);
  }

  // Forward + loss + backward of M rows X[idx[row0 + i]]; gradients into the
  // arena views. Returns the loss (BCE sum + beta * KLD).
  double forward_backward(const std::vector<at::Tensor>& w, std::vector<at::Tensor> g, const at::Tensor& X,
                          const at::Tensor& idx, int64_t row0, int64_t M, int64_t seed, int64_t stream, int64_t step,
                          double beta, bool backward) {
    TORCH_CHECK(w.size() == 10 && g.size() == 10, "weights/grads: fc1.w fc1.b fc21.w fc21.b fc22.w fc22.b fc3.w fc3.b fc4.w fc4.b");
    TORCH_CHECK(M >= 1 && M <= B_ && X.dim() == 2 && X.size(1) == D_ && X.scalar_type() == torch::kFloat32 &&
                X.is_contiguous() && idx.scalar_type() == torch::kInt32 && row0 >= 0 && row0 + M <= idx.numel(),
                "MlpCpuStep: bad batch");
    const int64_t D = D_, H = H_, Z = Z_;
    auto x = x_.narrow(0, 0, M), h1 = h1_.narrow(0, 0, M), mulv = mulv_.narrow(0, 0, M), z = z_.narrow(0, 0, M);
    auto h3 = h3_.narrow(0, 0, M), t = t_.narrow(0, 0, M), dh3 = dh3_.narrow(0, 0, M), dz = dz_.narrow(0, 0, M);
    auto dmulv = dmulv_.narrow(0, 0, M), dh1 = dh1_.narrow(0, 0, M);
    // W2 = [W21; W22] is one contiguous [2Z][H] block of the arena (layout invariant)
    TORCH_CHECK(w[4].data_ptr<float>() == w[2].data_ptr<float>() + Z * H, "fc21/fc22 weights must be adjacent");
    auto W2 = w[2].as_strided({2 * Z, H}, {H, 1}, w[2].storage_offset());
    auto G2 = g[2].as_strided({2 * Z, H}, {H, 1}, g[2].storage_offset());
    TORCH_CHECK(g[4].data_ptr<float>() == g[2].data_ptr<float>() + Z * H, "fc21/fc22 grads must be adjacent");
    b2_.narrow(0, 0, Z).copy_(w[3]);
    b2_.narrow(0, Z, Z).copy_(w[5]);

    const float* Xp = X.data_ptr<float>();
    const int* ip = idx.data_ptr<int>() + row0;
    float* xp = x.data_ptr<float>();
    at::parallel_for(0, M, 8, [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i) std::memcpy(xp + i * D, Xp + (int64_t)ip[i] * D, D * sizeof(float));
    });
    at::addmm_out(h1, w[1], x, w[0].t());
    relu_(h1);
    at::addmm_out(mulv, b2_, h1, W2.t());
    // reparameterisation + KLD
    const float* mv = mulv.data_ptr<float>();
    float* ep = eps_.data_ptr<float>();
    float* zp = z.data_ptr<float>();
    const uint32_t slo = (uint32_t)((uint64_t)step & 0xffffffffu), shi = (uint32_t)((uint64_t)step >> 32);
    const uint32_t k0 = (uint32_t)((uint64_t)seed & 0xffffffffu), k1 = (uint32_t)((uint64_t)seed >> 32);
    double kld = 0.0;
    for (int64_t i = 0; i < M; ++i) {
      for (int64_t c = 0; c < Z; ++c) {
        const Ph r = philox10(Ph{(uint32_t)(i * Z + c), (uint32_t)stream, slo, shi}, k0, k1);
        const float e = normal_bits(r.x, r.y);
        const float mu = mv[i * 2 * Z + c], lv = mv[i * 2 * Z + Z + c];
        const float sd = std::exp(0.5f * lv);
        ep[i * Z + c] = e;
        zp[i * Z + c] = mu + e * sd;
        kld += (double)(1.f + lv - mu * mu - sd * sd);
      }
    }
    kld *= -0.5;
    at::addmm_out(h3, w[7], z, w[6].t());
    relu_(h3);
    at::addmm_out(t, w[9], h3, w[8].t());
    // BCE with the reference's log clamp (F.binary_cross_entropy: log >= -100) + dlogits, one pass
    // (cpu_mlp_bce.cpp: the only fast-math translation unit, for vectorised exp/log)
    float* tp = t.data_ptr<float>();
    std::vector<double> part((size_t)at::get_num_threads() + 1, 0.0);
    at::parallel_for(0, M, 4, [&](int64_t a, int64_t b) {
      double s = 0.0;
      for (int64_t i = a; i < b; ++i) s += bce_dlogits_row(tp + i * D, xp + i * D, D);
      part[(size_t)at::get_thread_num()] += s;
    });
    double bce = 0.0;
    for (double v : part) bce += v;
    last_m_ = M;
    if (!backward) return bce + beta * kld;  // eval: forward + loss only (recon(): sigmoid(t) = t + x)
    // backward (t now holds dlogits)
    at::mm_out(g[8], t.t(), h3);
    at::sum_out(g[9], t, {0});
    at::mm_out(dh3, t, w[8]);
    mask_(dh3, h3);
    at::mm_out(g[6], dh3.t(), z);
    at::sum_out(g[7], dh3, {0});
    at::mm_out(dz, dh3, w[6]);
    const float* dzp = dz.data_ptr<float>();
    float* dm = dmulv.data_ptr<float>();
    const float fb = (float)beta;
    for (int64_t i = 0; i < M; ++i) {
      for (int64_t c = 0; c < Z; ++c) {
        const float mu = mv[i * 2 * Z + c], sd = std::exp(0.5f * mv[i * 2 * Z + Z + c]);
        const float d = dzp[i * Z + c];
        dm[i * 2 * Z + c] = d + fb * mu;
        dm[i * 2 * Z + Z + c] = 0.5f * d * ep[i * Z + c] * sd + 0.5f * fb * (sd * sd - 1.f);
      }
    }
    at::mm_out(G2, dmulv.t(), h1);
    auto gb2 = dmulv.sum(0);
    g[3].copy_(gb2.narrow(0, 0, Z));
    g[5].copy_(gb2.narrow(0, Z, Z));
    at::mm_out(dh1, dmulv, W2);
    mask_(dh1, h1);
    at::mm_out(g[0], dh1.t(), x);
    at::sum_out(g[1], dh1, {0});
    return bce + beta * kld;
  }

  // sigmoid(logits) of the last batch (the loss pass left dlogits = p - x in t)
  at::Tensor recon() const { return t_.narrow(0, 0, last_m_) + x_.narrow(0, 0, last_m_); }

  // torch.optim.Adam (Adam / AdamW) over the whole flat arena in one pass;
  // step is the 1-based t. Padding between parameters is zero and stays zero.
  static void adam(at::Tensor P, const at::Tensor& G, at::Tensor Mo, at::Tensor Vo, int64_t step, double lr,
                   double beta1, double beta2, double eps, double wd, double gs, bool decoupled) {
    TORCH_CHECK(P.is_contiguous() && G.is_contiguous() && Mo.is_contiguous() && Vo.is_contiguous() &&
                    G.numel() == P.numel() && Mo.numel() == P.numel() && Vo.numel() == P.numel(),
                "adam: flat contiguous arenas of one size");
    float* p = P.data_ptr<float>();
    const float* g = G.data_ptr<float>();
    float* m = Mo.data_ptr<float>();
    float* v = Vo.data_ptr<float>();
    const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
    const float step_size = (float)(lr / bc1), bc2s = (float)std::sqrt(bc2);
    const float b1 = (float)beta1, b2 = (float)beta2, fe = (float)eps, fwd = (float)wd, fgs = (float)gs;
    const float decay = (float)(1.0 - lr * wd);
    at::parallel_for(0, P.numel(), 16384, [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i) {
        float gr = g[i] * fgs;
        float pi = p[i];
        if (fwd != 0.f) {
          if (decoupled) pi *= decay;
          else gr += fwd * pi;
        }
        const float mi = m[i] + (1.f - b1) * (gr - m[i]);
        const float vi = v[i] * b2 + (1.f - b2) * gr * gr;
        m[i] = mi;
        v[i] = vi;
        p[i] = pi - step_size * (mi / (std::sqrt(vi) / bc2s + fe));
      }
    });
  }

 private:
  static void relu_(at::Tensor& a) {
    float* p = a.data_ptr<float>();
    at::parallel_for(0, a.numel(), 32768, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) p[i] = p[i] > 0.f ? p[i] : 0.f;
    });
  }
  static void mask_(at::Tensor& d, const at::Tensor& act) {
    float* p = d.data_ptr<float>();
    const float* q = act.data_ptr<float>();
    at::parallel_for(0, d.numel(), 32768, [&](int64_t lo, int64_t hi) {
      for (int64_t i = lo; i < hi; ++i) p[i] = q[i] > 0.f ? p[i] : 0.f;
    });
  }

  int64_t B_, D_, H_, Z_, last_m_ = 0;
  at::Tensor x_, h1_, mulv_, eps_, z_, h3_, t_, dh3_, dz_, dmulv_, dh1_, b2_;
};

void bind_cpu(pybind11::module& m) {
  namespace py = pybind11;
  py::class_<MlpCpuStep>(m, "MlpCpuStep")
      .def(py::init<int64_t, int64_t, int64_t, int64_t>(), py::arg("B"), py::arg("D"), py::arg("H"), py::arg("Z"))
      .def("forward_backward", &MlpCpuStep::forward_backward, py::arg("weights"), py::arg("grads"), py::arg("X"),
           py::arg("idx"), py::arg("row0"), py::arg("M"), py::arg("seed"), py::arg("stream"), py::arg("step"),
           py::arg("beta"), py::arg("backward") = true, py::call_guard<py::gil_scoped_release>())
      .def("recon", &MlpCpuStep::recon)
      .def_static("adam", &MlpCpuStep::adam, py::arg("P"), py::arg("G"), py::arg("M"), py::arg("V"), py::arg("step"),
                  py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"),
                  py::arg("grad_scale"), py::arg("decoupled"), py::call_guard<py::gil_scoped_release>());
}

}  // namespace mdt
