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

#include "../kernels/conv_igemm.h"

extern "C" {
int mdt_igemm_plan(int mode, mdt::ConvDesc d, int allow_split, int* info, int fwd);
void mdt_dconv_stamps(unsigned long long* p);
int mdt_wgrad_plan(mdt::ConvDesc d, int* info);
int mdt_igemm(int mode, const void* A, int a_is_f32, const void* B16, mdt::ConvDesc d, const float* bias, int relu,
              void* y16, float* y32, const void* omask, float* colsum, float* ws, int skip_combine, hipStream_t s,
              const mdt::APro* pro, int fwd);
int mdt_wgrad(const void* G16, const void* X, int x_is_f32, mdt::ConvDesc d, float* out, hipStream_t s);
int mdt_colsum(const void* G16, int M, int N, int rows_per, float* slab, hipStream_t s);
int mdt_gather_rows(const float* X, const int* idx, const void* st, int B, int M, int P, float* xb, hipStream_t s);
int mdt_reparam(const float* mulv, float* eps, void* z16, float* z32, int B, int Z, const void* st, const void* hp,
                unsigned stream, float* kld_part, hipStream_t s);
int mdt_reparam_bwd(const float* dz, const float* mulv, const float* eps, float* dmulv, void* dmulv16, int B, int Z,
                    const void* hp, hipStream_t s);
int mdt_bce_logits(const float* logits, const float* X, const int* rows, int B, int P, void* dlog16, float* recon,
                   float* part, float* gpart, hipStream_t s);
int mdt_conv_loss_finalize(const float* bce_part, int nb, const float* kld_part, int nk, void* st, const void* hp,
                           int advance_cursor, hipStream_t s);
int mdt_step_begin(void* st, const void* hp, hipStream_t s);
int mdt_adam_cast(float* P, const float* G, float* Mo, float* Vo, void* w16, const void* segs, int nseg,
                  long long total, const void* st, const void* hp, int do_adam, hipStream_t s);
int mdt_grad_finalize(float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs, const void* units,
                      int nunits, const void* st, const void* hp, int do_adam, const float* gX, const int* gidx,
                      float* xn, unsigned* xtag, int gB, hipStream_t s);
int mdt_wtrans(const void* w16, void* w16t, const void* segs, const void* units, int nunits, hipStream_t s);
int mdt_thin_conv(const void* X, int x_is_f32, const float* Wf, mdt::ConvDesc d, const float* bias, int relu, void* y16,
                  const void* omask, float* colsum, const int* idx, void* st, const void* hp, int B, float* xb,
                  hipStream_t s);
int mdt_thin_blocks(int tconv, mdt::ConvDesc d);
int mdt_thin_tconv(const void* G16, const float* Wf, mdt::ConvDesc d, const float* bias, float* y32, const float* X,
                   void* dlog16, float* recon, float* part, float* gpart, hipStream_t s);
int mdt_job_igemm(mdt::JobBlob* g, mdt::JobBlob* c, int mode, const void* A, int a_is_f32, const void* B16,
                  mdt::ConvDesc d, const float* bias, int relu, void* y16, float* y32, const void* omask,
                  float* colsum, float* ws, int skip_combine);
int mdt_job_finalize(mdt::JobBlob* j, float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs,
                     const void* units, int nunits, const void* st, const void* hp, int do_adam, int dep);
int mdt_job_gather(mdt::JobBlob* j, const float* X, const int* idx, const void* st, float* xn, unsigned* xtag, int B);
int mdt_jobs_dep_words();
int mdt_jobs_dep_err();
int mdt_pack_jobs_multi_deps(void* img, void* ctr, const unsigned* wait, int n);
int mdt_job_wtrans(mdt::JobBlob* j, const void* w16, void* w16t, const void* segs, const void* units, int nunits);
int mdt_job_comm(mdt::JobBlob* j, float* P, float* G, float* Mo, float* Vo, void* w16, const void* segs,
                 const void* units, int nunits, const void* st, const void* hp, int do_adam, const void* ctx, int mode);
int mdt_combine_reparam(const float* slab, int ks, const float* bias, float* mulv, float* eps, void* z16, float* z32,
                        int B, int Z, const void* st, const void* hp, unsigned stream, float* kld_part, hipStream_t s);
int mdt_combine_reparam_blocks(int ks, int B, int Z);
int mdt_combine_reparam_bwd(const float* slab, int ks, const float* mulv, const float* eps, float* dmulv,
                            void* dmulv16, float* dz, int B, int Z, const void* hp, hipStream_t s);
int mdt_job_wgrad(mdt::JobBlob* j, const void* G16, const void* X, int x_is_f32, mdt::ConvDesc d, float* out);
int mdt_job_thin_conv(mdt::JobBlob* j, const void* X, int x_is_f32, const float* Wf, mdt::ConvDesc d,
                      const float* bias, int relu, void* y16, const void* omask, float* colsum, const int* idx,
                      void* st, const void* hp, int B, float* xb);
int mdt_job_colsum(mdt::JobBlob* j, const void* G16, int M, int N, int rows_per, float* slab);
int mdt_job_loss(mdt::JobBlob* j, const float* bce_part, int nb, const float* kld_part, int nk, void* st,
                 const void* hp, int advance_cursor);
int mdt_launch_jobs(const mdt::JobBlob* jobs, int n, hipStream_t s);
int mdt_jobs_multi_bytes();
int mdt_pack_jobs_multi(const mdt::JobBlob* jobs, int n, void* dst);
int mdt_pack_jobs_multi_stamps(void* img, void* stamps);
int mdt_launch_jobs_multi(const void* dev_pack, int grid, int dep, hipStream_t s);
int mdt_f28_forward(const long long* p, int B, int M, unsigned stream, int train, hipStream_t s);
int mdt_f28_forward_pair(const long long* p, const long long* pp, int B, int M, unsigned stream, hipStream_t s);
int mdt_f28_backward(const long long* p, int M, hipStream_t s);
int mdt_f28_step(const long long* pf, const long long* pb, const long long* pp, int B, int M, unsigned stream,
                 int pair, int delay_us, hipStream_t s);
int mdt_f28_pair_words();
int mdt_launch_job1(const mdt::JobBlob* j, hipStream_t s);
}

namespace mdt {

// A recorded launch for the horizontally fused job kernels (conv_jobs.hip):
// the op bindings below take an optional Job; when given, they validate and
// RECORD the launch into it instead of issuing it. `post` is the dependent
// follow-up (split-K combine) to launch after the job's own kernel.
struct Job {
  JobBlob main{}, post{};
  int kind() const { return main.kind; }
  bool has_post() const { return post.kind != 0; }
};

static hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }
static void rc(int r, const char* w) { TORCH_CHECK(r == 0, "mdt: ", w, " failed (", r, ")"); }
static const void* opt_ptr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

static ConvDesc desc(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 11, "conv desc needs 11 ints (N,H,W,C,OH,OW,CO,KH,KW,S,P)");
  for (auto x : v) TORCH_CHECK(x >= 0 && x < (1 << 30), "conv desc value out of range");
  return ConvDesc{(int)v[0], (int)v[1], (int)v[2], (int)v[3], (int)v[4], (int)v[5],
                  (int)v[6], (int)v[7], (int)v[8], (int)v[9], (int)v[10]};
}

static void check_bf16(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kBFloat16 && t.is_contiguous(), n,
              " must be a contiguous CUDA bfloat16 tensor");
}
static void check_f32(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous(), n,
              " must be a contiguous CUDA float32 tensor");
}
static void check_min(const c10::optional<at::Tensor>& t, int64_t n, const char* w) {
  if (t.has_value() && t->defined()) TORCH_CHECK(t->numel() >= n, w, " too small: ", t->numel(), " < ", n);
}

// fwd: the forward-pass call of this geometry (may select the direct kernel
// where the backward-data call of the same geometry keeps the fusable one)
std::vector<int64_t> igemm_plan(int64_t mode, const std::vector<int64_t>& dv, bool allow_split, bool fwd) {
  int info[12];
  rc(mdt_igemm_plan((int)mode, desc(dv), allow_split ? 1 : 0, info, fwd ? 1 : 0), "igemm_plan (unsupported geometry)");
  return std::vector<int64_t>(info, info + 12);
}

std::vector<int64_t> wgrad_plan(const std::vector<int64_t>& dv) {
  int info[8];
  rc(mdt_wgrad_plan(desc(dv), info), "wgrad_plan (unsupported geometry)");
  return std::vector<int64_t>(info, info + 8);
}

// mode 0: conv (fwd / convT bwd-data), mode 1: parity-class transposed conv
// (conv bwd-data / convT fwd; B16 = parity-ordered transposed weights).
void igemm(int64_t mode, const at::Tensor& A, const at::Tensor& B16, const std::vector<int64_t>& dv,
           const c10::optional<at::Tensor>& bias, bool relu, const c10::optional<at::Tensor>& y16,
           const c10::optional<at::Tensor>& y32, const c10::optional<at::Tensor>& omask,
           const c10::optional<at::Tensor>& colsum, const c10::optional<at::Tensor>& ws, Job* job, bool combine,
           const c10::optional<at::Tensor>& a_slab, int64_t a_ks, const c10::optional<at::Tensor>& a_bias,
           bool a_relu, const c10::optional<at::Tensor>& a_out16, bool fwd) {
  const ConvDesc d = desc(dv);
  TORCH_CHECK(A.is_cuda() && A.is_contiguous(), "A must be contiguous CUDA");
  const bool f32 = A.scalar_type() == torch::kFloat32;
  TORCH_CHECK(f32 || A.scalar_type() == torch::kBFloat16, "A must be f32 or bf16");
  check_bf16(B16, "B16");
  int info[12];
  rc(mdt_igemm_plan((int)mode, d, ws.has_value() && ws->defined() ? 1 : 0, info, fwd ? 1 : 0), "igemm_plan");
  TORCH_CHECK(!(fwd && job), "igemm: fwd calls have no job form");
  const int64_t classes = info[3], M = info[4], Ncols = info[5], K = info[6], ksplit = info[10];
  const int64_t rows_total = classes * M;
  const int64_t a_need = mode == kModeConv ? (int64_t)d.N * d.H * d.W * d.C : (int64_t)d.N * d.OH * d.OW * d.CO;
  TORCH_CHECK(A.numel() >= a_need, "A too small: ", A.numel(), " < ", a_need);
  TORCH_CHECK(B16.numel() >= classes * Ncols * K, "B16 too small");
  check_min(y16, rows_total * Ncols, "y16");
  check_min(y32, rows_total * Ncols, "y32");
  check_min(omask, rows_total * Ncols, "omask");
  check_min(bias, Ncols, "bias");
  check_min(colsum, (int64_t)info[11] * Ncols, "colsum");
  if (ksplit > 1) check_min(ws, ksplit * M * Ncols, "ws");
  APro pro{};
  if (a_slab.has_value() && a_slab->defined()) {
    // A is formed from the producing layer's split-K partial slabs (see APro)
    TORCH_CHECK(!job, "igemm: the A prologue has no job form");
    TORCH_CHECK(a_bias.has_value() && a_bias->defined() && a_out16.has_value() && a_out16->defined(),
                "igemm: a_slab needs a_bias and a_out16");
    check_f32(*a_slab, "a_slab");
    check_bf16(*a_out16, "a_out16");
    TORCH_CHECK(a_ks >= 1 && a_slab->numel() >= a_ks * a_need, "a_slab too small");
    TORCH_CHECK(a_out16->numel() >= a_need, "a_out16 too small");
    const int64_t cin = a_bias->numel();
    TORCH_CHECK(cin % 8 == 0 && a_need % cin == 0, "a_bias length must divide the A row layout");
    pro = APro{(const float*)a_slab->data_ptr(), (const float*)a_bias->data_ptr(),
               a_out16->data_ptr(), (int)a_ks, a_relu ? 1 : 0, (int)cin, (long long)a_need};
  }
  if (job) {
    rc(mdt_job_igemm(&job->main, &job->post, (int)mode, A.data_ptr(), f32, B16.data_ptr(), d,
                     (const float*)opt_ptr(bias), relu, const_cast<void*>(opt_ptr(y16)), (float*)opt_ptr(y32),
                     opt_ptr(omask), (float*)opt_ptr(colsum), (float*)opt_ptr(ws), combine ? 0 : 1),
       "job_igemm");
    return;
  }
  rc(mdt_igemm((int)mode, A.data_ptr(), f32, B16.data_ptr(), d, (const float*)opt_ptr(bias), relu,
               const_cast<void*>(opt_ptr(y16)), (float*)opt_ptr(y32), opt_ptr(omask), (float*)opt_ptr(colsum),
               (float*)opt_ptr(ws), combine ? 0 : 1, cur(), pro.slab ? &pro : nullptr, fwd ? 1 : 0),
     "igemm");
}

void wgrad(const at::Tensor& G16, const at::Tensor& X, const std::vector<int64_t>& dv, at::Tensor out, Job* job) {
  const ConvDesc d = desc(dv);
  check_bf16(G16, "G16");
  check_f32(out, "out");
  const bool f32 = X.scalar_type() == torch::kFloat32;
  TORCH_CHECK(X.is_cuda() && X.is_contiguous() && (f32 || X.scalar_type() == torch::kBFloat16), "X dtype/layout");
  int info[8];
  rc(mdt_wgrad_plan(d, info), "wgrad_plan");
  TORCH_CHECK(G16.numel() >= (int64_t)d.N * d.OH * d.OW * d.CO, "G16 too small");
  TORCH_CHECK(X.numel() >= (int64_t)d.N * d.H * d.W * d.C, "X too small");
  TORCH_CHECK(out.numel() >= (int64_t)info[6] * d.CO * d.KH * d.KW * d.C, "wgrad out too small for ", info[6],
              " partial slabs");
  if (job) {
    rc(mdt_job_wgrad(&job->main, G16.data_ptr(), X.data_ptr(), f32, d, out.data_ptr<float>()), "job_wgrad");
    return;
  }
  rc(mdt_wgrad(G16.data_ptr(), X.data_ptr(), f32, d, out.data_ptr<float>(), cur()), "wgrad");
}

// Single-channel edge layers (conv_thin.hip): Wf is the f32 master weight
// [CO][KH][KW][1] (read with wave-uniform scalar loads).
void thin_conv(const at::Tensor& X, const at::Tensor& Wf, const std::vector<int64_t>& dv,
               const c10::optional<at::Tensor>& bias, bool relu, at::Tensor y16,
               const c10::optional<at::Tensor>& omask, const c10::optional<at::Tensor>& colsum, Job* job,
               const c10::optional<at::Tensor>& idx, const c10::optional<at::Tensor>& state,
               const c10::optional<at::Tensor>& hparams, int64_t B, const c10::optional<at::Tensor>& xb) {
  const ConvDesc d = desc(dv);
  const bool f32 = X.scalar_type() == torch::kFloat32;
  TORCH_CHECK(X.is_cuda() && X.is_contiguous() && (f32 || X.scalar_type() == torch::kBFloat16), "X dtype/layout");
  check_f32(Wf, "Wf");
  check_bf16(y16, "y16");
  const int64_t M = (int64_t)d.N * d.OH * d.OW;
  TORCH_CHECK(X.numel() >= (int64_t)d.N * d.H * d.W, "X too small");
  TORCH_CHECK(Wf.numel() >= (int64_t)d.CO * d.KH * d.KW, "Wf too small");
  TORCH_CHECK(y16.numel() >= M * d.CO, "y16 too small");
  check_min(omask, M * d.CO, "omask");
  check_min(colsum, (int64_t)mdt_thin_blocks(0, d) * d.CO, "colsum");
  check_min(bias, d.CO, "bias");
  const bool gather = idx.has_value() && idx->defined();
  if (gather) {
    TORCH_CHECK(idx->scalar_type() == torch::kInt32 && state.has_value() && B >= d.N, "thin_conv gather arguments");
    TORCH_CHECK(X.dim() == 2 && X.size(1) == (int64_t)d.H * d.W, "thin_conv gather: X must be [rows, H*W]");
  }
  check_min(xb, (int64_t)d.N * d.H * d.W, "xb");
  if (job) {
    rc(mdt_job_thin_conv(&job->main, X.data_ptr(), f32, Wf.data_ptr<float>(), d, (const float*)opt_ptr(bias), relu,
                         y16.data_ptr(), opt_ptr(omask), (float*)opt_ptr(colsum), (const int*)opt_ptr(idx),
                         const_cast<void*>(opt_ptr(state)), opt_ptr(hparams), (int)B, (float*)opt_ptr(xb)),
       "job_thin_conv");
    return;
  }
  rc(mdt_thin_conv(X.data_ptr(), f32, Wf.data_ptr<float>(), d, (const float*)opt_ptr(bias), relu, y16.data_ptr(),
                   opt_ptr(omask), (float*)opt_ptr(colsum), (const int*)opt_ptr(idx), const_cast<void*>(opt_ptr(state)),
                   opt_ptr(hparams), (int)B, (float*)opt_ptr(xb), cur()),
     "thin_conv");
}

int64_t thin_blocks(bool tconv, const std::vector<int64_t>& dv) { return mdt_thin_blocks(tconv ? 1 : 0, desc(dv)); }

void thin_tconv(const at::Tensor& G16, const at::Tensor& Wf, const std::vector<int64_t>& dv,
                const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& y32,
                const c10::optional<at::Tensor>& X, const c10::optional<at::Tensor>& dlog16,
                const c10::optional<at::Tensor>& recon, const c10::optional<at::Tensor>& part,
                const c10::optional<at::Tensor>& gpart) {
  const ConvDesc d = desc(dv);
  check_bf16(G16, "G16");
  check_f32(Wf, "Wf");
  const int64_t npix = (int64_t)d.N * d.H * d.W;
  const int64_t nb = mdt_thin_blocks(1, d);
  TORCH_CHECK(G16.numel() >= (int64_t)d.N * d.OH * d.OW * d.CO, "G16 too small");
  TORCH_CHECK(Wf.numel() >= (int64_t)d.CO * d.KH * d.KW, "Wf too small");
  check_min(y32, npix, "y32");
  check_min(X, npix, "X");
  check_min(dlog16, npix, "dlog16");
  check_min(recon, npix, "recon");
  check_min(part, nb, "part");
  check_min(gpart, nb, "gpart");
  rc(mdt_thin_tconv(G16.data_ptr(), Wf.data_ptr<float>(), d, (const float*)opt_ptr(bias), (float*)opt_ptr(y32),
                    (const float*)opt_ptr(X), const_cast<void*>(opt_ptr(dlog16)), (float*)opt_ptr(recon),
                    (float*)opt_ptr(part), (float*)opt_ptr(gpart), cur()),
     "thin_tconv");
}

void colsum(const at::Tensor& G16, int64_t M, int64_t N, int64_t rows_per, at::Tensor slab, Job* job) {
  check_bf16(G16, "G16");
  check_f32(slab, "slab");
  TORCH_CHECK(G16.numel() >= M * N, "G16 too small");
  TORCH_CHECK(slab.numel() >= ((M + rows_per - 1) / rows_per) * N, "colsum slab too small");
  if (job) {
    rc(mdt_job_colsum(&job->main, G16.data_ptr(), (int)M, (int)N, (int)rows_per, slab.data_ptr<float>()), "job_colsum");
    return;
  }
  rc(mdt_colsum(G16.data_ptr(), (int)M, (int)N, (int)rows_per, slab.data_ptr<float>(), cur()), "colsum");
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
                at::Tensor part, const c10::optional<at::Tensor>& gpart) {
  rc(mdt_bce_logits(logits.data_ptr<float>(), X.data_ptr<float>(), (const int*)opt_ptr(rows), (int)B, (int)P,
                    const_cast<void*>(opt_ptr(dlog16)), (float*)opt_ptr(recon), part.data_ptr<float>(),
                    (float*)opt_ptr(gpart), cur()),
     "bce_logits");
}

void loss_finalize2(const at::Tensor& bce_part, int64_t nb, const at::Tensor& kld_part, int64_t nk, at::Tensor state,
                    const at::Tensor& hparams, bool advance_cursor, Job* job, bool advance_step) {
  TORCH_CHECK(bce_part.numel() >= nb && kld_part.numel() >= nk, "loss partials too small");
  if (job) {
    rc(mdt_job_loss(&job->main, bce_part.data_ptr<float>(), (int)nb, kld_part.data_ptr<float>(), (int)nk,
                    state.data_ptr(), hparams.data_ptr(), (advance_cursor ? 1 : 0) | (advance_step ? 2 : 0)),
       "job_loss");
    return;
  }
  rc(mdt_conv_loss_finalize(bce_part.data_ptr<float>(), (int)nb, kld_part.data_ptr<float>(), (int)nk,
                            state.data_ptr(), hparams.data_ptr(), (advance_cursor ? 1 : 0) | (advance_step ? 2 : 0),
                            cur()),
     "loss_finalize");
}

// Launch recorded jobs as ONE fused kernel when an instantiation exists for
// their kinds (returns true), else launch nothing and return false (the caller
// then issues the ops' own kernels). Follow-up combines run right after.
bool launch_jobs(const std::vector<Job*>& jobs) {
  TORCH_CHECK(jobs.size() >= 2 && jobs.size() <= 3, "launch_jobs takes 2 or 3 jobs");
  JobBlob v[3];
  for (size_t i = 0; i < jobs.size(); ++i) {
    TORCH_CHECK(jobs[i] != nullptr, "null job");
    v[i] = jobs[i]->main;
  }
  const int r = mdt_launch_jobs(v, (int)jobs.size(), cur());
  TORCH_CHECK(r >= 0 && r != 2, "mdt: launch_jobs failed (", r, ")");
  if (r != 0) return false;
  for (auto* j : jobs)
    if (j->has_post()) rc(mdt_launch_job1(&j->post, cur()), "job follow-up");
  return true;
}

// Pack recorded jobs (any supported kinds, up to 8; up to 16 with `wait`) into
// a job table for ONE jobs_multi_k launch: returns (uint8 CPU tensor image, grid). The caller keeps
// the table in device memory for the lifetime of the plan (graph replays).
std::tuple<at::Tensor, int64_t> pack_jobs_multi(const std::vector<Job*>& jobs,
                                                const c10::optional<at::Tensor>& stamps,
                                                const std::vector<int64_t>& wait,
                                                const c10::optional<at::Tensor>& dep_ctr) {
  TORCH_CHECK(!jobs.empty() && jobs.size() <= (wait.empty() ? 8u : 16u),
              "pack_jobs_multi takes 1..8 jobs (1..16 with a dependency table)");
  std::vector<JobBlob> v;
  for (auto* j : jobs) {
    TORCH_CHECK(j != nullptr && !j->has_post(), "pack_jobs_multi: null job or job with a follow-up pass");
    TORCH_CHECK(j->main.kind > 0, "pack_jobs_multi: job has no fused form (kind 0)");
    v.push_back(j->main);
  }
  auto img = torch::zeros({(int64_t)mdt_jobs_multi_bytes()}, torch::kUInt8);
  const int grid = mdt_pack_jobs_multi(v.data(), (int)v.size(), img.data_ptr());
  TORCH_CHECK(grid > 0, "pack_jobs_multi: unsupported job kind or bad job (", grid, ")");
  if (stamps.has_value() && stamps->defined()) {  // profiling: [grid][2] int64 per-workgroup start / end stamps
    TORCH_CHECK(stamps->is_cuda() && stamps->scalar_type() == torch::kInt64 && stamps->numel() >= 2 * grid,
                "pack_jobs_multi: stamps must be an int64 CUDA tensor of >= 2 * grid elements");
    mdt_pack_jobs_multi_stamps(img.data_ptr(), stamps->data_ptr());
  }
  if (!wait.empty()) {  // in-launch dependencies (conv_jobs.hip JobPackN): wait[i] = bit mask of jobs job i waits for
    TORCH_CHECK(wait.size() == jobs.size(), "pack_jobs_multi: one wait mask per job");
    TORCH_CHECK(dep_ctr.has_value() && dep_ctr->defined() && dep_ctr->is_cuda() &&
                    dep_ctr->scalar_type() == torch::kInt32 && dep_ctr->is_contiguous() &&
                    dep_ctr->numel() >= mdt_jobs_dep_words(),
                "pack_jobs_multi: dep_ctr must be a zeroed contiguous int32 CUDA tensor of >= ",
                mdt_jobs_dep_words(), " words");
    std::vector<unsigned> w(wait.begin(), wait.end());
    TORCH_CHECK(mdt_pack_jobs_multi_deps(img.data_ptr(), dep_ctr->data_ptr(), w.data(), (int)w.size()) == 0,
                "pack_jobs_multi: bad dependency table (a job may wait only for earlier jobs that do not wait)");
  }
  return {img, (int64_t)grid};
}

void launch_jobs_multi(const at::Tensor& dev_pack, int64_t grid, bool dep) {
  TORCH_CHECK(dev_pack.is_cuda() && dev_pack.scalar_type() == torch::kUInt8 &&
                  dev_pack.numel() >= mdt_jobs_multi_bytes(), "launch_jobs_multi: device job table");
  const int r = mdt_launch_jobs_multi(dev_pack.data_ptr(), (int)grid, dep ? 1 : 0, cur());
  TORCH_CHECK(r == 0, "mdt: launch_jobs_multi failed (", r, ")");
}

// Fused 28x28 step launches (conv28_fused.hip). `t` lists the tensors in the
// kernel's pointer-table order (None -> nullptr where optional); every tensor is
// checked for device, contiguity, dtype and minimum size BEFORE the launch, so
// a wrong buffer is a Python error rather than an out-of-bounds access. Not
// checkable here: the gathered rows X[idx[cursor * B + n]] depend on device
// state (the cursor) and on the index VALUES; the trainer guarantees them
// (bind_train_data pads idx to whole batches of in-range rows, set_cursor
// keeps cursor < nbatches), and the checks below pin the shapes they assume.
namespace {
struct Slot {
  const char* name;
  char dtype;        // 'f' f32, 'b' bf16, 'i' int32, 'u' uint8 (state blobs)
  int64_t per_m;     // elements per sample (or fixed count when fixed)
  bool fixed;        // per_m is a fixed element count
  bool optional;
};

std::vector<long long> f28_ptrs(const std::vector<c10::optional<at::Tensor>>& t, const std::vector<Slot>& slots,
                                int64_t M, int dev) {
  TORCH_CHECK(t.size() <= slots.size(), "f28: expected ", slots.size(), " tensors, got ", t.size());
  for (size_t i = t.size(); i < slots.size(); ++i)  // trailing slots left out: must be optional (null)
    TORCH_CHECK(slots[i].optional, "f28: expected ", slots.size(), " tensors, got ", t.size());
  std::vector<long long> p(slots.size(), 0);
  for (size_t i = 0; i < t.size(); ++i) {
    const Slot& s = slots[i];
    if (!t[i].has_value() || !t[i]->defined()) {
      TORCH_CHECK(s.optional, "f28: tensor ", s.name, " is required");
      continue;
    }
    const at::Tensor& x = *t[i];
    TORCH_CHECK(x.is_cuda() && x.device().index() == dev && x.is_contiguous(), "f28: ", s.name,
                " must be a contiguous tensor on cuda:", dev);
    const auto st = x.scalar_type();
    const bool ok = (s.dtype == 'f' && st == torch::kFloat32) || (s.dtype == 'b' && st == torch::kBFloat16) ||
                    (s.dtype == 'i' && st == torch::kInt32) || (s.dtype == 'u' && st == torch::kUInt8) ||
                    (s.dtype == 'l' && st == torch::kInt64);
    TORCH_CHECK(ok, "f28: ", s.name, " has dtype ", st);
    const int64_t need = s.fixed ? s.per_m : s.per_m * M;
    TORCH_CHECK(x.numel() >= need, "f28: ", s.name, " has ", x.numel(), " elements, needs ", need);
    p[i] = (long long)(intptr_t)x.data_ptr();
  }
  return p;
}

const std::vector<Slot>& f28_weight_slots() {
  static const std::vector<Slot> w = {
      {"W1f", 'f', 512, true, false},    {"b1", 'f', 32, true, false},    {"W2", 'b', 32768, true, false},
      {"b2", 'f', 64, true, false},      {"Wh", 'b', 200704, true, false}, {"bh", 'f', 64, true, false},
      {"Wd", 'b', 100352, true, false},  {"bd", 'f', 3136, true, false},  {"W3", 'b', 32768, true, false},
      {"b3", 'f', 32, true, false},      {"W4f", 'f', 512, true, false},  {"b4", 'f', 1, true, false}};
  return w;
}
}  // namespace

std::vector<Slot> f28_fwd_slots(int64_t B, bool train) {
  std::vector<Slot> slots = f28_weight_slots();
  const std::vector<Slot> rest = {
      {"X", 'f', 784, true, false},        {"idx", 'i', B, true, false},
      {"state", 'u', (int64_t)sizeof(TrainState), true, false}, {"hparams", 'u', (int64_t)sizeof(HParams), true, false},
      {"xb", 'f', 784, false, !train},     {"a1", 'b', 6272, false, !train},  {"a2", 'b', 3136, false, !train},
      {"mulv", 'f', 64, false, !train},    {"eps", 'f', 32, false, !train},   {"z16", 'b', 32, false, !train},
      {"d0", 'b', 3136, false, !train},    {"d1", 'b', 6272, false, !train},  {"dlog", 'f', 784, false, !train},
      {"recon", 'f', 784, false, true},    {"bce_part", 'f', 1, false, false}, {"kld_part", 'f', 1, false, false},
      {"db4_part", 'f', 1, false, true},   {"stamps", 'l', 32, false, true},
      {"xn", 'f', 784, false, true},       {"xtag", 'i', 1, false, true}};
  slots.insert(slots.end(), rest.begin(), rest.end());
  return slots;
}

std::vector<Slot> f28_bwd_slots() {
  std::vector<Slot> slots = f28_weight_slots();
  const std::vector<Slot> rest = {
      {"hparams", 'u', (int64_t)sizeof(HParams), true, false},
      {"mulv", 'f', 64, false, false},     {"eps", 'f', 32, false, false},     {"a1", 'b', 6272, false, false},
      {"a2", 'b', 3136, false, false},     {"d0", 'b', 3136, false, false},    {"d1", 'b', 6272, false, false},
      {"dlog", 'f', 784, false, false},    {"gd1", 'b', 6272, false, false},   {"gd0", 'b', 3136, false, false},
      {"dbd_part", 'f', 3136, false, false}, {"dmulv", 'f', 64, false, false}, {"dmulv16", 'b', 64, false, false},
      {"ga2", 'b', 3136, false, false},    {"ga1", 'b', 6272, false, false},   {"db3_part", 'f', 32, false, false},
      {"db2_part", 'f', 128, false, false}, {"db1_part", 'f', 32, false, false},
      {"stamps", 'l', 32, false, true}};
  slots.insert(slots.end(), rest.begin(), rest.end());
  return slots;
}

// X is [rows][784] and idx whole batches of B (cursor * B + n indexes it).
void f28_check_data(const std::vector<c10::optional<at::Tensor>>& t, int64_t B) {
  TORCH_CHECK(t.size() > 13 && t[12].has_value() && t[13].has_value(), "f28: X and idx are required");
  TORCH_CHECK(t[12]->numel() % 784 == 0, "f28: X must be [rows][784], has ", t[12]->numel(), " elements");
  TORCH_CHECK(t[13]->numel() % B == 0, "f28: idx must hold whole batches of ", B, ", has ", t[13]->numel());
}

std::vector<long long> f28_pair_ptrs(const std::vector<c10::optional<at::Tensor>>& pair, int64_t M, int dev) {
  const std::vector<Slot> ps = {{"xchg", 'l', 2 * (int64_t)mdt_f28_pair_words(), false, false},
                                {"pairw", 'i', 1, false, false},
                                {"err", 'i', 1, true, false}};
  return f28_ptrs(pair, ps, M, dev);
}

// `pair` (eval only, train = false): the same three tensors as f28_step's;
// the forward then runs two workgroups per sample (mdt_f28_forward_pair).
void f28_forward(const std::vector<c10::optional<at::Tensor>>& t, int64_t B, int64_t M, int64_t stream, bool train,
                 const std::vector<c10::optional<at::Tensor>>& pair) {
  TORCH_CHECK(M > 0 && M <= B, "f28_forward: bad M ", M, " for B ", B);
  TORCH_CHECK(pair.empty() || !train, "f28_forward: the paired forward is eval-only");
  f28_check_data(t, B);
  const int dev = t[0].has_value() ? (int)t[0]->device().index() : 0;
  const auto p = f28_ptrs(t, f28_fwd_slots(B, train), M, dev);
  if (!pair.empty()) {
    const auto pp = f28_pair_ptrs(pair, M, dev);
    rc(mdt_f28_forward_pair(p.data(), pp.data(), (int)B, (int)M, (unsigned)stream, cur()), "f28_forward(pair)");
    return;
  }
  rc(mdt_f28_forward(p.data(), (int)B, (int)M, (unsigned)stream, train ? 1 : 0, cur()), "f28_forward");
}

void f28_backward(const std::vector<c10::optional<at::Tensor>>& t, int64_t M) {
  TORCH_CHECK(M > 0, "f28_backward: bad M");
  const int dev = t[0].has_value() ? (int)t[0]->device().index() : 0;
  const auto p = f28_ptrs(t, f28_bwd_slots(), M, dev);
  rc(mdt_f28_backward(p.data(), (int)M, cur()), "f28_backward");
}

// Forward + backward of one training step in ONE launch (f28_step_k). With
// `pair` (three tensors: exchange granules int64 [B][2][f28_pair_words()],
// pairing words int32 [B], error word int32 [1], all zero-initialised) the
// launch runs two workgroups per sample.
void f28_step(const std::vector<c10::optional<at::Tensor>>& tf, const std::vector<c10::optional<at::Tensor>>& tb,
              int64_t B, int64_t M, int64_t stream, const std::vector<c10::optional<at::Tensor>>& pair,
              int64_t pair_delay_us) {
  TORCH_CHECK(M > 0 && M <= B, "f28_step: bad M ", M, " for B ", B);
  f28_check_data(tf, B);
  const int dev = tf[0].has_value() ? (int)tf[0]->device().index() : 0;
  const auto pf = f28_ptrs(tf, f28_fwd_slots(B, true), M, dev);
  const auto pb = f28_ptrs(tb, f28_bwd_slots(), M, dev);
  std::vector<long long> pp;
  if (!pair.empty()) pp = f28_pair_ptrs(pair, M, dev);
  rc(mdt_f28_step(pf.data(), pb.data(), pp.empty() ? nullptr : pp.data(), (int)B, (int)M, (unsigned)stream,
                  pp.empty() ? 0 : 1, (int)pair_delay_us, cur()),
     "f28_step");
}

void step_begin(at::Tensor state, const at::Tensor& hparams) {
  rc(mdt_step_begin(state.data_ptr(), hparams.data_ptr(), cur()), "step_begin");
}

// segment = (off, numel, slab_ptr, nsplit, co, k, s, ci, toff); slab_ptr is a
// device address (tensor.data_ptr()) or 0. The caller keeps the slabs alive.
at::Tensor make_grad_segs(const std::vector<std::vector<int64_t>>& segs, int64_t device_index) {
  std::vector<GradSeg> v;
  for (auto& s : segs) {
    TORCH_CHECK(s.size() == 9, "segment = (off, numel, slab_ptr, nsplit, co, k, s, ci, toff)");
    GradSeg g;
    g.off = s[0]; g.numel = s[1];
    g.slab = reinterpret_cast<const float*>((uintptr_t)s[2]);
    g.nsplit = (int)s[3]; g.co = (int)s[4]; g.k = (int)s[5]; g.s = (int)s[6]; g.ci = (int)s[7]; g.toff = s[8];
    TORCH_CHECK(g.toff < 0 || (g.s > 0 && g.k % g.s == 0), "transposed copy needs k % s == 0");
    v.push_back(g);
  }
  auto cpu = torch::empty({(int64_t)(v.size() * sizeof(GradSeg))}, torch::kUInt8);
  std::memcpy(cpu.data_ptr(), v.data(), v.size() * sizeof(GradSeg));
  return cpu.to(torch::Device(torch::kCUDA, device_index));
}

at::Tensor make_grad_units(const std::vector<std::vector<int64_t>>& units, int64_t device_index) {
  std::vector<GradUnit> v;
  for (auto& u : units) {
    // count <= 256: one element (column) per thread group; 256 < count <= 1024: 4 elements per thread
    TORCH_CHECK(u.size() == 3 && u[2] >= 1 && u[2] <= 1024, "unit = (seg, start, count<=1024)");
    v.push_back(GradUnit{(int)u[0], (int)u[1], (int)u[2]});
  }
  auto cpu = torch::empty({(int64_t)std::max<size_t>(1, v.size() * sizeof(GradUnit))}, torch::kUInt8);
  if (!v.empty()) std::memcpy(cpu.data_ptr(), v.data(), v.size() * sizeof(GradUnit));
  return cpu.to(torch::Device(torch::kCUDA, device_index));
}

at::Tensor make_tr_units(const std::vector<std::vector<int64_t>>& units, int64_t device_index) {
  std::vector<TrUnit> v;
  for (auto& u : units) {
    TORCH_CHECK(u.size() == 4, "unit = (seg, tap, co0, ci0)");
    v.push_back(TrUnit{(int)u[0], (int)u[1], (int)u[2], (int)u[3]});
  }
  auto cpu = torch::empty({(int64_t)std::max<size_t>(1, v.size() * sizeof(TrUnit))}, torch::kUInt8);
  if (!v.empty()) std::memcpy(cpu.data_ptr(), v.data(), v.size() * sizeof(TrUnit));
  return cpu.to(torch::Device(torch::kCUDA, device_index));
}

void adam_cast(at::Tensor P, const at::Tensor& G, at::Tensor M, at::Tensor V, at::Tensor w16, const at::Tensor& segs,
               int64_t nseg, const at::Tensor& state, const at::Tensor& hparams, bool do_adam) {
  TORCH_CHECK(G.numel() == P.numel() && M.numel() == P.numel() && V.numel() == P.numel() && w16.numel() == P.numel(),
              "adam_cast: P, G, m, v and w16 must be arenas of one size");
  rc(mdt_adam_cast(P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(),
                   w16.data_ptr(), segs.data_ptr(), (int)nseg, P.numel(), state.data_ptr(), hparams.data_ptr(),
                   do_adam ? 1 : 0, cur()),
     "adam_cast");
}

void grad_finalize(at::Tensor P, at::Tensor G, at::Tensor M, at::Tensor V, at::Tensor w16, const at::Tensor& segs,
                   const at::Tensor& units, int64_t nunits, const at::Tensor& state, const at::Tensor& hparams,
                   bool do_adam, Job* job, const std::vector<at::Tensor>& gather, int64_t gather_B, bool dep) {
  TORCH_CHECK(units.numel() >= nunits * (int64_t)sizeof(GradUnit), "grad_finalize: unit table too small");
  if (job) {
    TORCH_CHECK(gather.empty(), "grad_finalize: a finalize job takes no gather (use gather_job)");
    rc(mdt_job_finalize(&job->main, P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(),
                        V.data_ptr<float>(), w16.data_ptr(), segs.data_ptr(), units.data_ptr(), (int)nunits,
                        state.data_ptr(), hparams.data_ptr(), do_adam ? 1 : 0, dep ? 1 : 0),
       "job_finalize");
    return;
  }
  TORCH_CHECK(!dep, "grad_finalize: dep applies to finalize jobs only");
  // optional next-batch gather (the fused 28x28 step): [X, idx, xn, xtag] and the batch size
  const float* gX = nullptr;
  const int* gidx = nullptr;
  float* xn = nullptr;
  unsigned* xtag = nullptr;
  if (!gather.empty()) {
    TORCH_CHECK(gather.size() == 4 && gather_B > 0, "grad_finalize: gather = [X, idx, xn, xtag] with gather_B > 0");
    const int dev = P.get_device();
    const char* nm[4] = {"X", "idx", "xn", "xtag"};
    for (int i = 0; i < 4; ++i)
      TORCH_CHECK(gather[i].is_cuda() && gather[i].get_device() == dev && gather[i].is_contiguous(),
                  "grad_finalize: gather ", nm[i], " must be a contiguous tensor on the arena's device");
    TORCH_CHECK(gather[0].scalar_type() == torch::kFloat32 && gather[0].numel() % 784 == 0, "grad_finalize: X [rows][784] f32");
    TORCH_CHECK(gather[1].scalar_type() == torch::kInt32 && gather[1].numel() % gather_B == 0,
                "grad_finalize: idx int32 in whole batches");
    TORCH_CHECK(gather[2].scalar_type() == torch::kFloat32 && gather[2].numel() >= gather_B * 784, "grad_finalize: xn");
    TORCH_CHECK(gather[3].scalar_type() == torch::kInt32 && gather[3].numel() >= gather_B, "grad_finalize: xtag");
    gX = gather[0].data_ptr<float>();
    gidx = gather[1].data_ptr<int>();
    xn = gather[2].data_ptr<float>();
    xtag = reinterpret_cast<unsigned*>(gather[3].data_ptr<int>());
  }
  rc(mdt_grad_finalize(P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(),
                       w16.data_ptr(), segs.data_ptr(), units.data_ptr(), (int)nunits, state.data_ptr(),
                       hparams.data_ptr(), do_adam ? 1 : 0, gX, gidx, xn, xtag, (int)gather_B, cur()),
     "grad_finalize");
}

// Next-batch gather as a job of a dependent multi-job launch (it waits for
// the launch's loss/step job): rows idx[cursor * B + n] of X -> xn, xtag = step.
void gather_job(const at::Tensor& X, const at::Tensor& idx, const at::Tensor& state, at::Tensor xn, at::Tensor xtag,
                int64_t B, Job* job) {
  TORCH_CHECK(job != nullptr, "gather_job: records into a Job");
  const int dev = X.get_device();
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&idx, &state, &xn, &xtag})
    TORCH_CHECK(t->is_cuda() && t->get_device() == dev && t->is_contiguous(), "gather_job: tensors on one device");
  TORCH_CHECK(X.is_cuda() && X.is_contiguous() && X.scalar_type() == torch::kFloat32 && X.numel() % 784 == 0,
              "gather_job: X [rows][784] f32");
  TORCH_CHECK(B > 0 && idx.scalar_type() == torch::kInt32 && idx.numel() % B == 0, "gather_job: idx int32 in whole batches");
  TORCH_CHECK(xn.scalar_type() == torch::kFloat32 && xn.numel() >= B * 784, "gather_job: xn");
  TORCH_CHECK(xtag.scalar_type() == torch::kInt32 && xtag.numel() >= B, "gather_job: xtag");
  TORCH_CHECK(state.numel() >= (int64_t)sizeof(TrainState), "gather_job: state");
  rc(mdt_job_gather(&job->main, X.data_ptr<float>(), idx.data_ptr<int>(), state.data_ptr(), xn.data_ptr<float>(),
                    reinterpret_cast<unsigned*>(xtag.data_ptr<int>()), (int)B),
     "job_gather");
}

// Record a fused all-reduce job (csrc/kernels/comm_jobs.h) over `nunits`
// finalize units: mode 1 push, 2 reduce(+Adam), 3 both. `ctx` is the device
// address from XgmiP2PReducer.comm_ctx(). Jobs only: they run inside a
// jobs_multi_k launch next to other work of the step.
void comm_job(at::Tensor P, at::Tensor G, at::Tensor M, at::Tensor V, at::Tensor w16, const at::Tensor& segs,
              const at::Tensor& units, int64_t nunits, const at::Tensor& state, const at::Tensor& hparams,
              bool do_adam, int64_t ctx, int64_t mode, Job* job) {
  TORCH_CHECK(job != nullptr, "comm_job: records into a Job (no stand-alone launch)");
  TORCH_CHECK(units.numel() >= nunits * (int64_t)sizeof(GradUnit), "comm_job: unit table too small");
  TORCH_CHECK(P.numel() == G.numel() && M.numel() == G.numel() && V.numel() == G.numel() && w16.numel() == G.numel(),
              "comm_job: arenas differ in size");
  rc(mdt_job_comm(&job->main, P.data_ptr<float>(), G.data_ptr<float>(), M.data_ptr<float>(), V.data_ptr<float>(),
                  w16.data_ptr(), segs.data_ptr(), units.data_ptr(), (int)nunits, state.data_ptr(),
                  hparams.data_ptr(), do_adam ? 1 : 0, reinterpret_cast<const void*>((intptr_t)ctx), (int)mode),
     "job_comm");
}

void wtrans(const at::Tensor& w16, at::Tensor w16t, const at::Tensor& segs, const at::Tensor& units, int64_t nunits,
            Job* job) {
  check_bf16(w16, "w16");
  check_bf16(w16t, "w16t");
  TORCH_CHECK(units.numel() >= nunits * (int64_t)sizeof(TrUnit), "wtrans: unit table too small");
  if (job) {
    rc(mdt_job_wtrans(&job->main, w16.data_ptr(), w16t.data_ptr(), segs.data_ptr(), units.data_ptr(), (int)nunits),
       "job_wtrans");
    return;
  }
  rc(mdt_wtrans(w16.data_ptr(), w16t.data_ptr(), segs.data_ptr(), units.data_ptr(), (int)nunits, cur()), "wtrans");
}

// Split-K combine of the encoder head fused with the reparameterisation, and
// of the decoder Linear's backward-data fused with its backward.
void combine_reparam(const at::Tensor& ws, int64_t ks, const c10::optional<at::Tensor>& bias, at::Tensor mulv,
                     at::Tensor eps, at::Tensor z16, const c10::optional<at::Tensor>& z32, int64_t B, int64_t Z,
                     const at::Tensor& state, const at::Tensor& hparams, int64_t stream, at::Tensor kld_part) {
  check_f32(ws, "ws");
  TORCH_CHECK(ws.numel() >= ks * B * 2 * Z && mulv.numel() >= B * 2 * Z && eps.numel() >= B * Z &&
                  z16.numel() >= B * Z && kld_part.numel() >= mdt_combine_reparam_blocks((int)ks, (int)B, (int)Z),
              "combine_reparam: buffer too small");
  rc(mdt_combine_reparam(ws.data_ptr<float>(), (int)ks, (const float*)opt_ptr(bias), mulv.data_ptr<float>(),
                         eps.data_ptr<float>(), z16.data_ptr(), (float*)opt_ptr(z32), (int)B, (int)Z, state.data_ptr(),
                         hparams.data_ptr(), (unsigned)stream, kld_part.data_ptr<float>(), cur()),
     "combine_reparam");
}

void combine_reparam_bwd(const at::Tensor& ws, int64_t ks, const at::Tensor& mulv, const at::Tensor& eps,
                         at::Tensor dmulv, const c10::optional<at::Tensor>& dmulv16,
                         const c10::optional<at::Tensor>& dz, int64_t B, int64_t Z, const at::Tensor& hparams) {
  check_f32(ws, "ws");
  TORCH_CHECK(ws.numel() >= ks * B * Z && dmulv.numel() >= B * 2 * Z, "combine_reparam_bwd: buffer too small");
  rc(mdt_combine_reparam_bwd(ws.data_ptr<float>(), (int)ks, mulv.data_ptr<float>(), eps.data_ptr<float>(),
                             dmulv.data_ptr<float>(), const_cast<void*>(opt_ptr(dmulv16)), (float*)opt_ptr(dz), (int)B,
                             (int)Z, hparams.data_ptr(), cur()),
     "combine_reparam_bwd");
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
  m.def("igemm_plan", &igemm_plan, py::arg("mode"), py::arg("desc"), py::arg("allow_split"), py::arg("fwd") = false);
  m.def("dconv_stamps", [](const c10::optional<at::Tensor>& t) {
    // profiling: per-workgroup s_memrealtime stamps of the direct conv kernels ([grid][8] int64), None = off
    if (t.has_value() && t->defined()) {
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64, "dconv_stamps: int64 CUDA tensor");
      mdt_dconv_stamps(reinterpret_cast<unsigned long long*>(t->data_ptr()));
    } else {
      mdt_dconv_stamps(nullptr);
    }
  });
  m.def("wgrad_plan", &wgrad_plan);
  py::class_<Job>(m, "Job")
      .def(py::init<>())
      .def_property_readonly("kind", &Job::kind)
      .def_property_readonly("nblk", [](const Job& j) { return j.main.nblk; })
      .def_property_readonly("has_post", &Job::has_post);
  m.def("launch_jobs", &launch_jobs);
  m.def("pack_jobs_multi", &pack_jobs_multi, py::arg("jobs"), py::arg("stamps") = py::none(),
        py::arg("wait") = std::vector<int64_t>{}, py::arg("dep_ctr") = py::none());
  m.def("launch_jobs_multi", &launch_jobs_multi, py::arg("dev_pack"), py::arg("grid"), py::arg("dep") = false);
  m.def("f28_forward", &f28_forward, py::arg("tensors"), py::arg("B"), py::arg("M"), py::arg("stream"),
        py::arg("train"), py::arg("pair") = std::vector<c10::optional<at::Tensor>>{});
  m.def("f28_backward", &f28_backward, py::arg("tensors"), py::arg("M"));
  m.def("f28_pair_words", &mdt_f28_pair_words);
  m.def("f28_step", &f28_step, py::arg("fwd_tensors"), py::arg("bwd_tensors"), py::arg("B"), py::arg("M"),
        py::arg("stream"), py::arg("pair") = std::vector<c10::optional<at::Tensor>>{},
        py::arg("pair_delay_us") = 0);
  m.def("igemm", &igemm, py::arg("mode"), py::arg("A"), py::arg("B16"), py::arg("desc"), py::arg("bias"),
        py::arg("relu"), py::arg("y16"), py::arg("y32"), py::arg("omask") = py::none(),
        py::arg("colsum") = py::none(), py::arg("ws") = py::none(), py::arg("job") = py::none(),
        py::arg("combine") = true, py::arg("a_slab") = py::none(), py::arg("a_ks") = 0,
        py::arg("a_bias") = py::none(), py::arg("a_relu") = false, py::arg("a_out16") = py::none(),
        py::arg("fwd") = false);
  m.def("wgrad", &wgrad, py::arg("G16"), py::arg("X"), py::arg("desc"), py::arg("out"), py::arg("job") = py::none());
  m.def("colsum", &colsum, py::arg("G16"), py::arg("M"), py::arg("N"), py::arg("rows_per"), py::arg("slab"),
        py::arg("job") = py::none());
  m.def("thin_conv", &thin_conv, py::arg("X"), py::arg("Wf"), py::arg("desc"), py::arg("bias"), py::arg("relu"),
        py::arg("y16"), py::arg("omask") = py::none(), py::arg("colsum") = py::none(), py::arg("job") = py::none(),
        py::arg("idx") = py::none(), py::arg("state") = py::none(), py::arg("hparams") = py::none(),
        py::arg("B") = 0, py::arg("xb") = py::none());
  m.def("thin_blocks", &thin_blocks);
  m.def("thin_tconv", &thin_tconv, py::arg("G16"), py::arg("Wf"), py::arg("desc"), py::arg("bias"),
        py::arg("y32") = py::none(), py::arg("X") = py::none(), py::arg("dlog16") = py::none(),
        py::arg("recon") = py::none(), py::arg("part") = py::none(), py::arg("gpart") = py::none());
  m.def("gather_rows", &gather_rows);
  m.def("reparam", &reparam);
  m.def("reparam_bwd", &reparam_bwd);
  m.def("bce_logits", &bce_logits, py::arg("logits"), py::arg("X"), py::arg("rows"), py::arg("B"), py::arg("P"),
        py::arg("dlog16"), py::arg("recon"), py::arg("part"), py::arg("gpart") = py::none());
  m.def("loss_finalize2", &loss_finalize2, py::arg("bce_part"), py::arg("nb"), py::arg("kld_part"), py::arg("nk"),
        py::arg("state"), py::arg("hparams"), py::arg("advance_cursor"), py::arg("job") = py::none(),
        py::arg("advance_step") = false);
  m.def("step_begin", &step_begin);
  m.def("make_grad_segs", &make_grad_segs);
  m.def("make_grad_units", &make_grad_units);
  m.def("make_tr_units", &make_tr_units);
  m.def("adam_cast", &adam_cast);
  m.def("graph_upload", [](int64_t exec) {
    // Upload an instantiated step graph to the device ahead of its first
    // replay, so that launch's one-time cost stays out of a timed region.
    TORCH_CHECK(exec != 0, "graph_upload: null graph exec");
    rc((int)hipGraphUpload(reinterpret_cast<hipGraphExec_t>((intptr_t)exec), cur()), "hipGraphUpload");
  });
  m.def("grad_finalize", &grad_finalize, py::arg("P"), py::arg("G"), py::arg("M"), py::arg("V"), py::arg("w16"),
        py::arg("segs"), py::arg("units"), py::arg("nunits"), py::arg("state"), py::arg("hparams"),
        py::arg("do_adam"), py::arg("job") = py::none(), py::arg("gather") = std::vector<at::Tensor>{},
        py::arg("gather_B") = 0, py::arg("dep") = false);
  m.def("gather_job", &gather_job, py::arg("X"), py::arg("idx"), py::arg("state"), py::arg("xn"), py::arg("xtag"),
        py::arg("B"), py::arg("job"));
  // dependency counter block of a dependent multi-job launch: (words, index of the error word)
  m.def("jobs_dep_layout", [] { return std::make_tuple((int64_t)mdt_jobs_dep_words(), (int64_t)mdt_jobs_dep_err()); });
  m.def("comm_job", &comm_job, py::arg("P"), py::arg("G"), py::arg("M"), py::arg("V"), py::arg("w16"),
        py::arg("segs"), py::arg("units"), py::arg("nunits"), py::arg("state"), py::arg("hparams"),
        py::arg("do_adam"), py::arg("ctx"), py::arg("mode"), py::arg("job"));
  m.def("wtrans", &wtrans, py::arg("w16"), py::arg("w16t"), py::arg("segs"), py::arg("units"), py::arg("nunits"),
        py::arg("job") = py::none());
  m.def("combine_reparam", &combine_reparam);
  m.def("combine_reparam_bwd", &combine_reparam_bwd);
  m.def("combine_reparam_blocks", &mdt_combine_reparam_blocks);
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
