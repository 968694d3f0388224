// Native owner of one MLP-VAE trial's device memory and kernel sequence.
//
// Memory is laid out for HBM residency and contiguous collectives:
//   params / grads / exp_avg / exp_avg_sq : one flat fp32 arena each, same
//     layout, every tensor 256-byte aligned. fc4 (the first gradients to
//     become final in backward) is placed LAST so gradient bucket 0 is the
//     arena tail and bucket 1 the head: both are contiguous views, the
//     all-reduce needs no pack/unpack copies.
//   acts : one arena for every saved activation / gradient-of-activation.
//   train_state / eval_state / hparams : device structs read by the kernels,
//     so a captured hipGraph replays across batches and hparam changes.
#pragma once
#include <torch/extension.h>

#include <string>
#include <tuple>
#include <vector>

namespace mdt {

struct LayoutEntry {
  std::string name;
  int64_t offset;
  std::vector<int64_t> shape;
};

class MlpVaeEngine {
 public:
  MlpVaeEngine(int64_t batch, int64_t D, int64_t H, int64_t Z, int64_t device_index);

  std::vector<std::tuple<std::string, int64_t, std::vector<int64_t>>> layout() const;
  int64_t numel() const { return total_; }
  int64_t bucket_split() const { return split_; }  // arena offset where fc4 starts

  void set_hparams(double lr, double beta1, double beta2, double eps, double weight_decay,
                   double kl_beta, double grad_scale, int64_t seed, bool decoupled_wd);
  void set_cursor(bool eval, int64_t cursor, int64_t nbatches);
  void set_step(int64_t step);
  void reset_loss(bool eval);
  std::vector<double> read_state(bool eval);          // step, cursor, nbatches, epoch_loss, epoch_count
  at::Tensor loss_history(bool eval);                  // CPU float tensor [kLossHist]

  void forward(const at::Tensor& X, const at::Tensor& idx, int64_t M, bool train, bool eval,
               int64_t rng_stream, bool want_recon);
  void backward(const at::Tensor& X, const at::Tensor& idx, int64_t M, int64_t part, bool fuse_adam);
  void adam();
  void loss_finalize(bool eval);
  at::Tensor decode(const at::Tensor& z);  // sigmoid(fc4(relu(fc3 z))) -> [M, D]
  at::Tensor act(const std::string& name, int64_t M);
  void set_stamps(at::Tensor t) { stamps_ = t; }  // int64 [6*512*8*8] or undefined

  at::Tensor params, grads, exp_avg, exp_avg_sq, acts, partials, train_state, eval_state, hparams;

 private:
  void fill_args(void* args, const at::Tensor& X, const at::Tensor& idx, int64_t M, bool train,
                 bool eval, int64_t rng_stream, bool want_recon);
  void write_pows(at::Tensor& state, int64_t step);
  int64_t B_, D_, H_, Z_, total_, split_;
  double beta1_ = -1.0, beta2_ = -1.0;
  int last_f2_blocks_ = 0, last_f3_blocks_ = 0;
  std::vector<LayoutEntry> layout_;
  at::Tensor stamps_;
  std::vector<std::pair<std::string, int64_t>> act_off_;
};

}  // namespace mdt
