// Thin torch wrappers over the hardware probe kernels (csrc/kernels/probe.hip).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

extern "C" int mdt_probe_clock(unsigned long long* out, int iters, hipStream_t s);
extern "C" int mdt_probe_latency(const int* idx, int hops, unsigned long long* out, hipStream_t s);
extern "C" int mdt_probe_empty(int blocks, int threads, hipStream_t s);
extern "C" int mdt_probe_lds_poison(unsigned pattern, int blocks, hipStream_t s);
extern "C" int mdt_probe_cu_ids(unsigned* out, int blocks, hipStream_t s);

namespace mdt {

void probe_clock(at::Tensor out, int64_t iters) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kInt64 && out.numel() >= 3, "out: cuda int64[3]");
  TORCH_CHECK(mdt_probe_clock(reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()), (int)iters,
                              c10::hip::getCurrentHIPStream().stream()) == 0, "probe_clock");
}

void probe_latency(at::Tensor idx, int64_t hops, at::Tensor out) {
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == torch::kInt32, "idx: cuda int32");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kInt64 && out.numel() >= 2, "out: cuda int64[2]");
  TORCH_CHECK(mdt_probe_latency(idx.data_ptr<int32_t>(), (int)hops,
                                reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>()),
                                c10::hip::getCurrentHIPStream().stream()) == 0, "probe_latency");
}

void probe_empty(int64_t blocks, int64_t threads) {
  TORCH_CHECK(mdt_probe_empty((int)blocks, (int)threads, c10::hip::getCurrentHIPStream().stream()) == 0,
              "probe_empty");
}

void probe_lds_poison(int64_t pattern, int64_t blocks) {
  TORCH_CHECK(blocks > 0 && blocks <= 65536, "probe_lds_poison: blocks");
  TORCH_CHECK(mdt_probe_lds_poison((unsigned)pattern, (int)blocks, c10::hip::getCurrentHIPStream().stream()) == 0,
              "probe_lds_poison");
}

void probe_cu_ids(at::Tensor out) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == torch::kInt32 && out.numel() >= 1, "out: cuda int32[blocks]");
  TORCH_CHECK(mdt_probe_cu_ids(reinterpret_cast<unsigned*>(out.data_ptr<int32_t>()), (int)out.numel(),
                               c10::hip::getCurrentHIPStream().stream()) == 0, "probe_cu_ids");
}

}  // namespace mdt
