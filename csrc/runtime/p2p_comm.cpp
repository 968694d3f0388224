// XgmiP2PReducer: one-shot / two-shot peer-to-peer bucket all-reduce over xGMI (hipIpc).
//
// on a fully connected 8x MI355X node a group of s GPUs
// has s-1 direct xGMI links per GPU. RCCL's ring crosses one link per step and
// pays 2(s-1) hops of latency, which dominates the small (1-4 MB) gradient
// buckets of the VAE models (/root/reference/vae-hpo.py:130 uses torch DDP's
// ring all-reduce for them). This reducer pushes each bucket to every peer at
// once (kernel: csrc/kernels/p2p_allreduce.hip) and needs no communicator:
//   * each rank allocates ONE uncached device region (receive slabs
//     [bucket][parity][src][n], or for a two-shot bucket reduce-scatter and
//     all-gather slabs [2][parity][src][n/s] + per-(phase, src, block) flags +
//     epoch counters),
//   * buckets of at least `two_shot_min_bytes` (-1: never) run two-shot:
//     reduce-scatter to the chunk owners, then all-gather, so each of the s-1
//     links carries 2/s of the bucket (one-shot: all of it) -- the
//     bandwidth-bound regime of the 128x128 model's ~18 MB of gradients,
//     exports it with hipIpcGetMemHandle, and maps every peer's region with
//     hipIpcOpenMemHandle (handles are exchanged by the caller over the gloo
//     control plane, parallel/ddp.py::make_p2p_reducer);
//   * launch/wait/readiness semantics, the high-priority stream and the event
//     fences come from StreamBuckets, so it drops in for RcclBucketReducer and
//     stays hipGraph-capturable;
//   * waits are time-bounded in the kernel; `status()` reports a timed-out
//     bucket instead of hanging the GPU.
// `connect_local` maps peers that live in the same process (single-GPU tests
// run s "ranks" on one device, each with its own stream).
// With `fused` the region also holds the receive slots / flags / epochs of the
// all-reduce JOBS (csrc/kernels/comm_jobs.h; one epoch per step, read from the
// trainer's step counter): models that issue their own
// backward launches put the push and the reduce+Adam of the gradient arena
// into those launches instead of calling launch()/wait() (one stream, no
// events); `comm_ctx()` is the device descriptor those jobs take.
#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <list>
#include <mutex>
#include <utility>

#include "kernels/p2p_allreduce.h"
#include "runtime/stream_buckets.h"

namespace mdt {

// Process-lifetime pool of the uncached regions. A freed region is kept for
// the next reducer of the same device and size class instead of going back to
// the runtime: otherwise its address range -- still mapped uncached -- was
// handed out again to torch's caching allocator, and later trainers'
// activations and partial slabs landed in it (scripts/diag/diag_uc_reuse.py); the
// reducer-free 28x28 step then stopped being run-to-run bitwise in the
// processes where that happened (profiles/r4_determinism). On the round-6
// tree the pool-off A/B no longer reproduces, and a freed range reused by a
// later buffer stays bitwise (profiles/r6_determinism): the pool is kept as a
// safe default, not as a fix. Sizes are rounded up to a power of two (>= 1 MiB) so reducers
// with different bucket layouts share regions; a parked region is kept for the
// life of the process (the round-5 eviction of the oldest region
// re-opened exactly the reuse path above). The parked count is bounded by the
// peak number of reducers alive at once per size class.
// MDT_UC_POOL=0 turns the pool off (regions go back to the runtime with
// hipFree, the round-3 behaviour): the A/B switch of profiles/r6_determinism.
class UncachedPool {
 public:
  static bool enabled() {
    static const bool on = [] {
      const char* v = std::getenv("MDT_UC_POOL");
      return !(v && v[0] == '0');
    }();
    return on;
  }
  static size_t size_class(size_t bytes) {
    size_t c = (size_t)1 << 20;
    while (c < bytes) c <<= 1;
    return c;
  }
  static void* take(int dev, size_t bytes) {
    if (!enabled()) return nullptr;
    std::lock_guard<std::mutex> g(mu());
    auto& l = free_list();
    for (auto it = l.rbegin(); it != l.rend(); ++it) {  // the most recently freed region of that class
      if (it->dev == dev && it->bytes == bytes) {
        void* p = it->p;
        l.erase(std::next(it).base());
        return p;
      }
    }
    return nullptr;
  }
  static void give(int dev, size_t bytes, void* p) {
    if (!enabled()) {  // the caller synchronized the device: no kernel still touches it
      (void)hipFree(p);
      return;
    }
    std::lock_guard<std::mutex> g(mu());
    free_list().push_back({dev, bytes, p});
  }
  static int64_t parked(int dev) {
    std::lock_guard<std::mutex> g(mu());
    int64_t n = 0;
    for (const auto& r : free_list()) n += r.dev == dev;
    return n;
  }

 private:
  struct Region {
    int dev;
    size_t bytes;
    void* p;
  };
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::list<Region>& free_list() {
    static auto* l = new std::list<Region>();  // never destroyed: outlives every reducer
    return *l;
  }
};

class XgmiP2PReducer : public StreamBuckets {
 public:
  XgmiP2PReducer(int64_t rank, int64_t size, at::Tensor flat, std::vector<int64_t> bounds, bool average,
                 double scale, int64_t max_blocks, double timeout_s, int64_t two_shot_min_bytes, bool fused)
      : StreamBuckets(std::move(flat), std::move(bounds)), me_((int)rank), s_((int)size), fused_(fused) {
    TORCH_CHECK(s_ >= 1 && s_ <= kP2PMaxRanks, "XgmiP2PReducer: group size must be 1..", kP2PMaxRanks);
    TORCH_CHECK(me_ >= 0 && me_ < s_, "XgmiP2PReducer: rank out of range");
    TORCH_CHECK(flat_.scalar_type() == torch::kFloat32, "XgmiP2PReducer: f32 gradient arena required");
    scale_ = (float)(scale > 0 ? scale : (average ? 1.0 / s_ : 1.0));
    timeout_ticks_ = (long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    const int64_t nb = num_buckets();
    long long roff = 0, foff = 0, eoff = 0;
    for (int64_t b = 0; b < nb; ++b) {
      const long long n = bounds_[b + 1] - bounds_[b];
      // two-shot (reduce-scatter + all-gather) for big buckets of groups >= 2: every link carries 2/s of
      // the bucket instead of all of it, for one extra hop of latency
      const bool two = s_ >= 2 && two_shot_min_bytes >= 0 && n * 4 >= two_shot_min_bytes;
      const long long cs = ((n + s_ - 1) / s_ + 3) / 4 * 4;  // chunk per owner (kernel: same formula)
      long long g = ((two ? cs : n) + 2047) / 2048;            // >= 2K elements (8 KB) per block
      g = std::max(1LL, std::min(g, (long long)max_blocks));
      grid_.push_back((int)g);
      two_.push_back(two ? 1 : 0);
      recv_off_.push_back(roff);
      flag_off_.push_back(foff);
      ep_off_.push_back(eoff);
      roff += two ? 4LL * s_ * ((cs + 63) / 64 * 64) : 2LL * s_ * ((n + 63) / 64 * 64);
      foff += 2LL * s_ * g;
      eoff += g;
    }
    recv_elems_ = roff;
    // one region: [recv floats][flags u32][epochs u32][status i32], each part 256-B aligned
    auto al = [](long long x) { return (x + 255) / 256 * 256; };
    flags_byte_ = al(recv_elems_ * 4);
    ep_byte_ = flags_byte_ + al(foff * 4);
    status_byte_ = ep_byte_ + al(eoff * 4);
    bytes_ = status_byte_ + 256;
    if (fused_) {  // comm_jobs.h: recv [2][s][numel] f32 | flags [s][numel] u32 (one epoch per step: none stored)
      const long long n = flat_.numel();
      // the jobs' two-shot form (reduce-scatter to chunk owners + all-gather, 2/s of the arena per link)
      // under the same rule as the buckets': groups >= 3 and an arena of at least two_shot_min_bytes
      fused_two_ = s_ >= 3 && two_shot_min_bytes >= 0 && n * 4 >= two_shot_min_bytes;
      frecv_byte_ = bytes_;
      fflags_byte_ = frecv_byte_ + al(2LL * s_ * n * 4);
      bytes_ = fflags_byte_ + al((long long)s_ * n * 4);
    }
    alloc_bytes_ = (long long)UncachedPool::size_class((size_t)bytes_);
    DeviceGuard dg(device_);
    base_ = UncachedPool::take(device_, (size_t)alloc_bytes_);
    if (!base_) MDT_HIP_CHECK(hipExtMallocWithFlags(&base_, (size_t)alloc_bytes_, hipDeviceMallocUncached));
    MDT_HIP_CHECK(hipMemset((char*)base_ + flags_byte_, 0, (size_t)(bytes_ - flags_byte_)));
    // the host's abort word (abort()): pinned, mapped into the device address space, read uncached by the waits
    MDT_HIP_CHECK(hipHostMalloc((void**)&abort_host_, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    *abort_host_ = 0;
    MDT_HIP_CHECK(hipHostGetDevicePointer((void**)&abort_dev_, abort_host_, 0));
    MDT_HIP_CHECK(hipDeviceSynchronize());
    for (int p = 0; p < kP2PMaxRanks; ++p) peer_base_[p] = nullptr;
    peer_base_[me_] = base_;
  }

  ~XgmiP2PReducer() override {
    DeviceGuard dg(device_);
    // the fused jobs run on the trainer's stream, not stream_: no kernel of
    // any stream may still read ctx_ / the abort word / the region below
    (void)hipDeviceSynchronize();
    if (ctx_) (void)hipFree(ctx_);
    for (void* m : test_mem_) (void)hipFree(m);
    if (test_bad_) (void)hipFree(test_bad_);
    for (int p = 0; p < s_; ++p)
      if (p != me_ && peer_base_[p] && opened_[p]) (void)hipIpcCloseMemHandle(peer_base_[p]);
    if (base_) UncachedPool::give(device_, (size_t)alloc_bytes_, base_);
    if (abort_host_) (void)hipHostFree(abort_host_);
  }

  // 64-byte hipIpcMemHandle_t of this rank's region (uint8 CPU tensor)
  at::Tensor ipc_handle() {
    DeviceGuard dg(device_);
    hipIpcMemHandle_t h;
    MDT_HIP_CHECK(hipIpcGetMemHandle(&h, base_));
    auto t = torch::empty({(int64_t)sizeof(h)}, torch::kUInt8);
    std::memcpy(t.data_ptr(), &h, sizeof(h));
    return t;
  }
  int64_t local_base() const { return (int64_t)(uintptr_t)base_; }
  int64_t region_bytes() const { return bytes_; }

  void connect(std::vector<at::Tensor> handles) {
    TORCH_CHECK((int)handles.size() == s_, "connect: need one handle per rank");
    DeviceGuard dg(device_);
    for (int p = 0; p < s_; ++p) {
      if (p == me_) continue;
      TORCH_CHECK(handles[p].numel() == (int64_t)sizeof(hipIpcMemHandle_t), "bad IPC handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[p].contiguous().data_ptr(), sizeof(h));
      void* ptr = nullptr;
      MDT_HIP_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
      peer_base_[p] = ptr;
      opened_[p] = true;
    }
    connected_ = true;
  }
  void connect_local(std::vector<int64_t> bases) {
    TORCH_CHECK((int)bases.size() == s_, "connect_local: need one base per rank");
    for (int p = 0; p < s_; ++p)
      if (p != me_) peer_base_[p] = (void*)(uintptr_t)bases[p];
    connected_ = true;
  }

  int64_t status() {
    DeviceGuard dg(device_);
    int v = 0;
    MDT_HIP_CHECK(hipStreamSynchronize(stream_));
    MDT_HIP_CHECK(hipMemcpy(&v, (char*)base_ + status_byte_, sizeof(int), hipMemcpyDeviceToHost));
    return v;
  }
  double scale() const { return scale_; }
  bool fused() const { return fused_; }
  bool fused_two_shot() const { return fused_two_; }

  // Abandon every wait of this reducer, now and later (the runner's _abort
  // after a peer was lost): the host-mapped word is visible to kernels that
  // are already spinning, so the queued steps drain at once (status() then
  // reports kCommAborted unless a timeout was recorded first). No sync.
  void abort() { __atomic_store_n(abort_host_, 1, __ATOMIC_SEQ_CST); }
  bool aborted() const { return __atomic_load_n(abort_host_, __ATOMIC_SEQ_CST) != 0; }

  // The fused jobs' epoch of a step is TrainState.step + ep_base. Call when the
  // host moves the trainer's step counter from `old_step` back to `new_step`
  // (every member of the group the same way, at a point where no step is in
  // flight): the epochs keep increasing, so no stale peer flag looks current.
  void rebase_epochs(int64_t old_step, int64_t new_step) {
    if (new_step >= old_step) return;
    ep_base_ += (old_step - new_step) + 2;
    if (ctx_) {
      DeviceGuard dg(device_);
      MDT_HIP_CHECK(hipDeviceSynchronize());
      MDT_HIP_CHECK(hipMemcpy((char*)ctx_ + offsetof(CommCtx, ep_base), &ep_base_, sizeof(ep_base_),
                              hipMemcpyHostToDevice));
    }
  }
  int64_t epoch_base() const { return ep_base_; }
  static int64_t pooled_regions(int64_t dev) { return UncachedPool::parked((int)dev); }
  int64_t alloc_bytes() const { return alloc_bytes_; }

  // Device address of the CommCtx the fused all-reduce jobs take (built once,
  // after connect; a one-rank group needs no connect).
  int64_t comm_ctx() {
    TORCH_CHECK(fused_, "XgmiP2PReducer: built without fused=True");
    TORCH_CHECK(connected_ || s_ == 1, "XgmiP2PReducer: connect() before comm_ctx()");
    if (!ctx_) {
      DeviceGuard dg(device_);
      const CommCtx c = host_ctx();
      MDT_HIP_CHECK(hipMalloc(&ctx_, sizeof(CommCtx)));
      MDT_HIP_CHECK(hipMemcpy(ctx_, &c, sizeof(CommCtx), hipMemcpyHostToDevice));
    }
    return (int64_t)(uintptr_t)ctx_;
  }

  // CommCtx of the construction-time data-plane self-test
  // (parallel/ddp.py::selftest_fused): the production peer mappings, layout
  // and scale, but its own status word, epoch base 0 (the test runs epochs
  // 1 and 2; rebase_epochs moves the trainer's epochs past them), a short
  // timeout and the given one-/two-shot form. Freed with the reducer.
  int64_t selftest_ctx(double timeout_s, bool two_shot) {
    TORCH_CHECK(fused_, "XgmiP2PReducer: built without fused=True");
    TORCH_CHECK(connected_ || s_ == 1, "XgmiP2PReducer: connect() before selftest_ctx()");
    DeviceGuard dg(device_);
    void* mem = nullptr;
    MDT_HIP_CHECK(hipMalloc(&mem, 256 + sizeof(CommCtx)));
    test_mem_.push_back(mem);
    MDT_HIP_CHECK(hipMemset(mem, 0, 256));
    CommCtx c = host_ctx();
    c.status = (int*)mem;
    c.ep_base = 0;
    c.two_shot = (two_shot && s_ > 2) ? 1 : 0;
    c.timeout_ticks = (long long)(timeout_s * 1e8);
    MDT_HIP_CHECK(hipMemcpy((char*)mem + 256, &c, sizeof(CommCtx), hipMemcpyHostToDevice));
    return (int64_t)(uintptr_t)((char*)mem + 256);
  }
  // The self-test's rank-coded pattern of rank q in `g` (f32, flat-arena
  // sized), and the count of elements of `g` that differ bitwise from the
  // rank-order sum of all s patterns x this reducer's scale (syncs the device).
  void selftest_fill(at::Tensor g, int64_t q) {
    TORCH_CHECK(g.is_cuda() && g.scalar_type() == torch::kFloat32 && g.is_contiguous() && g.numel() == flat_.numel(),
                "selftest_fill: f32 tensor of the arena's size");
    DeviceGuard dg(device_);
    TORCH_CHECK(mdt_selftest_fill(g.data_ptr<float>(), g.numel(), (int)q, c10::hip::getCurrentHIPStream().stream()) == 0,
                "selftest_fill launch failed");
  }
  int64_t selftest_check(const at::Tensor& g) {
    TORCH_CHECK(g.is_cuda() && g.scalar_type() == torch::kFloat32 && g.is_contiguous() && g.numel() == flat_.numel(),
                "selftest_check: f32 tensor of the arena's size");
    DeviceGuard dg(device_);
    if (!test_bad_) {
      MDT_HIP_CHECK(hipMalloc(&test_bad_, sizeof(int)));
    }
    hipStream_t st = c10::hip::getCurrentHIPStream().stream();
    MDT_HIP_CHECK(hipMemsetAsync(test_bad_, 0, sizeof(int), st));
    TORCH_CHECK(mdt_selftest_check(g.data_ptr<float>(), g.numel(), s_, scale_, test_bad_, st) == 0,
                "selftest_check launch failed");
    int bad = 0;
    MDT_HIP_CHECK(hipMemcpyAsync(&bad, test_bad_, sizeof(int), hipMemcpyDeviceToHost, st));
    MDT_HIP_CHECK(hipStreamSynchronize(st));
    return bad;
  }
  // status word of a self-test ctx (device sync first: every job has ended)
  int64_t selftest_status(int64_t ctx) {
    DeviceGuard dg(device_);
    bool known = false;
    for (void* m : test_mem_) known = known || (int64_t)(uintptr_t)((char*)m + 256) == ctx;
    TORCH_CHECK(known, "selftest_status: not a self-test ctx of this reducer");
    MDT_HIP_CHECK(hipDeviceSynchronize());
    int v = 0;
    MDT_HIP_CHECK(hipMemcpy(&v, (char*)(uintptr_t)ctx - 256, sizeof(int), hipMemcpyDeviceToHost));
    return v;
  }
  std::vector<int64_t> grids() const { return std::vector<int64_t>(grid_.begin(), grid_.end()); }
  std::vector<int64_t> two_shot() const { return std::vector<int64_t>(two_.begin(), two_.end()); }

 protected:
  void issue(int64_t b, hipStream_t s) override {
    TORCH_CHECK(connected_ || s_ == 1, "XgmiP2PReducer: connect() before launching");
    P2PArgs a{};
    a.data = (float*)flat_.data_ptr() + bounds_[b];
    a.n = bounds_[b + 1] - bounds_[b];
    for (int p = 0; p < kP2PMaxRanks; ++p) {
      a.peer_recv[p] = p < s_ ? (float*)peer_base_[p] : nullptr;
      a.peer_flags[p] = p < s_ ? (unsigned*)((char*)peer_base_[p] + flags_byte_) : nullptr;
    }
    a.my_recv = (float*)base_;
    a.my_flags = (unsigned*)((char*)base_ + flags_byte_);
    a.ep = (unsigned*)((char*)base_ + ep_byte_) + ep_off_[b];
    a.status = (int*)((char*)base_ + status_byte_);
    a.recv_off = recv_off_[b];
    a.flag_off = flag_off_[b];
    a.me = me_;
    a.s = s_;
    a.bucket = (int)b;
    a.two_shot = two_[b];
    a.scale = scale_;
    a.timeout_ticks = timeout_ticks_;
    a.abort_flag = abort_dev_;
    if (s_ == 1 && scale_ == 1.0f) return;
    const int rc = mdt_p2p_allreduce(&a, grid_[b], s);
    TORCH_CHECK(rc == 0, "p2p all-reduce launch failed: ", rc);
  }

 private:
  CommCtx host_ctx() const {
    CommCtx c{};
    for (int p = 0; p < kP2PMaxRanks; ++p) {
      c.peer_recv[p] = p < s_ ? (float*)((char*)peer_base_[p] + frecv_byte_) : nullptr;
      c.peer_flags[p] = p < s_ ? (unsigned*)((char*)peer_base_[p] + fflags_byte_) : nullptr;
    }
    c.status = (int*)((char*)base_ + status_byte_);
    c.abort_flag = abort_dev_;
    c.ep_base = ep_base_;
    c.numel = flat_.numel();
    c.me = me_;
    c.s = s_;
    c.two_shot = fused_two_ ? 1 : 0;
    c.scale = scale_;
    c.timeout_ticks = timeout_ticks_;
    return c;
  }

  int me_, s_;
  bool fused_ = false, fused_two_ = false;
  void* ctx_ = nullptr;
  std::vector<void*> test_mem_;
  int* test_bad_ = nullptr;
  long long frecv_byte_ = 0, fflags_byte_ = 0, alloc_bytes_ = 0;
  int64_t ep_base_ = 0;
  int* abort_host_ = nullptr;
  int* abort_dev_ = nullptr;
  float scale_ = 1.0f;
  long long timeout_ticks_ = 0;
  void* base_ = nullptr;
  void* peer_base_[kP2PMaxRanks];
  bool opened_[kP2PMaxRanks] = {};
  bool connected_ = false;
  long long recv_elems_ = 0, flags_byte_ = 0, ep_byte_ = 0, status_byte_ = 0, bytes_ = 0;
  std::vector<int> grid_, two_;
  std::vector<long long> recv_off_, flag_off_, ep_off_;
};

void bind_p2p(pybind11::module& m) {
  namespace py = pybind11;
  auto c = py::class_<XgmiP2PReducer>(m, "XgmiP2PReducer")
               .def(py::init<int64_t, int64_t, at::Tensor, std::vector<int64_t>, bool, double, int64_t, double, int64_t, bool>(),
                    py::arg("rank"), py::arg("size"), py::arg("flat"), py::arg("bounds"), py::arg("average") = true,
                    py::arg("scale") = 0.0, py::arg("max_blocks") = 64, py::arg("timeout_s") = 60.0,
                    py::arg("two_shot_min_bytes") = -1, py::arg("fused") = false)
               .def("ipc_handle", &XgmiP2PReducer::ipc_handle)
               .def("local_base", &XgmiP2PReducer::local_base)
               .def("region_bytes", &XgmiP2PReducer::region_bytes)
               .def("connect", &XgmiP2PReducer::connect)
               .def("connect_local", &XgmiP2PReducer::connect_local)
               .def("status", &XgmiP2PReducer::status)
               .def("fused", &XgmiP2PReducer::fused)
               .def("fused_two_shot", &XgmiP2PReducer::fused_two_shot)
               .def("comm_ctx", &XgmiP2PReducer::comm_ctx)
               .def("selftest_ctx", &XgmiP2PReducer::selftest_ctx, py::arg("timeout_s"), py::arg("two_shot"))
               .def("selftest_status", &XgmiP2PReducer::selftest_status)
               .def("selftest_fill", &XgmiP2PReducer::selftest_fill)
               .def("selftest_check", &XgmiP2PReducer::selftest_check)
               .def("scale", &XgmiP2PReducer::scale)
               .def("grids", &XgmiP2PReducer::grids)
               .def("two_shot", &XgmiP2PReducer::two_shot)
               .def("abort", &XgmiP2PReducer::abort)
               .def("aborted", &XgmiP2PReducer::aborted)
               .def("rebase_epochs", &XgmiP2PReducer::rebase_epochs)
               .def("epoch_base", &XgmiP2PReducer::epoch_base)
               .def("alloc_bytes", &XgmiP2PReducer::alloc_bytes)
               .def_static("pooled_regions", &XgmiP2PReducer::pooled_regions);
  def_bucket_api(c);
}

}  // namespace mdt
