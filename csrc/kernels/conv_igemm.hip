// LDS-tiled implicit-GEMM convolution kernels for the conv-VAE on CDNA4
// (gfx950): bf16 operands, v_mfma_f32_16x16x32_bf16, f32 accumulation.
//
// Design (docs/KERNELS.md, "Conv/deconv VAE"):
//  * igemm_fwd_k — forward-type GEMM  Y[rows][cols] = sum_k A(row, k) * Bw[col][k]
//      kModeConv : rows = conv output pixels, k = (ky, kx, ci)   (conv fwd, convT bwd-data)
//      kModeTconv: rows = conv INPUT pixels of one stride-parity class (blockIdx.z),
//                  k = (ty, tx, co) over the taps that actually hit the class
//                  (conv bwd-data, convT fwd). No zero-insertion work: for the
//                  k4/s2 layers each class sees exactly 2x2 of the 16 taps.
//  * wgrad_k     — dW[co][k'] = sum_m G[m][co] * im2col(X)[m][k'] with the m
//                  reduction on the MFMA k axis: both operands are staged m-major
//                  (coalesced 16-B rows) and read with ds_read_b64_tr_b16, the
//                  CDNA4 transposing LDS read. Split over m into f32 partial
//                  slabs reduced deterministically by grad_finalize_k.
//  * grad_finalize_k / wtrans_k (conv_bf16.hip) — partial-slab reduction
//                  (+ fused Adam and bf16 cast), then an LDS-tiled transpose
//                  into the parity-ordered weights the kModeTconv GEMM reads.
// Tiles are 64-deep in k, double-buffered in LDS (register staging: loads for
// tile k+1 are in flight while the MFMAs of tile k run), XOR-swizzled images,
// blockIdx remapped so neighbouring tiles share an XCD's L2.
// Epilogues fuse bias, ReLU, the ReLU-backward mask of the produced gradient
// and the per-block column sums that become the next layer's bias gradient.
#include <algorithm>

#include "conv_igemm_dev.h"
#include "conv_direct.h"
#include "conv_dwgrad.h"
#include "conv_thin_wg.h"

namespace mdt {

__global__ void __launch_bounds__(256) splitk_combine_k(CombineArgs c) {
  __shared__ float red[256];
  splitk_combine_body(c, red, blockIdx.x);
}

__global__ void __launch_bounds__(256) colsum_k(ColsumArgs c) { colsum_body(c, blockIdx.x); }

}  // namespace mdt

// =================================================================== host ====
using namespace mdt;

namespace {
inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
}  // namespace

namespace mdt {
using namespace mdt::tiles;

// Patch-resident direct kernel (conv_direct.h) for a geometry: configuration
// index, or -1. MDT_CONV_DIRECT=0 keeps every layer on the im2col kernels.
struct DcInfo {
  int RB, NBB, MT, NB;
};
template <class CF>
constexpr DcInfo dc_info() { return DcInfo{CF::RB, CF::NBB, CF::MT, CF::NB}; }
static const DcInfo kDcInfo[] = {dc_info<DcS1>(), dc_info<DcS2>(), dc_info<DcT2>(),
                                  dc_info<DcT3>(), dc_info<DcS3>(), dc_info<DcT1>()};

// the 16x16 <-> 8x8 geometries (MDT_DCONV_SMALL=0 keeps them on im2col)
static bool direct_small() {
  static const bool on = [] {
    const char* e = getenv("MDT_DCONV_SMALL");
    return !(e && e[0] == '0');
  }();
  return on;
}

int direct_cfg(int mode, const ConvDesc& d, bool fwd) {
  static const bool on = [] {
    const char* e = getenv("MDT_CONV_DIRECT");
    return !(e && e[0] == '0');
  }();
  // the two-workgroups-per-CU tiles (R = 4): measured 15-18 % faster than
  // one-per-CU R = 8 tiles and 3-4 % faster than three-per-CU R = 2 tiles at
  // B = 64 and 128 (profiles/r2_dconv)
  // MDT_DCONV_BWD=0: forward calls only (backward-data keeps the fusable im2col kernel)
  static const bool bwd = [] {
    const char* e = getenv("MDT_DCONV_BWD");
    return !(e && e[0] == '0');
  }();
  if (!on || d.KH != 4 || d.KW != 4 || d.S != 2 || d.P != 1) return -1;
  if (!fwd && !bwd) return -1;
  if (d.H != d.W || d.OH != d.OW || d.H != 2 * d.OH) return -1;
  if (mode == kModeConv) {  // A = input (H, C), columns = CO
    if (d.C == 32 && d.H == 64 && d.CO == 64) return 0;
    if (d.C == 64 && d.H == 32 && d.CO == 128) return 1;
    // 16x16 -> 8x8: forward only; as a backward-data GEMM the im2col kernel
    // fuses with the weight gradient in one launch, which measured faster
    if (d.C == 128 && d.H == 16 && d.CO == 256 && fwd && direct_small()) return 4;
  } else {  // A = conv output (OH, CO), columns = C
    if (d.CO == 128 && d.OH == 16 && d.C == 64) return 2;
    if (d.CO == 64 && d.OH == 32 && d.C == 32) return 3;
    if (d.CO == 256 && d.OH == 8 && d.C == 128 && fwd && direct_small()) return 5;
  }
  return -1;
}

bool plan_fwd(int mode, const ConvDesc& d, bool allow_split, FwdPlan* p, bool allow_direct, bool fwd) {
  FwdPlan q{};
  const int dc = allow_direct ? direct_cfg(mode, d, fwd) : -1;
  if (dc >= 0) {
    const DcInfo& di = kDcInfo[dc];
    q.direct = dc + 1;
    q.classes = mode == kModeConv ? 1 : 4;
    q.M = mode == kModeConv ? d.N * d.OH * d.OW : d.N * d.OH * d.OW;
    q.Ncols = mode == kModeConv ? d.CO : d.C;
    q.K = mode == kModeConv ? 16 * d.C : 4 * d.CO;
    q.BM = di.MT; q.BN = di.NB;
    q.mtiles = d.N * di.RB; q.ntiles = di.NBB; q.ktiles = q.K / 64;
    q.ksplit = 1; q.kt_per_split = q.ktiles;
    q.colsum_rows = d.N * di.RB;
    q.cfg = 100 + dc;
    *p = q;
    return true;
  }
  if (mode == kModeConv) {
    q.classes = 1;
    q.M = d.N * d.OH * d.OW;
    q.Ncols = d.CO;
    q.K = d.KH * d.KW * d.C;
    q.thin = (d.C % 8) != 0;
  } else {
    if (d.KH % d.S || d.KW % d.S || d.H % d.S || d.W % d.S || d.CO % 8) return false;
    q.classes = d.S * d.S;
    q.M = d.N * (d.H / d.S) * (d.W / d.S);
    q.Ncols = d.C;
    q.K = (d.KH / d.S) * (d.KW / d.S) * d.CO;
    q.thin = 0;
  }
  if (q.K % 8 || q.M <= 0) return false;
  q.BN = q.Ncols >= 128 ? 128 : q.Ncols > 32 ? 64 : q.Ncols > 16 ? 32 : 16;
  if (q.thin) q.BN = 32;
  // narrower column tiles for deep (>= MDT_CONV_BN_SPLIT_MIN_KT = 16 k-tiles)
  // problems whose grid would stay under MDT_CONV_BN_SPLIT_BELOW = 512 blocks:
  // more workgroups in flight for the wide-N, short-M 128x128 layers (4 % on
  // that step); shallow ones (the 28x28 decoder Linear, K = 32) lose from the
  // extra A re-reads, so they keep their tiles (profiles/r1_knobs)
  static const int bn_split_below = [] {
    const char* e = getenv("MDT_CONV_BN_SPLIT_BELOW");
    return e ? atoi(e) : 512;
  }();
  static const int bn_split_min_kt = [] {
    const char* e = getenv("MDT_CONV_BN_SPLIT_MIN_KT");
    return e ? atoi(e) : 16;
  }();
  // ... and, at any depth, while the grid would stay under
  // MDT_CONV_BN_SPLIT_TINY = 512 blocks: the shallow Linear GEMMs (the 28x28
  // decoder Linear / head backward-data, M = 128: 50 blocks of 64x128; the
  // 128x128 model's dec_fc forward and head backward-data, M = 64, K <= 128:
  // 128 blocks) spread over more CUs. 64 -> 512 measured conv128 B=64
  // 0.3727-0.374 -> 0.3644-0.3645 ms/step, 1024 0.3767 (profiles/r4_tiles);
  // 28x28 layer path: profiles/r1_defer/bn_tiny
  static const int bn_split_tiny = [] {
    const char* e = getenv("MDT_CONV_BN_SPLIT_TINY");
    return e ? atoi(e) : 512;
  }();
  auto grid64 = [&] { return (long long)q.classes * cdiv(q.M, 64) * cdiv(q.Ncols, q.BN); };
  while (q.BN > 32 && !q.thin &&
         ((cdiv(q.K, 64) >= bn_split_min_kt && grid64() < bn_split_below) || grid64() < bn_split_tiny))
    q.BN /= 2;
  q.ntiles = cdiv(q.Ncols, q.BN);
  q.ktiles = cdiv(q.K, 64);
  // 64-row tiles when 128-row tiles would leave the grid under `bm64_below`
  // blocks (MDT_CONV_BM64_BELOW; default 1024 = 4 per CU, measured 3 % faster
  // than 512 on the 128x128 step and 0.5 % on the 28x28 one, profiles/r1_knobs)
  static const int bm64_below = [] {
    const char* e = getenv("MDT_CONV_BM64_BELOW");
    return e ? atoi(e) : 1024;
  }();
  q.BM = 128;
  if ((long long)q.classes * cdiv(q.M, 128) * q.ntiles < bm64_below) q.BM = 64;
  q.mtiles = cdiv(q.M, q.BM);
  const long long blocks = (long long)q.classes * q.mtiles * q.ntiles;
  q.ksplit = 1;
  // split-K only for deep problems (>= 8 k-tiles, MDT_CONV_SPLIT_MIN_KT) whose
  // grid is under-filled; the combine is fused into a following launch where
  // the model allows it (enc_head -> reparam, dec_fc dgrad -> reparam backward)
  static const int min_kt = [] {
    const char* e = getenv("MDT_CONV_SPLIT_MIN_KT");
    return e ? atoi(e) : 8;
  }();
  // at least `kt_per` k-tiles per split (MDT_CONV_SPLIT_KT_PER, default 1):
  // fewer k-steps per block against more partial slabs for the combine pass
  // to read; 1 measured 3 % faster than 4 on the 28x28 step (profiles/r1_knobs)
  static const int kt_per = [] {
    const char* e = getenv("MDT_CONV_SPLIT_KT_PER");
    const int v = e ? atoi(e) : 1;
    return v < 1 ? 1 : v;
  }();
  if (allow_split && q.classes == 1 && blocks < 256 && q.ktiles >= min_kt) {
    int ks = cdiv(512, blocks);
    if (ks > q.ktiles / kt_per) ks = q.ktiles / kt_per;
    if (ks < 1) ks = 1;
    q.ksplit = ks;
  }
  q.kt_per_split = cdiv(q.ktiles, q.ksplit);
  q.ksplit = cdiv(q.ktiles, q.kt_per_split);
  q.colsum_rows = q.classes * q.mtiles;
  const int bn_i = q.BN == 128 ? 0 : q.BN == 64 ? 1 : q.BN == 32 ? 2 : 3;
  q.cfg = (q.BM == 128 ? 0 : 4) + bn_i;
  *p = q;
  return true;
}

// Direct weight-gradient geometry (conv_dwgrad.h) of `d`: 0 = DwL1, 1 = DwL2,
// -1 = none. MDT_DWGRAD=0 keeps every layer on the im2col kernel; DwL2 (the
// 32x32x64 -> 16x16x128 layer) only with MDT_DWGRAD_L2=1: its [N][128][1024]
// partial rows are 4x the im2col kernel's slab.
int dwgrad_cfg(const ConvDesc& d) {
  static const bool on = [] {
    const char* e = getenv("MDT_DWGRAD");
    return !(e && e[0] == '0');
  }();
  const char* e2 = getenv("MDT_DWGRAD_L2");  // read per plan (tests switch it inside one process)
  const bool l2 = e2 && e2[0] == '1';
  if (!on || d.S != 2 || d.P != 1 || d.KH != 4 || d.KW != 4 || d.H != d.W || d.OH != d.OW || d.OH * 2 != d.H)
    return -1;
  if (d.H == DwL1::H && d.C == DwL1::C && d.CO == DwL1::CO) return 0;
  if (l2 && d.H == DwL2::H && d.C == DwL2::C && d.CO == DwL2::CO) return 1;
  return -1;
}

bool plan_wgrad(const ConvDesc& d, WgradPlan* p) {
  WgradPlan q{};
  if (d.CO % 8) return false;
  if (thin_wgrad_mfma_ok(d)) {  // conv_thin_wg.h: one partial row per 4 output rows
    q.cfg = 110;
    q.thin = true;
    q.M = d.N * d.OH * d.OW;
    q.K2 = d.KH * d.KW * d.C;
    q.BM = d.CO;
    q.BN = q.K2;
    q.cotiles = q.ktiles = 1;
    q.mtiles = d.N * d.OH / 4;
    q.nsplit = q.mtiles;
    q.mt_per_split = 1;
    *p = q;
    return true;
  }
  const int dw = dwgrad_cfg(d);
  if (dw >= 0) {  // one partial row per image (the workgroups of its four kernel rows)
    q.cfg = 100 + dw;
    q.M = d.N * d.OH * d.OW;
    q.K2 = d.KH * d.KW * d.C;
    q.BM = d.CO;
    q.BN = q.K2;
    q.cotiles = q.ktiles = 1;
    q.mtiles = d.N;
    q.nsplit = d.N;
    q.mt_per_split = 1;
    *p = q;
    return true;
  }
  q.M = d.N * d.OH * d.OW;
  q.K2 = d.KH * d.KW * d.C;
  q.thin = (d.C % 8) != 0;
  q.BM = d.CO > 32 ? 64 : 32;
  q.BN = q.K2 > 32 ? 64 : q.K2 > 16 ? 32 : 16;
  if (q.thin && q.BN == 32) q.BN = 64;
  q.cotiles = cdiv(d.CO, q.BM);
  q.ktiles = cdiv(q.K2, q.BN);
  q.mtiles = cdiv(q.M, 64);
  const int tiles = q.cotiles * q.ktiles;
  // m-splits so the grid reaches ~`target` blocks. Default: ~16 m-steps per
  // block, clamped to [160, 640] blocks -- measured on MI355X (profiles/r1_knobs):
  // the 28x28 layers (98 m-tiles) want few splits (fewer partial slabs for the
  // finalize to read), the 128x128 layers (up to 4096 m-tiles) want the grid
  // wide (a 320-block grid left ~200 serial m-steps per block).
  // MDT_CONV_WG_TARGET pins the target instead.
  static const int fixed_target = [] {
    const char* e = getenv("MDT_CONV_WG_TARGET");
    return e ? atoi(e) : 0;
  }();
  // MDT_CONV_WG_TARGET_THIN pins the target of the single-channel-input
  // (thin) layers only: their finalize sits on the optimizer tail
  static const int thin_target = [] {
    const char* e = getenv("MDT_CONV_WG_TARGET_THIN");
    return e ? atoi(e) : 0;
  }();
  int target = q.thin && thin_target > 0 ? thin_target : fixed_target;
  if (target <= 0) {
    const long long work = (long long)q.mtiles * tiles;
    target = (int)std::min<long long>(640, std::max<long long>(160, work / 16));
  }
  int ns = cdiv(target, tiles);
  if (ns > q.mtiles / 2) ns = q.mtiles / 2;
  if (ns < 1) ns = 1;
  q.mt_per_split = cdiv(q.mtiles, ns);
  q.nsplit = cdiv(q.mtiles, q.mt_per_split);
  q.cfg = (q.BM == 64 ? 0 : 3) + (q.BN == 64 ? 0 : q.BN == 32 ? 1 : 2);
  *p = q;
  return true;
}

int build_igemm(int mode, const void* A, const void* B16, ConvDesc d, const float* bias, int relu, void* y16,
                float* y32, const void* omask, float* colsum, float* ws, IgArgs* pa, FwdPlan* pq, CombineArgs* pc,
                int* nc) {
  FwdPlan q;
  const bool can_split = ws != nullptr && omask == nullptr && colsum == nullptr;
  if (!plan_fwd(mode, d, can_split, &q, false)) return 1;
  IgArgs a{};
  a.d = d;
  a.A = A;
  a.B = reinterpret_cast<const __bf16*>(B16);
  a.relu = relu;
  a.M = q.M; a.Ncols = q.Ncols; a.K = q.K; a.mtiles = q.mtiles; a.ntiles = q.ntiles; a.ktiles = q.ktiles;
  a.kt_per_split = q.kt_per_split;
  if (mode == kModeConv) {
    a.f_pix = make_fastdiv(d.OH * d.OW); a.f_w = make_fastdiv(d.OW);
    a.f_ch = make_fastdiv(d.C); a.f_tw = make_fastdiv(d.KW);
  } else {
    a.f_pix = make_fastdiv((d.H / d.S) * (d.W / d.S)); a.f_w = make_fastdiv(d.W / d.S);
    a.f_ch = make_fastdiv(d.CO); a.f_tw = make_fastdiv(d.KW / d.S);
  }
  *nc = 0;
  if (q.ksplit > 1) {
    a.slab = ws;
    const long long MN = (long long)q.M * q.Ncols;
    int rp = 1;
    while (rp < 64 && rp * 4 < q.ksplit) rp *= 2;
    const int cnt = 256 / rp;
    *pc = CombineArgs{ws, q.ksplit, q.M, q.Ncols, cnt, bias, relu, y32, reinterpret_cast<__bf16*>(y16)};
    *nc = cdiv(MN, cnt);
  } else {
    a.y16 = reinterpret_cast<__bf16*>(y16); a.y32 = y32; a.bias = bias;
    a.omask = reinterpret_cast<const __bf16*>(omask); a.colsum = colsum;
  }
  *pa = a;
  *pq = q;
  return 0;
}

int build_wgrad(const void* G16, const void* X, ConvDesc d, float* out, WgArgs* pa, WgradPlan* pq) {
  WgradPlan q;
  if (!plan_wgrad(d, &q)) return 1;
  WgArgs a{};
  a.d = d;
  a.G = reinterpret_cast<const __bf16*>(G16);
  a.X = X;
  a.out = out;
  a.M = q.M; a.K2 = q.K2; a.cotiles = q.cotiles; a.ktiles = q.ktiles; a.mtiles = q.mtiles;
  a.mt_per_split = q.mt_per_split;
  a.f_pix = make_fastdiv(d.OH * d.OW); a.f_w = make_fastdiv(d.OW);
  a.f_c = make_fastdiv(d.C); a.f_kw = make_fastdiv(d.KW);
  *pa = a;
  *pq = q;
  return 0;
}

template <typename XT>
__global__ void __launch_bounds__(256) thin_wgrad_k(WgArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[thin_wgrad_mfma_lds_bytes()];
  thin_wgrad_mfma_body<XT>(a, lds, blockIdx.x);
}

static unsigned long long* g_dc_stamps = nullptr;

template <class CF>
void launch_dc(const DcArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((dconv_k<CF>), dim3(a.nimg * CF::RB * CF::NBB), dim3(CF::THREADS), 0, s, a);
}

int launch_direct(int cfg, const void* A, const void* B16, const ConvDesc& d, const float* bias, int relu, void* y16,
                  float* y32, const void* omask, float* colsum, hipStream_t s) {
  DcArgs a{};
  a.A = reinterpret_cast<const __bf16*>(A);
  a.B = reinterpret_cast<const __bf16*>(B16);
  a.y16 = reinterpret_cast<__bf16*>(y16);
  a.y32 = y32;
  a.bias = bias;
  a.omask = reinterpret_cast<const __bf16*>(omask);
  a.colsum = colsum;
  a.stamps = g_dc_stamps;
  a.relu = relu;
  a.nimg = d.N;
  switch (cfg) {
    case 0: launch_dc<DcS1>(a, s); break;
    case 1: launch_dc<DcS2>(a, s); break;
    case 2: launch_dc<DcT2>(a, s); break;
    case 3: launch_dc<DcT3>(a, s); break;
    case 4: launch_dc<DcS3>(a, s); break;
    case 5: launch_dc<DcT1>(a, s); break;
    default: return 2;
  }
  return (int)hipGetLastError();
}

int launch_splitk_combine(const CombineArgs& c, int nblk, hipStream_t s) {
  hipLaunchKernelGGL(splitk_combine_k, dim3(nblk), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

}  // namespace mdt

namespace {
using namespace mdt::tiles;

template <int MODE, typename AT, bool VEC, class TC, bool PRO = false>
void launch_fwd(const IgArgs& a, const FwdPlan& q, hipStream_t s) {
  dim3 grid(q.mtiles * q.ntiles, q.ksplit, q.classes);
  hipLaunchKernelGGL((igemm_fwd_k<MODE, AT, VEC, TC, PRO>), grid, dim3(256), 0, s, a);
}

template <int MODE, typename AT, bool VEC, bool PRO = false>
int dispatch_fwd_cfg(const IgArgs& a, const FwdPlan& q, hipStream_t s) {
  switch (q.cfg) {
    case 0: launch_fwd<MODE, AT, VEC, F0, PRO>(a, q, s); return 0;
    case 1: launch_fwd<MODE, AT, VEC, F1, PRO>(a, q, s); return 0;
    case 2: launch_fwd<MODE, AT, VEC, F2, PRO>(a, q, s); return 0;
    case 3: launch_fwd<MODE, AT, VEC, F3, PRO>(a, q, s); return 0;
    case 4: launch_fwd<MODE, AT, VEC, F4, PRO>(a, q, s); return 0;
    case 5: launch_fwd<MODE, AT, VEC, F5, PRO>(a, q, s); return 0;
    case 6: launch_fwd<MODE, AT, VEC, F6, PRO>(a, q, s); return 0;
    case 7: launch_fwd<MODE, AT, VEC, F7, PRO>(a, q, s); return 0;
  }
  return 2;
}

template <typename AT>
int dispatch_thin(const IgArgs& a, const FwdPlan& q, hipStream_t s) {
  if (q.cfg == 2) { launch_fwd<kModeConv, AT, false, F2>(a, q, s); return 0; }
  if (q.cfg == 6) { launch_fwd<kModeConv, AT, false, F6>(a, q, s); return 0; }
  return 2;
}

template <typename XT, bool VEC, class TC>
void launch_wg(const WgArgs& a, const WgradPlan& q, hipStream_t s) {
  dim3 grid(q.cotiles * q.ktiles * q.nsplit);
  hipLaunchKernelGGL((wgrad_k<XT, VEC, TC>), grid, dim3(256), 0, s, a);
}

}  // namespace

extern "C" {

// info[12] = {cfg, BM, BN, classes, M, Ncols, K, mtiles, ntiles, ktiles, ksplit, colsum_rows}
int mdt_igemm_plan(int mode, ConvDesc d, int allow_split, int* info, int fwd) {
  FwdPlan q;
  if (!plan_fwd(mode, d, allow_split != 0, &q, true, fwd != 0)) return 1;
  const int v[12] = {q.cfg, q.BM, q.BN, q.classes, q.M, q.Ncols, q.K, q.mtiles, q.ntiles, q.ktiles, q.ksplit,
                     q.colsum_rows};
  for (int i = 0; i < 12; ++i) info[i] = v[i];
  return 0;
}

// info[8] = {cfg, BM, BN, cotiles, ktiles, mtiles, nsplit, mt_per_split}
int mdt_wgrad_plan(ConvDesc d, int* info) {
  WgradPlan q;
  if (!plan_wgrad(d, &q)) return 1;
  const int v[8] = {q.cfg, q.BM, q.BN, q.cotiles, q.ktiles, q.mtiles, q.nsplit, q.mt_per_split};
  for (int i = 0; i < 8; ++i) info[i] = v[i];
  return 0;
}

// Forward-type implicit GEMM. `ws` (f32, >= ksplit*M*Ncols) enables split-K
// for deep, narrow problems (then bias/relu/y16/y32 are applied by a combine
// pass; omask/colsum are not allowed with split-K).
int mdt_igemm(int mode, const void* A, int a_is_f32, const void* B16, ConvDesc d, const float* bias, int relu,
              void* y16, float* y32, const void* omask, float* colsum, float* ws, int skip_combine, hipStream_t s,
              const APro* pro, int fwd) {
  IgArgs a;
  FwdPlan q;
  CombineArgs c;
  int nc = 0;
  const int dc = direct_cfg(mode, d, fwd != 0);
  if (dc >= 0) {  // the planner reported the direct tiling: never fall back silently
    if ((pro && pro->slab) || a_is_f32) return 5;
    return launch_direct(dc, A, B16, d, bias, relu, y16, y32, omask, colsum, s);
  }
  if (build_igemm(mode, A, B16, d, bias, relu, y16, y32, omask, colsum, ws, &a, &q, &c, &nc)) return 1;
  int rc;
  if (pro && pro->slab) {
    // A from the producer's split-K slabs: conv-mode, bf16 vector gathers only
    if (mode != kModeConv || q.thin || a_is_f32 || pro->cin % 8 || pro->ks < 1) return 4;
    a.pro = *pro;
    rc = dispatch_fwd_cfg<kModeConv, __bf16, true, true>(a, q, s);
  } else if (mode == kModeConv) {
    if (q.thin) rc = a_is_f32 ? dispatch_thin<float>(a, q, s) : dispatch_thin<__bf16>(a, q, s);
    else if (a_is_f32) rc = 3;
    else rc = dispatch_fwd_cfg<kModeConv, __bf16, true>(a, q, s);
  } else if (a_is_f32) {
    rc = 3;
  } else {
    rc = dispatch_fwd_cfg<kModeTconv, __bf16, true>(a, q, s);
  }
  if (rc) return rc;
  if (nc > 0 && !skip_combine) hipLaunchKernelGGL(splitk_combine_k, dim3(nc), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

int mdt_wgrad(const void* G16, const void* X, int x_is_f32, ConvDesc d, float* out, hipStream_t s) {
  WgArgs a;
  WgradPlan q;
  if (build_wgrad(G16, X, d, out, &a, &q)) return 1;
  if (q.cfg == 110) {
    if (x_is_f32) hipLaunchKernelGGL(thin_wgrad_k<float>, dim3(q.nsplit), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(thin_wgrad_k<__bf16>, dim3(q.nsplit), dim3(256), 0, s, a);
    return (int)hipGetLastError();
  }
  if (q.cfg >= 100) {
    if (x_is_f32) return 3;
    const DwArgs da{reinterpret_cast<const __bf16*>(X), reinterpret_cast<const __bf16*>(G16), out, d.N, g_dc_stamps};
    if (q.cfg == 100) hipLaunchKernelGGL(dwgrad_k<DwL1>, dim3(d.N * 4), dim3(DwL1::THREADS), 0, s, da);
    else if (q.cfg == 101) hipLaunchKernelGGL(dwgrad_k<DwL2>, dim3(d.N * 4), dim3(DwL2::THREADS), 0, s, da);
    else return 2;
    return (int)hipGetLastError();
  }
  if (!q.thin) {
    if (x_is_f32) return 3;
    switch (q.cfg) {
      case 0: launch_wg<__bf16, true, W0>(a, q, s); break;
      case 1: launch_wg<__bf16, true, W1>(a, q, s); break;
      case 2: launch_wg<__bf16, true, W2>(a, q, s); break;
      case 3: launch_wg<__bf16, true, W3>(a, q, s); break;
      case 4: launch_wg<__bf16, true, W4>(a, q, s); break;
      case 5: launch_wg<__bf16, true, W5>(a, q, s); break;
      default: return 2;
    }
  } else {
    // thin inputs (C % 8 != 0): k' tiles of 16 or 64
    switch (q.cfg) {
      case 0: if (x_is_f32) launch_wg<float, false, W0>(a, q, s); else launch_wg<__bf16, false, W0>(a, q, s); break;
      case 2: if (x_is_f32) launch_wg<float, false, W2>(a, q, s); else launch_wg<__bf16, false, W2>(a, q, s); break;
      case 3: if (x_is_f32) launch_wg<float, false, W3>(a, q, s); else launch_wg<__bf16, false, W3>(a, q, s); break;
      case 5: if (x_is_f32) launch_wg<float, false, W5>(a, q, s); else launch_wg<__bf16, false, W5>(a, q, s); break;
      default: return 2;
    }
  }
  return (int)hipGetLastError();
}

// Profiling: per-workgroup s_memrealtime stamps ([grid][8]) of the direct kernels, or null.
void mdt_dconv_stamps(unsigned long long* p) { g_dc_stamps = p; }

int mdt_colsum(const void* G16, int M, int N, int rows_per, float* slab, hipStream_t s) {
  if (N % 8 || rows_per < 1) return 1;
  const int gx = cdiv(N / 8, 256);
  const ColsumArgs c{reinterpret_cast<const __bf16*>(G16), M, N, rows_per, gx, slab};
  hipLaunchKernelGGL(colsum_k, dim3(gx * cdiv(M, rows_per)), dim3(256), 0, s, c);
  return (int)hipGetLastError();
}

}  // extern "C"
