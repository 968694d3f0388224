// Device code of the conv-VAE implicit-GEMM kernels (design notes in
// conv_igemm.hip). Shared by conv_igemm.hip (stand-alone kernels + host
// dispatch) and conv_jobs.hip (horizontally fused job kernels).
#pragma once
#include <stdlib.h>

#include "common.h"
#include "conv_igemm.h"

namespace mdt {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) { return (__umulhi(n, f.mul) + n) >> f.shr; }

// Bijective XCD-aware remap: blocks dispatched to the same XCD (orig % 8)
// receive consecutive tile ids, so a tile row's A panel stays in one L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
  return z;
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ bf16x8 load_chunk(const T* p);
template <>
__device__ __forceinline__ bf16x8 load_chunk<__bf16>(const __bf16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}
template <>
__device__ __forceinline__ bf16x8 load_chunk<float>(const float* p) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  bf16x8 r;
  r[0] = (__bf16)a.x; r[1] = (__bf16)a.y; r[2] = (__bf16)a.z; r[3] = (__bf16)a.w;
  r[4] = (__bf16)b.x; r[5] = (__bf16)b.y; r[6] = (__bf16)b.z; r[7] = (__bf16)b.w;
  return r;
}

// Row-major [rows][64] bf16 image (128-B rows) read by rows: 16-B chunk ch of
// row r lives at chunk slot ch ^ (r & 7).
__device__ __forceinline__ int rimg(int r, int ch) { return (r << 7) + (((ch ^ r) & 7) << 4); }

// m-major [64][WD] bf16 image read with ds_read_b64_tr_b16: the XOR keeps the
// eight 32-B row segments a 32-lane half reads (rows 8g+q and 8g+8+q) on
// disjoint banks for every row width used here.
template <int WD>
__device__ __forceinline__ int trsw(int r) {
  if constexpr (WD == 128) return 2 * ((r & 3) | (((r >> 3) & 1) << 2));
  else if constexpr (WD == 64) return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1));
  else if constexpr (WD == 32) return 2 * ((r >> 3) & 1);
  else return 0;
}
template <int WD>
__device__ __forceinline__ int timg(int r, int ch) { return r * (WD * 2) + ((ch ^ trsw<WD>(r)) << 4); }

// 16x16x32 MFMA operand whose 16 "rows" are image columns c0..c0+15 and whose
// 32 k values are image rows kb..kb+31: lane l gets column l&15, rows
// kb + 8(l>>4) + 0..7, via two transposing reads of 4 rows each.
template <int WD>
__device__ __forceinline__ bf16x8 tr_frag(const uint8_t* img, int c0, int kb, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r0 = kb + 8 * g + q, r1 = r0 + 4;
  const int ch = (c0 >> 3) + (p >> 1);
  const int sub = (p & 1) << 3;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + timg<WD>(r0, ch) + sub));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + timg<WD>(r1, ch) + sub));
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

template <int BM_, int BN_, int WM_, int WN_>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int KWS = 4 / (WM * WN);  // waves splitting the 64-deep k tile
  static constexpr int FM = BM / (16 * WM), FN = BN / (16 * WN);
  static_assert(WM * WN * KWS == 4 && KWS <= 2 && FM >= 1 && FN >= 1, "bad tile config");
  static constexpr int RED_BYTES = KWS == 2 ? WM * WN * FM * FN * 64 * 16 : 0;
};

// ================================================================ forward ====
struct IgArgs {
  ConvDesc d;
  APro pro;
  const void* A;
  const __bf16* B;  // [classes][Ncols][K]
  __bf16* y16;
  float* y32;
  const float* bias;
  const __bf16* omask;
  float* colsum;    // [classes*mtiles][Ncols] or null
  float* slab;      // split-K partials [ksplit][M][Ncols] (then no epilogue) or null
  int relu;
  int M, Ncols, K, mtiles, ntiles, ktiles, kt_per_split;
  FastDiv f_pix, f_w, f_ch, f_tw;
};

// Shared epilogue of the forward-type kernels: combine k-halves (KWS == 2),
// then either raw split-K partials or bias + ReLU + output mask + bf16/f32
// stores + per-block column sums. `lds` must be free (caller passed a barrier).
template <int MODE, class TC>
__device__ __forceinline__ void igemm_epilogue(const IgArgs& a, f32x4 (&acc)[TC::FM][TC::FN], uint8_t* lds, int mt,
                                               int nt, int kz, int cls, int oa, int ob) {
  constexpr int BM = TC::BM, BN = TC::BN, WM = TC::WM, WN = TC::WN, KWS = TC::KWS, FM = TC::FM, FN = TC::FN;
  const ConvDesc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = w / (WM * WN), wm = (w % (WM * WN)) / WN, wn = w % WN;
  if constexpr (KWS == 2) {  // combine the two k-halves
    float* red = reinterpret_cast<float*>(lds);
    const int slot = w % (WM * WN);
    if (wk == 1) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          *reinterpret_cast<f32x4*>(red + (((slot * FM + fm) * FN + fn) * 64 + lane) * 4) = acc[fm][fn];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] += *reinterpret_cast<const f32x4*>(red + (((slot * FM + fm) * FN + fn) * 64 + lane) * 4);
    }
  }

  const bool epi = (KWS == 1) || wk == 0;
  const int rbase = mt * BM + wm * (BM / WM) + 4 * (lane >> 4);
  const int cbase = nt * BN + wn * (BN / WN) + (lane & 15);
  if (a.slab) {
    if (epi) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = rbase + fm * 16 + r;
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            const int col = cbase + fn * 16;
            if (m < a.M && col < a.Ncols) a.slab[((size_t)kz * a.M + m) * a.Ncols + col] = acc[fm][fn][r];
          }
        }
    }
    return;
  }
  // Epilogue order: mask loads, values and column sums in registers, the
  // column-sum exchange (LDS + barrier), THEN the global stores. A barrier
  // after the stores would wait for their acknowledgements (vmcnt counts
  // stores on CDNA) before the column sums could be combined.
  float cs[FN];
#pragma unroll
  for (int fn = 0; fn < FN; ++fn) cs[fn] = 0.f;
  int grow[FM][4];
  bool rok[FM][4];
  if (epi) {
    float bv[FN];
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int col = cbase + fn * 16;
      bv[fn] = (a.bias && col < a.Ncols) ? a.bias[col] : 0.f;
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = rbase + fm * 16 + r;
        rok[fm][r] = m < a.M;
        if constexpr (MODE == kModeConv) {
          grow[fm][r] = m;
        } else {
          const uint32_t mm = rok[fm][r] ? (uint32_t)m : 0u;
          const uint32_t n = fdiv(mm, a.f_pix);
          const uint32_t rem = mm - n * a.f_pix.d;
          const uint32_t yy = fdiv(rem, a.f_w);
          const uint32_t xx = rem - yy * a.f_w.d;
          grow[fm][r] = ((int)n * d.H + (int)yy * d.S + oa) * d.W + (int)xx * d.S + ob;
        }
      }
    }
    float mk[FM][4][FN];
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int col = cbase + fn * 16;
          const bool ok = rok[fm][r] && col < a.Ncols;
          mk[fm][r][fn] = (a.omask && ok) ? (float)a.omask[(size_t)grow[fm][r] * a.Ncols + col] : 1.f;
        }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int col = cbase + fn * 16;
          const bool ok = rok[fm][r] && col < a.Ncols;
          float v = acc[fm][fn][r] + bv[fn];
          if (a.relu) v = fmaxf(v, 0.f);
          v = mk[fm][r][fn] > 0.f ? v : 0.f;
          acc[fm][fn][r] = v;
          cs[fn] += ok ? v : 0.f;
        }
  }
  float* sc = reinterpret_cast<float*>(lds + TC::RED_BYTES);
  if (a.colsum) {
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      cs[fn] += __shfl_xor(cs[fn], 16, 64);
      cs[fn] += __shfl_xor(cs[fn], 32, 64);
    }
    if (epi && lane < 16) {
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) sc[wm * BN + wn * (BN / WN) + fn * 16 + lane] = cs[fn];
    }
    __syncthreads();
  }
  if (epi) {
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int col = cbase + fn * 16;
          if (rok[fm][r] && col < a.Ncols) {
            const size_t o = (size_t)grow[fm][r] * a.Ncols + col;
            if (a.y16) a.y16[o] = (__bf16)acc[fm][fn][r];
            if (a.y32) a.y32[o] = acc[fm][fn][r];
          }
        }
  }
  if (a.colsum && tid < BN) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < WM; ++q) t += sc[q * BN + tid];
    const int col = nt * BN + tid;
    if (col < a.Ncols) a.colsum[(size_t)(cls * a.mtiles + mt) * a.Ncols + col] = t;
  }
}

// Register-prefetch depth of the k-loops: k-tiles whose global loads are in
// flight while the MFMAs of the current LDS tile run. One: a 3-deep ring for
// small tiles / 2-deep for large ones measured 0.4-1.4 us SLOWER per conv GEMM
// on MI355X (113-134 VGPRs instead of 64-78; profiles/r1_conv_jobs/README.md).
__device__ __forceinline__ void kloop_barrier() { __syncthreads(); }
template <int STAGE_REGS>
constexpr int prefetch_depth() {
  return 1;
}
template <class TC>
constexpr int ig_prefetch() { return prefetch_depth<TC::BM / 32 + (TC::BN * 8 + 255) / 256>(); }
template <int A_CH, int B_CH>
constexpr int wg_prefetch() { return prefetch_depth<A_CH + B_CH>(); }

template <class TC>
constexpr int igemm_lds_bytes() { return 2 * (TC::BM * 128 + TC::BN * 128); }

// Block body of the forward-type GEMM: tile `tb` of `ntb` (m x n tiles of one
// (k-split, class) plane), k-split `kz`, parity class `cls`. `lds` holds
// igemm_lds_bytes<TC>() bytes. Shared by the stand-alone kernel and the
// horizontally fused job kernels (conv_jobs.h).
template <int MODE, typename AT, bool VEC, class TC, bool PRO = false>
__device__ __forceinline__ void igemm_body(const IgArgs& a, uint8_t* lds, int tb, int ntb, int kz, int cls) {
  constexpr int BM = TC::BM, BN = TC::BN, WM = TC::WM, WN = TC::WN, KWS = TC::KWS, FM = TC::FM, FN = TC::FN;
  constexpr int A_CH = BM / 32;                // 16-B chunks per thread of the BM x 64 A tile
  constexpr int B_CH = (BN * 8 + 255) / 256;   // ... of the BN x 64 B tile
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  static_assert(TC::RED_BYTES + WM * BN * 4 <= 2 * STAGE, "epilogue scratch exceeds LDS");
  static_assert(VEC || MODE == kModeConv, "thin gathers exist for conv mode only");

  const ConvDesc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = w / (WM * WN), wm = (w % (WM * WN)) / WN, wn = w % WN;
  const int tile = xcd_remap(tb, ntb);
  const int mt = tile / a.ntiles, nt = tile - mt * a.ntiles;
  const int kt0 = kz * a.kt_per_split;
  const int kt1 = min(a.ktiles, kt0 + a.kt_per_split);

  int ea = 0, eb = 0, oa = 0, ob = 0;
  if constexpr (MODE == kModeTconv) {
    const int ca = cls / d.S, cb = cls - ca * d.S;
    oa = ((ca - d.P) % d.S + d.S) % d.S;
    ob = ((cb - d.P) % d.S + d.S) % d.S;
    ea = (oa + d.P - ca) / d.S;
    eb = (ob + d.P - cb) / d.S;
  }

  // ---- per-thread staging coordinates (fixed for the whole k loop)
  const int ach = tid & 7;
  int abase[A_CH], ay[A_CH], ax[A_CH];
  bool aok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int m = mt * BM + (tid >> 3) + 32 * i;
    aok[i] = m < a.M;
    const uint32_t mm = aok[i] ? (uint32_t)m : 0u;
    const uint32_t n = fdiv(mm, a.f_pix);
    const uint32_t rem = mm - n * a.f_pix.d;
    const uint32_t yy = fdiv(rem, a.f_w);
    const uint32_t xx = rem - yy * a.f_w.d;
    if constexpr (MODE == kModeConv) {
      abase[i] = (int)n * d.H * d.W * d.C;
      ay[i] = (int)yy * d.S - d.P;
      ax[i] = (int)xx * d.S - d.P;
    } else {
      abase[i] = (int)n * d.OH * d.OW * d.CO;
      ay[i] = (int)yy + ea;
      ax[i] = (int)xx + eb;
    }
  }
  const AT* Ap = reinterpret_cast<const AT*>(a.A);
  const __bf16* Bc = a.B + (size_t)cls * a.Ncols * a.K;

  // register prefetch ring: PF k-tiles in flight ahead of the LDS stage
  constexpr int PF = ig_prefetch<TC>();
  // Out-of-range chunks load from a valid address and are zeroed when staged
  // to LDS (bit i of `okm`: A chunk i, bit 16+i: B chunk i), so the loaded
  // registers are not consumed until the LDS store: a select on them right
  // after the load would wait for it and serialise every k-step.
  bf16x8 ra_s[PF][A_CH], rb_s[PF][B_CH];
  uint32_t okm_s[PF];
  auto gload = [&](int kt, bf16x8 (&ra)[A_CH], bf16x8 (&rb)[B_CH], uint32_t& okm) {
    const int kk = kt * 64 + 8 * ach;
    okm = 0u;
    if constexpr (VEC) {
      const uint32_t tap = fdiv((uint32_t)kk, a.f_ch);
      const int ch = kk - (int)(tap * a.f_ch.d);
      const uint32_t t0 = fdiv(tap, a.f_tw);
      const int t1 = (int)(tap - t0 * a.f_tw.d);
      const bool kok = kk < a.K;
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
        int off;
        bool ok;
        if constexpr (MODE == kModeConv) {
          const int iy = ay[i] + (int)t0, ix = ax[i] + t1;
          ok = aok[i] && kok && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
          off = abase[i] + (iy * d.W + ix) * d.C + ch;
        } else {
          const int oy = ay[i] - (int)t0, ox = ax[i] - t1;
          ok = aok[i] && kok && (unsigned)oy < (unsigned)d.OH && (unsigned)ox < (unsigned)d.OW;
          off = abase[i] + (oy * d.OW + ox) * d.CO + ch;
        }
        if constexpr (PRO) {
          // split-K combine of the producing layer (fixed slab order: deterministic)
          const size_t o = ok ? (size_t)off : 0;
          const int c0 = (int)(o % (size_t)a.pro.cin);
          f32x4 s0 = *reinterpret_cast<const f32x4*>(a.pro.bias + c0);
          f32x4 s1 = *reinterpret_cast<const f32x4*>(a.pro.bias + c0 + 4);
          for (int z = 0; z < a.pro.ks; ++z) {
            const float* q = a.pro.slab + (size_t)z * a.pro.stride + o;
            s0 += *reinterpret_cast<const f32x4*>(q);
            s1 += *reinterpret_cast<const f32x4*>(q + 4);
          }
          bf16x8 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            v[j] = (__bf16)(a.pro.relu ? fmaxf(s0[j], 0.f) : s0[j]);
            v[4 + j] = (__bf16)(a.pro.relu ? fmaxf(s1[j], 0.f) : s1[j]);
          }
          ra[i] = v;
          if (ok && nt == 0) *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.pro.out16) + o) = v;
        } else {
          ra[i] = load_chunk<AT>(Ap + (ok ? off : 0));
        }
        okm |= (uint32_t)ok << i;
      }
    } else {
      okm = (1u << A_CH) - 1u;  // per-element gathers are zeroed in place
      float v[A_CH][8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = kk + j;
        const uint32_t tap = fdiv((uint32_t)k, a.f_ch);
        const int ch = k - (int)(tap * a.f_ch.d);
        const uint32_t ky = fdiv(tap, a.f_tw);
        const int kx = (int)(tap - ky * a.f_tw.d);
        const bool kok = k < a.K;
#pragma unroll
        for (int i = 0; i < A_CH; ++i) {
          const int iy = ay[i] + (int)ky, ix = ax[i] + kx;
          const bool ok = aok[i] && kok && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
          const float x = (float)Ap[ok ? abase[i] + (iy * d.W + ix) * d.C + ch : 0];
          v[i][j] = ok ? x : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < A_CH; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ra[i][j] = (__bf16)v[i][j];
      }
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const int col = nt * BN + r;
      const bool ok = r < BN && col < a.Ncols && kk < a.K;
      rb[i] = load_chunk<__bf16>(Bc + (ok ? (size_t)col * a.K + kk : 0));
      okm |= (uint32_t)ok << (16 + i);
    }
  };
  auto sstore = [&](int buf, const bf16x8 (&ra)[A_CH], const bf16x8 (&rb)[B_CH], uint32_t okm) {
    uint8_t* As = lds + buf * STAGE;
    uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *reinterpret_cast<bf16x8*>(As + rimg(r, ach)) = ((okm >> i) & 1u) ? ra[i] : zero8();
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int r = (tid >> 3) + 32 * i;
      if (r < BN) *reinterpret_cast<bf16x8*>(Bs + rimg(r, ach)) = ((okm >> (16 + i)) & 1u) ? rb[i] : zero8();
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint8_t* As = lds + buf * STAGE;
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int s = (KWS == 2 ? 0 : 0); s < 2 / KWS; ++s) {
      const int ks = KWS == 2 ? wk : s;
      const int ch = ks * 4 + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
        af[fm] = *reinterpret_cast<const bf16x8*>(As + rimg(wm * (BM / WM) + fm * 16 + (lane & 15), ch));
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        bfr[fn] = *reinterpret_cast<const bf16x8*>(Bs + rimg(wn * (BN / WN) + fn * 16 + (lane & 15), ch));
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = mfma_bf16(af[fm], bfr[fn], acc[fm][fn]);
    }
  };

#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (kt0 + p < kt1) gload(kt0 + p, ra_s[p], rb_s[p], okm_s[p]);
  if (kt0 < kt1) sstore(0, ra_s[0], rb_s[0], okm_s[0]);
  __syncthreads();
  for (int kb = kt0; kb < kt1; kb += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int kt = kb + p;
      if (kt < kt1) {
        const int buf = (kt - kt0) & 1;
        if (kt + PF < kt1) gload(kt + PF, ra_s[p], rb_s[p], okm_s[p]);  // slot p's tile is already in LDS
        compute(buf);
        if (kt + 1 < kt1) sstore(buf ^ 1, ra_s[(p + 1) % PF], rb_s[(p + 1) % PF], okm_s[(p + 1) % PF]);
        kloop_barrier();
      }
    }
  }

  igemm_epilogue<MODE, TC>(a, acc, lds, mt, nt, kz, cls, oa, ob);
}

template <int MODE, typename AT, bool VEC, class TC, bool PRO = false>
__global__ void __launch_bounds__(256) igemm_fwd_k(IgArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[igemm_lds_bytes<TC>()];
  igemm_body<MODE, AT, VEC, TC, PRO>(a, lds, blockIdx.x, gridDim.x, blockIdx.y, blockIdx.z);
}

// ---------------------------------------------------------- LDS-DMA helpers ----
// Zero source for out-of-range chunks of an LDS-DMA tile load (static device
// memory is zero-initialised): a global_load_lds has no per-lane predicate, so
// masked lanes fetch 16 zero bytes instead.
static __device__ __attribute__((aligned(64))) uint8_t g_zero16[64];

// Issued through inline asm: the compiler's waitcnt pass counts a
// __builtin_amdgcn_global_load_lds as an out-of-order LGKM event, so with one
// in flight every later LDS read is followed by s_waitcnt lgkmcnt(0) (a k loop
// then waits out the reads issued for the NEXT k-step before each MFMA;
// profiles/r2_dconv/waitcnt). The hardware counts the DMA on vmcnt only, and
// every user waits for it explicitly (dc_wait_stages) before a
// barrier. `lds_base` must be wave-uniform.
__device__ __forceinline__ void glds16(const void* src, uint8_t* lds_base) {
  const uint32_t l = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_base;
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               ::"s"(__builtin_amdgcn_readfirstlane(l)), "v"(src) : "memory");
}

// Workgroup barrier that neither drains the LDS-DMA queue (unlike
// __syncthreads, whose fence waits vmcnt(0)) nor lets this wave's LDS reads
// of the previous stage still be in flight.
__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ================================================================= wgrad ====
struct WgArgs {
  ConvDesc d;
  const __bf16* G;  // [M][CO]
  const void* X;    // NHWC conv input
  float* out;       // [nsplit][CO][K2]
  int M, K2, cotiles, ktiles, mtiles, mt_per_split;
  FastDiv f_pix, f_w, f_c, f_kw;
};

// Epilogue of the weight-gradient kernels: combine k-halves, store the f32
// partial tile of this m-split.
template <class TC>
__device__ __forceinline__ void wgrad_epilogue(const WgArgs& a, f32x4 (&acc)[TC::FM][TC::FN], uint8_t* lds, int ct,
                                               int nt, int split) {
  constexpr int BM = TC::BM, BN = TC::BN, WM = TC::WM, WN = TC::WN, KWS = TC::KWS, FM = TC::FM, FN = TC::FN;
  const ConvDesc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = w / (WM * WN), wm = (w % (WM * WN)) / WN, wn = w % WN;
  if constexpr (KWS == 2) {
    float* red = reinterpret_cast<float*>(lds);
    const int slot = w % (WM * WN);
    if (wk == 1) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          *reinterpret_cast<f32x4*>(red + (((slot * FM + fm) * FN + fn) * 64 + lane) * 4) = acc[fm][fn];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
          acc[fm][fn] += *reinterpret_cast<const f32x4*>(red + (((slot * FM + fm) * FN + fn) * 64 + lane) * 4);
    }
  }
  if (KWS == 1 || wk == 0) {
    float* out = a.out + (size_t)split * d.CO * a.K2;
    if ((a.K2 & 3) == 0) {
      // The partial slab leaves through 16-B write-through (sc1) buffer stores:
      // plain 4-B stores left ~MBs of dirty L2 lines for the end-of-kernel
      // write-back, a tail after the last wave (removing the slab stores cut
      // the 28x28 weight-gradient launch 9.7 -> 7.6 us, profiles/r5_wt_stores).
      // Each 16x16 fragment goes through a wave-private LDS tile (row pitch 20
      // floats) so a lane holds 4 consecutive columns of one row.
      static_assert(TC::RED_BYTES + 4 * 16 * 20 * 4 <= 2 * (64 * TC::BM * 2 + 64 * TC::BN * 2),
                    "wgrad store staging exceeds wgrad_lds_bytes");
      float* stg = reinterpret_cast<float*>(lds + TC::RED_BYTES) + (w & 3) * 16 * 20;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, d.CO * a.K2 * 4, 0x00020000);
      typedef unsigned uvec4 __attribute__((ext_vector_type(4)));
      const int rr = lane >> 2, cq = lane & 3;
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[(4 * (lane >> 4) + r) * 20 + (lane & 15)] = acc[fm][fn][r];
          __builtin_amdgcn_wave_barrier();  // one wave's LDS ops run in order; keep the compiler's too
          const f32x4 v = *reinterpret_cast<const f32x4*>(stg + rr * 20 + 4 * cq);
          __builtin_amdgcn_wave_barrier();
          const int orow = ct * BM + wm * (BM / WM) + fm * 16 + rr;
          const int kp = nt * BN + wn * (BN / WN) + fn * 16 + 4 * cq;
          if (orow < d.CO && kp < a.K2)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uvec4, v), rs, (orow * a.K2 + kp) * 4, 0,
                                                   16 /* sc1 */);
        }
      return;
    }
#pragma unroll
    for (int fm = 0; fm < FM; ++fm)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int orow = ct * BM + wm * (BM / WM) + fm * 16 + 4 * (lane >> 4) + r;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int kp = nt * BN + wn * (BN / WN) + fn * 16 + (lane & 15);
          if (orow < d.CO && kp < a.K2) out[(size_t)orow * a.K2 + kp] = acc[fm][fn][r];
        }
      }
  }
}

template <class TC>
constexpr int wgrad_lds_bytes() { return 2 * (64 * TC::BM * 2 + 64 * TC::BN * 2); }

// Block body of the weight-gradient GEMM (block `bid` of `nblk`); `lds` holds
// wgrad_lds_bytes<TC>() bytes.
template <typename XT, bool VEC, class TC>
__device__ __forceinline__ void wgrad_body(const WgArgs& a, uint8_t* lds, int bid, int nblk) {
  constexpr int BM = TC::BM, BN = TC::BN, WM = TC::WM, WN = TC::WN, KWS = TC::KWS, FM = TC::FM, FN = TC::FN;
  constexpr int CPR_A = BM / 8, A_RPP = 256 / CPR_A, A_CH = 64 / A_RPP;
  constexpr int CPR_B = BN / 8, B_RPP = 256 / CPR_B, B_CH = (64 + B_RPP - 1) / B_RPP;
  constexpr int A_BYTES = 64 * BM * 2, B_BYTES = 64 * BN * 2, STAGE = A_BYTES + B_BYTES;
  static_assert(TC::RED_BYTES <= 2 * STAGE, "reduction scratch exceeds LDS");

  const ConvDesc& d = a.d;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = w / (WM * WN), wm = (w % (WM * WN)) / WN, wn = w % WN;
  // 1-D grid, split-major after the XCD remap: an XCD owns a contiguous
  // m-range for ALL (co, k') tiles, so its slice of G and X is fetched into
  // its L2 once instead of once per tile.
  const int wid = xcd_remap(bid, nblk);
  const int ntile = a.cotiles * a.ktiles;
  const int split = wid / ntile;
  const int tile = wid - split * ntile;
  const int ct = tile / a.ktiles, nt = tile - ct * a.ktiles;
  const int mt0 = split * a.mt_per_split;
  const int mt1 = min(a.mtiles, mt0 + a.mt_per_split);

  const int cha = tid % CPR_A, ra0 = tid / CPR_A;
  const int co = ct * BM + 8 * cha;
  const bool coka = co < d.CO;
  const int chb = tid % CPR_B, rb0 = tid / CPR_B;
  const XT* Xp = reinterpret_cast<const XT*>(a.X);
  const int HWC = d.H * d.W * d.C;

  // B-operand column coordinates (fixed per thread)
  int kyv[VEC ? 1 : 8], kxv[VEC ? 1 : 8], civ[VEC ? 1 : 8];
  bool kokv[VEC ? 1 : 8];
#pragma unroll
  for (int j = 0; j < (VEC ? 1 : 8); ++j) {
    const int kp = nt * BN + 8 * chb + j;
    kokv[j] = kp < a.K2;
    const uint32_t tap = fdiv((uint32_t)(kokv[j] ? kp : 0), a.f_c);
    civ[j] = (kokv[j] ? kp : 0) - (int)(tap * a.f_c.d);
    const uint32_t ky = fdiv(tap, a.f_kw);
    kyv[j] = (int)ky;
    kxv[j] = (int)(tap - ky * a.f_kw.d);
  }

  constexpr int PF = wg_prefetch<A_CH, B_CH>();
  // masks applied at the LDS store (see igemm_body)
  bf16x8 ra_s[PF][A_CH], rb_s[PF][B_CH];
  uint32_t okm_s[PF];
  auto gload = [&](int mtile, bf16x8 (&ra)[A_CH], bf16x8 (&rb)[B_CH], uint32_t& okm) {
    okm = 0u;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int m = mtile * 64 + ra0 + A_RPP * i;
      const bool ok = coka && m < a.M;
      ra[i] = load_chunk<__bf16>(a.G + (ok ? (size_t)m * d.CO + co : 0));
      okm |= (uint32_t)ok << i;
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int r = rb0 + B_RPP * i;
      const int m = mtile * 64 + r;
      const bool mok = r < 64 && m < a.M;
      const uint32_t mm = mok ? (uint32_t)m : 0u;
      const uint32_t n = fdiv(mm, a.f_pix);
      const uint32_t rem = mm - n * a.f_pix.d;
      const uint32_t oy = fdiv(rem, a.f_w);
      const uint32_t ox = rem - oy * a.f_w.d;
      const int iy0 = (int)oy * d.S - d.P, ix0 = (int)ox * d.S - d.P;
      if constexpr (VEC) {
        const int iy = iy0 + kyv[0], ix = ix0 + kxv[0];
        const bool ok = mok && kokv[0] && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
        rb[i] = load_chunk<XT>(Xp + (ok ? (int)n * HWC + (iy * d.W + ix) * d.C + civ[0] : 0));
        okm |= (uint32_t)ok << (16 + i);
      } else {
        okm |= 1u << (16 + i);  // per-element gathers are zeroed in place
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int iy = iy0 + kyv[j], ix = ix0 + kxv[j];
          const bool ok = mok && kokv[j] && (unsigned)iy < (unsigned)d.H && (unsigned)ix < (unsigned)d.W;
          const float x = (float)Xp[ok ? (int)n * HWC + (iy * d.W + ix) * d.C + civ[j] : 0];
          v[j] = ok ? x : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) rb[i][j] = (__bf16)v[j];
      }
    }
  };
  auto sstore = [&](int buf, const bf16x8 (&ra)[A_CH], const bf16x8 (&rb)[B_CH], uint32_t okm) {
    uint8_t* As = lds + buf * STAGE;
    uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int r = ra0 + A_RPP * i;
      *reinterpret_cast<bf16x8*>(As + timg<BM>(r, cha)) = ((okm >> i) & 1u) ? ra[i] : zero8();
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int r = rb0 + B_RPP * i;
      if (r < 64) *reinterpret_cast<bf16x8*>(Bs + timg<BN>(r, chb)) = ((okm >> (16 + i)) & 1u) ? rb[i] : zero8();
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const uint8_t* As = lds + buf * STAGE;
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2 / KWS; ++s) {
      const int kb = 32 * (KWS == 2 ? wk : s);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int fm = 0; fm < FM; ++fm) af[fm] = tr_frag<BM>(As, wm * (BM / WM) + 16 * fm, kb, lane);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) bfr[fn] = tr_frag<BN>(Bs, wn * (BN / WN) + 16 * fn, kb, lane);
#pragma unroll
      for (int fm = 0; fm < FM; ++fm)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = mfma_bf16(af[fm], bfr[fn], acc[fm][fn]);
    }
  };

#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (mt0 + p < mt1) gload(mt0 + p, ra_s[p], rb_s[p], okm_s[p]);
  if (mt0 < mt1) sstore(0, ra_s[0], rb_s[0], okm_s[0]);
  __syncthreads();
  for (int mb = mt0; mb < mt1; mb += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int mtile = mb + p;
      if (mtile < mt1) {
        const int buf = (mtile - mt0) & 1;
        if (mtile + PF < mt1) gload(mtile + PF, ra_s[p], rb_s[p], okm_s[p]);
        compute(buf);
        if (mtile + 1 < mt1) sstore(buf ^ 1, ra_s[(p + 1) % PF], rb_s[(p + 1) % PF], okm_s[(p + 1) % PF]);
        kloop_barrier();
      }
    }
  }

  wgrad_epilogue<TC>(a, acc, lds, ct, nt, split);
}

template <typename XT, bool VEC, class TC>
__global__ void __launch_bounds__(256) wgrad_k(WgArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[wgrad_lds_bytes<TC>()];
  wgrad_body<XT, VEC, TC>(a, lds, blockIdx.x, gridDim.x);
}

// ======================================================= small reductions ====
// Split-K combine: y = sum_z slab[z] + bias (+relu) -> f32 and/or bf16.
// `cnt` outputs per block, 256/cnt threads per output summing interleaved
// z slices (independent loads in flight), then a fixed-order LDS combine.
struct CombineArgs {
  const float* slab;
  int ksplit, M, N, cnt;
  const float* bias;
  int relu;
  float* y32;
  __bf16* y16;
};

__device__ __forceinline__ void splitk_combine_body(const CombineArgs& c, float* red, int bid) {
  const int t = threadIdx.x, rp = 256 / c.cnt, col = t % c.cnt, rl = t / c.cnt;
  const long long MN = (long long)c.M * c.N;
  const long long e = (long long)bid * c.cnt + col;
  float v = 0.f;
  if (rl < rp && e < MN) {
#pragma unroll 4
    for (int z = rl; z < c.ksplit; z += rp) v += c.slab[(size_t)z * MN + e];
  }
  red[t] = v;
  __syncthreads();
  if (rl == 0 && e < MN) {
    float acc = 0.f;
    for (int r = 0; r < rp; ++r) acc += red[r * c.cnt + col];
    if (c.bias) acc += c.bias[e % c.N];
    if (c.relu) acc = fmaxf(acc, 0.f);
    if (c.y32) c.y32[e] = acc;
    if (c.y16) c.y16[e] = (__bf16)acc;
  }
}


// Column sums of a bf16 [M][N] matrix (N % 8 == 0): partial row y of `slab`
// ([gy][N]) sums rows [y*rows_per, (y+1)*rows_per). Block (x, y) = bid.
struct ColsumArgs {
  const __bf16* G;
  int M, N, rows_per, gx;
  float* slab;
};

__device__ __forceinline__ void colsum_body(const ColsumArgs& c, int bid) {
  const int by = bid / c.gx, bx = bid - by * c.gx;
  const int c8 = bx * 256 + threadIdx.x;
  if (c8 * 8 >= c.N) return;
  const int r0 = by * c.rows_per, r1 = min(c.M, r0 + c.rows_per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int r = r0; r < r1; ++r) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(c.G + (size_t)r * c.N + 8 * c8);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += (float)v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) c.slab[(size_t)by * c.N + 8 * c8 + j] = s[j];
}


namespace tiles {
// forward-type tile configurations
using F0 = TileCfg<128, 128, 2, 2>;
using F1 = TileCfg<128, 64, 2, 2>;
using F2 = TileCfg<128, 32, 4, 1>;
using F3 = TileCfg<128, 16, 4, 1>;
using F4 = TileCfg<64, 128, 2, 2>;
using F5 = TileCfg<64, 64, 2, 2>;
using F6 = TileCfg<64, 32, 2, 1>;
using F7 = TileCfg<64, 16, 4, 1>;
// weight-gradient tile configurations (co x k'), capped at 64x64 so the
// m-split partial slabs stay small (slab bytes ~ blocks x BM x BN x 4)
using W0 = TileCfg<64, 64, 2, 2>;
using W1 = TileCfg<64, 32, 2, 1>;
using W2 = TileCfg<64, 16, 4, 1>;
using W3 = TileCfg<32, 64, 2, 2>;
using W4 = TileCfg<32, 32, 2, 1>;
using W5 = TileCfg<32, 16, 2, 1>;

}  // namespace tiles

// Host-side builders shared by the stand-alone entry points (conv_igemm.hip)
// and the job builders (conv_jobs.hip).
bool plan_fwd(int mode, const ConvDesc& d, bool allow_split, FwdPlan* p, bool allow_direct = true,
              bool fwd = false);
int direct_cfg(int mode, const ConvDesc& d, bool fwd);
int dwgrad_cfg(const ConvDesc& d);
bool plan_wgrad(const ConvDesc& d, WgradPlan* p);
// Kernel arguments of one forward-type GEMM; with split-K (q->ksplit > 1) `c`
// receives the combine pass (nc = its block count), else nc = 0.
int build_igemm(int mode, const void* A, const void* B16, ConvDesc d, const float* bias, int relu, void* y16,
                float* y32, const void* omask, float* colsum, float* ws, IgArgs* a, FwdPlan* q, CombineArgs* c,
                int* nc);
int build_wgrad(const void* G16, const void* X, ConvDesc d, float* out, WgArgs* a, WgradPlan* q);
int launch_splitk_combine(const CombineArgs& c, int nblk, hipStream_t s);

}  // namespace mdt
