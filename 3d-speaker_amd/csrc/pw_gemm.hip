// Persistent 1x1-conv (pointwise) GEMM for short K, fp16x3 MFMA, gfx950.
//
// The Res2Net 1x1 convs of ERes2Net(V2) stages 1-2 (K = 52..128, N = 56..256 on ~4 M
// pixels per batch) move 3-4 bytes of activations per FLOP: they are HBM-bound, and a
// tile-per-block GEMM spends most of each block's life waiting on two or three serialized
// memory round trips (operand tile, residual, store).  Here one block per CU keeps
//   * its N-slice of the weights resident in LDS as fp16 hi / lo planes (split once at
//     model creation, conv_gemm.hip "fp16x3"),
//   * the next TWO M-tiles of activations in flight in registers (two register sets),
//   * the current tile's residual in flight during its MFMAs,
// and walks M-tiles with a stride of the grid, so loads of later tiles overlap the
// compute and the stores of the current one.
//
// Tile: BM = 32*WM rows x BN = 32*WN columns, 8 waves (WM x WN), wave tile 32x32.  The A
// tile is split into fp16 hi / lo planes when it is staged into LDS (rows of KP+8 halves:
// conflict-free ds_read_b128).  Epilogue straight from the MFMA C layout (lane = column):
// each store instruction writes two full 128-B row segments.
#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>

#include <atomic>

#include "common.h"
#include "conv_epilogue.h"

namespace spk {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

template <int KP, int BN>
struct PwCfg {
  static constexpr int NT = 512, WN = BN / 32, WM = 8 / WN, BM = 32 * WM;
  static constexpr int LROW = KP + 8;                      // halves per LDS row
  static constexpr int QR = KP / 4;                        // float4 per A row
  static constexpr int AQ = BM * QR / NT;                  // float4 staged per thread per tile
  static constexpr int B_HALVES = 2 * BN * LROW;           // hi + lo weight planes
  static constexpr int A_HALVES = 2 * BM * LROW;           // hi + lo activation planes
  static constexpr int LDS_FLOATS = (B_HALVES + A_HALVES) / 2;
  static_assert(BM * QR % NT == 0, "A tile must split evenly over the block");
};

// RES (compile time): the layer adds a residual.  Inside the persistent loop every load
// must be one the compiler can count: a load behind a runtime `d.res ?` (or the ragged-row
// mask's length load) makes it wait vmcnt(0) -- for the whole two-tile prefetch -- at each
// use, which serialised the loop (ISA: sixteen such waits per tile).
template <int KP, int BN, bool S1, bool RES>
__global__ void __launch_bounds__(512, 1)
pw_gemm_x3_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
  // scaled split (common.h): operand x 2^-s at staging, accumulators x 2^s in the epilogue
  const float sc = range_scale_flat(d.range_in), back = pow2_div(sc, 0), back_x = pow2_div(sc, -11);
  using C = PwCfg<KP, BN>;
  __shared__ __attribute__((aligned(16))) float lds[C::LDS_FLOATS];
  _Float16* Bh = reinterpret_cast<_Float16*>(lds);
  _Float16* Bl = Bh + BN * C::LROW;
  _Float16* Ah = Bh + C::B_HALVES;
  _Float16* Al = Ah + C::BM * C::LROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + BN - 1) / BN;
  // the nN blocks of one M-tile walk get neighbouring logical ids, i.e. one XCD: the A
  // tiles they all read come from one L2
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = bid % nN;                                 // this block's N-slice (fixed)
  const int n0 = nb * BN;
  const int mtiles = (M + C::BM - 1) / C::BM;
  const int mstride = gridDim.x / nN;
  const int mt0 = bid / nN;
  const int K0 = d.s0.cin;                                 // s0 channels, then s1 (S1)
  const int K = d.K;
  // strided 1x1 (CAM++ FCM projection shortcut, frequency stride 2): output pixel m reads
  // input pixel (img, ho * sh, wo * sw); the s0 address of a row is re-derived from m
  const bool strided = d.s0.sh != 1 || d.s0.sw != 1;
  const int HoWo = d.Ho * d.Wo;

  // ---- weights of the N-slice -> LDS (once)
  for (int idx = tid; idx < BN * (KP / 8); idx += C::NT) {
    const int n = idx / (KP / 8), c = idx % (KP / 8);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 h = {0u, 0u, 0u, 0u}, l = {0u, 0u, 0u, 0u};
    if (n0 + n < d.N) {
      h = *reinterpret_cast<const u32x4*>(d.wh + (size_t)(n0 + n) * d.Kp + c * 8);
      l = *reinterpret_cast<const u32x4*>(d.wl + (size_t)(n0 + n) * d.Kp + c * 8);
    }
    *reinterpret_cast<u32x4*>(Bh + n * C::LROW + c * 8) = h;
    *reinterpret_cast<u32x4*>(Bl + n * C::LROW + c * 8) = l;
  }

  // ---- A staging: float4 i of this thread = (row, quad) of the tile
  auto load_a = [&](int mt, f32x4 (&v)[C::AQ]) {
#pragma unroll
    for (int i = 0; i < C::AQ; ++i) {
      const int idx = tid + C::NT * i;
      const int row = idx / C::QR, q = idx % C::QR;
      int m = mt * C::BM + row;
      m = m < M ? m : M - 1;
      int m0r = m;                                         // s0 row of output pixel m
      if (strided) {
        const int img = m / HoWo, rem = m - img * HoWo, ho = rem / d.Wo, wo = rem - ho * d.Wo;
        m0r = (img * d.s0.H + ho * d.s0.sh) * d.s0.W + wo * d.s0.sw;
      }
      const int k = 4 * q;
      const float* src;
      if (S1 && k >= K0) src = d.s1.p + (size_t)m * d.s1.ld + min(k - K0, d.s1.cin - 4);
      else src = d.s0.p + (size_t)m0r * d.s0.ld + min(k, K0 - 4);
      v[i] = *reinterpret_cast<const f32x4*>(src);
    }
  };
  auto store_a = [&](const f32x4 (&v)[C::AQ]) {
    split_pass(sc, [&](auto split) {                       // scaled split (common.h) when the word is set
#pragma unroll
      for (int i = 0; i < C::AQ; ++i) {
        const int idx = tid + C::NT * i;
        const int row = idx / C::QR, q = idx % C::QR;
        const bool kin = 4 * q < K;                        // K padding columns are zero
        f16x4 h, l;
        split(kin ? v[i] : f32x4{0.f, 0.f, 0.f, 0.f}, h, l);
        *reinterpret_cast<f16x4*>(Ah + row * C::LROW + 4 * q) = h;
        *reinterpret_cast<f16x4*>(Al + row * C::LROW + 4 * q) = l;
      }
    });
  };

  const int n = n0 + wn * 32 + li;                         // this lane's output column
  const bool nok = n < d.N;
  float* const ocol = out_at(d, 0, nok ? n : 0);           // its plane / offset, once
  const float bias = (nok && d.bias) ? d.bias[n] : 0.f;
  const float ps = (nok && d.post_scale) ? d.post_scale[n] : 1.f;
  const float pt = (nok && d.post_scale) ? d.post_shift[n] : 0.f;

  // residual of a tile: requested BEFORE the A prefetch of tile i+2 -- vmcnt retires
  // loads in order, so the epilogue's wait for it then does not also wait for the prefetch
  auto load_res = [&](int mt, float (&res)[16]) {
    const int mbase = mt * C::BM + wm * 32 + 4 * lh;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      int m = mbase + (r & 3) + 8 * (r >> 2);
      m = m < M ? m : M - 1;
      res[r] = RES ? d.res[(size_t)m * d.ldr + (nok ? n : 0)] : 0.f;
    }
  };
  auto tile = [&](int mt, const float (&res)[16]) {
    const int mbase = mt * C::BM + wm * 32 + 4 * lh;
    f32x16 acc, accx;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[r] = 0.f; accx[r] = 0.f; }
    const _Float16* a = Ah + (wm * 32 + li) * C::LROW + 8 * lh;
    const _Float16* b = Bh + (wn * 32 + li) * C::LROW + 8 * lh;
#pragma unroll
    for (int s = 0; s < KP / 16; ++s) {
      const f16x8 ah = *reinterpret_cast<const f16x8*>(a + 16 * s);
      const f16x8 al = *reinterpret_cast<const f16x8*>(a + 16 * s + C::BM * C::LROW);
      const f16x8 bh = *reinterpret_cast<const f16x8*>(b + 16 * s);
      const f16x8 bl = *reinterpret_cast<const f16x8*>(b + 16 * s + BN * C::LROW);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc, 0, 0, 0);
      accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, accx, 0, 0, 0);
      accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, accx, 0, 0, 0);
    }
    if (nok) {
      float amax = 0.f;
      // the activation resolved once per tile: compile-time forms for the common layers
      auto rows = [&](auto actc) {
        constexpr int A = decltype(actc)::value;   // -1: general
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mbase + (r & 3) + 8 * (r >> 2);
          if (m >= M) continue;
          float v = acc[r] * back + accx[r] * back_x + bias + res[r];
          if constexpr (A >= 0) {
            v = apply_act(v, A);
          } else {
            v = apply_act(v, d.act);
            if (d.post_scale) v = v * ps + pt;
            v = apply_act(v, d.act2);                      // no ragged rows (pw_supported)
          }
          amax = fmaxf(amax, fabsf(v));
          ocol[(size_t)m * d.ldo] = v;
        }
      };
      const bool simple = !d.post_scale && d.act2 == ACT_NONE;
      if (simple && d.act == ACT_HTANH) rows(std::integral_constant<int, ACT_HTANH>{});
      else if (simple && d.act == ACT_RELU) rows(std::integral_constant<int, ACT_RELU>{});
      else if (simple && d.act == ACT_NONE) rows(std::integral_constant<int, ACT_NONE>{});
      else rows(std::integral_constant<int, -1>{});
      range_note(d.range_flag, amax);
    }
  };

  // ---- persistent walk over M-tiles mt0, mt0 + mstride, ...: set (i & 1) holds tile i
  f32x4 set0[C::AQ], set1[C::AQ];
  const int ntiles = mt0 < mtiles ? (mtiles - 1 - mt0) / mstride + 1 : 0;
  auto mt_of = [&](int i) { return mt0 + i * mstride; };
  if (ntiles > 0) load_a(mt_of(0), set0);
  if (ntiles > 1) load_a(mt_of(1), set1);
  if (ntiles > 0) store_a(set0);
  __syncthreads();
  for (int i = 0; i < ntiles; i += 2) {
    float res[16];
    load_res(mt_of(i), res);
    __builtin_amdgcn_sched_barrier(0);                    // keep the residual ahead of the prefetch
    load_a(mt_of(min(i + 2, ntiles - 1)), set0);         // set 0 was staged at the end of i-1;
                                                          // unconditional (clamped): counted waits
    tile(mt_of(i), res);
    __syncthreads();
    if (i + 1 >= ntiles) break;
    store_a(set1);
    __syncthreads();
    load_res(mt_of(i + 1), res);
    __builtin_amdgcn_sched_barrier(0);
    load_a(mt_of(min(i + 3, ntiles - 1)), set1);
    tile(mt_of(i + 1), res);
    __syncthreads();
    if (i + 2 < ntiles) store_a(set0);
    __syncthreads();
  }
}

template <int KP, int BN, bool S1, bool RES>
hipError_t launch_pw_t(const ConvDesc& d, hipStream_t s) {
  using C = PwCfg<KP, BN>;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + BN - 1) / BN;
  const int mtiles = (M + C::BM - 1) / C::BM;
  // every resident block slot gets one persistent block owning one N-slice: grid a multiple of nN
  auto k = pw_gemm_x3_kernel<KP, BN, S1, RES>;
  static const int per_cu = [&] {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 512, 0) != hipSuccess || n <= 0) n = 1;
    return n;
  }();
  const int slots = per_cu * device_cus();
  const int grid = std::max(nN, std::min(mtiles * nN, slots / nN * nN));
  hipLaunchKernelGGL(k, dim3(grid), dim3(512), 0, s, d);
  return hipGetLastError();
}

// the 32-wide slice exists for Kp == 32 only (SPK_PW(32, 32)); a deeper K with N <= 32 takes
// the 64-wide slice (its zero columns are masked)
int pw_bn(const ConvDesc& d) { return d.Kp == 32 ? 32 : d.N <= 64 ? 64 : 128; }

}  // namespace

int device_cus() {
  // per device (handles on different GPU models in one process), relaxed atomics: a racing
  // first query stores the same value twice
  static std::atomic<int> cached[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cached[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

bool pw_supported(const ConvDesc& d) {
  static const bool off = std::getenv("SPK_NO_PW") != nullptr;   // diagnostics: implicit GEMM instead
  if (off) return false;
  const ConvSrc& a = d.s0;
  const bool s1_ok = !d.s1.p && d.s1.cin == 0
                         ? true
                         : (d.s1.kh == 1 && d.s1.kw == 1 && d.s1.sh == 1 && d.s1.sw == 1 && d.s1.ph == 0 &&
                            d.s1.pw == 0 && d.s1.cin % 4 == 0 && d.s1.ld % 4 == 0);
  // stride: output rows map onto every sh-th / sw-th input row (pad 0); the K-concatenated
  // s1 operand keeps the output geometry
  const bool geom = a.sh >= 1 && a.sw >= 1 && (a.H - 1) / a.sh + 1 == d.Ho && (a.W - 1) / a.sw + 1 == d.Wo &&
                    ((a.sh == 1 && a.sw == 1) || (!d.s1.p && d.s1.cin == 0));
  return d.wh && d.wl && !a.vlen && a.kh == 1 && a.kw == 1 && geom && a.ph == 0 && a.pw == 0 && !a.reflect &&
         !a.pre_scale && !a.p2 && a.ld2 == 0 && s1_ok && (d.Kp == 32 || d.Kp == 64 || d.Kp == 128) && d.N <= 256 &&
         (d.Kp != 32 || d.N <= 32) && d.N % 4 == 0 && !d.affx && !d.gate && !d.rowbias && !d.rowlen && d.ksplit == 1 &&
         a.cin % 4 == 0 && d.nimg * d.Ho * d.Wo >= 65536;
}

std::string pw_kernel_name(const ConvDesc& d) {
  const bool s1 = d.s1.p != nullptr || d.s1.cin > 0;
  const bool res = d.res != nullptr || d.ldr > 0;
  return "pw_gemm_x3_kernel<" + std::to_string(d.Kp) + ", " + std::to_string(pw_bn(d)) + ", " +
         (s1 ? "true" : "false") + ", " + (res ? "true" : "false") + ">";
}

hipError_t launch_pw(const ConvDesc& d, hipStream_t s) {
  if (!pw_supported(d)) return hipErrorInvalidValue;
  const bool s1 = d.s1.p != nullptr;
  const int bn = pw_bn(d);
#define SPK_PW(KP, BNV)                                                         \
  if (d.Kp == KP && bn == BNV)                                                  \
    return s1 ? (d.res ? launch_pw_t<KP, BNV, true, true>(d, s) : launch_pw_t<KP, BNV, true, false>(d, s)) \
              : (d.res ? launch_pw_t<KP, BNV, false, true>(d, s) : launch_pw_t<KP, BNV, false, false>(d, s));
  SPK_PW(32, 32)
  SPK_PW(64, 64)
  SPK_PW(64, 128)
  SPK_PW(128, 64)
  SPK_PW(128, 128)
#undef SPK_PW
  return hipErrorInvalidValue;
}

}  // namespace spk
