// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32), gfx950.
//
// One kernel serves every conv / 1x1 / linear layer of the four embedding models
// (SURVEY.md §8(a) rows a3-a22): activations are channels-last so the GEMM K dimension
// (tap, channel) is contiguous in HBM, the M dimension is output pixels (img, h, w) and N
// is output channels.  BatchNorm is folded into the packed weights/bias on the host, and
// the epilogue fuses bias, residual add, the activation (ReLU / Hardtanh(0,20) / SiLU /
// sigmoid / tanh), a post-activation affine (ECAPA's conv->ReLU->BN), the AFF combine
// (fusion.py:22-28) and the CAM gate, writing into a channel slice of a wider buffer so
// torch.cat / torch.split never move data.
//
// Tiling: 64*WM*WN threads, block tile BM x BN, K-tile BK floats, LDS double buffer
// with register staging (one barrier per K-tile).  Each wave owns (BM/WM) x (BN/WN) as
// 32x32 MFMA tiles.  fp32 MFMA issues at 64 cycles / SIMD, so LDS bandwidth is not the
// limit: fragments are read as 2 x ds_read_b128 per 8 MFMA k-steps thanks to a k
// permutation (lane half h owns k = 8h + s of the 16-deep tile, identically for A and B).
// LDS rows are padded to 20 floats, which makes those b128 reads bank-conflict free.
#include <string>

#include "common.h"
#include "conv_epilogue.h"

namespace spk {

namespace {


constexpr int KP_ALIGN = 32;   // weights are packed with Kp a multiple of this

// XCD-aware bijective block remap: consecutive logical ids (same M tile, all N tiles) are
// placed on one XCD so the A tile they share stays in that XCD's L2
// (cdna_hip_programming.md §5.5 T1, bijective form).
__device__ __forceinline__ int xcd_remap(int orig, int nblk) {
  const int q = nblk / 8, r = nblk % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int BM, int BN, int BK, int WM, int WN, bool S1, bool ADD>
__global__ void __launch_bounds__(64 * WM * WN, 4)
conv_gemm_kernel(const ConvDesc d) {
  constexpr int NT = 64 * WM * WN;               // threads
  constexpr int WTM = BM / WM, WTN = BN / WN;    // wave tile
  constexpr int TM = WTM / 32, TN = WTN / 32;    // 32x32 MFMA tiles per wave
  constexpr int QPR = BK / 4;                    // float4 quads per tile row
  constexpr int RPP = NT / QPR;                  // rows staged per pass
  constexpr int AROWS = BM / RPP;                // A rows staged per thread
  constexpr int BROWS = (BN + RPP - 1) / RPP;    // B rows staged per thread
  constexpr int LDS_ROW = BK + 4;                // padded row: conflict-free ds_read_b128
  constexpr int HK = BK / 2;                     // k values per lane half per tile
  constexpr int FQ = HK / 4;                     // f32x4 per fragment
  static_assert(TM >= 1 && TN >= 1 && BM % RPP == 0, "tile shape");
  constexpr int LDS_STAGE = 2 * (BM + BN) * LDS_ROW;   // double-buffered A/B tiles
  constexpr int LDS_EPI = WM * WN * TM * TN * 1024;    // every accumulator of the block
  constexpr int LDS_FLOATS = LDS_STAGE > LDS_EPI ? LDS_STAGE : LDS_EPI;

  __shared__ __attribute__((aligned(16))) float lds[LDS_FLOATS];
  float* As = lds;                               // [2][BM][LDS_ROW]
  float* Bs = lds + 2 * BM * LDS_ROW;            // [2][BN][LDS_ROW]

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + BN - 1) / BN;
  const int nM = (M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, nM * nN);
  const int mt = lid / nN, nt = lid % nN;
  const int m0 = mt * BM, n0 = nt * BN;

  // K range of this split
  const int nkt_all = d.Kp / BK;
  const int per = (nkt_all + d.ksplit - 1) / d.ksplit;
  const int kt0 = blockIdx.z * per;
  const int kt1 = min(nkt_all, kt0 + per);

  // ---- per-thread A-row geometry (fixed across the K loop)
  const int kq = tid % QPR, row0 = tid / QPR;
  int a_img[AROWS], a_hb[AROWS], a_wb[AROWS], a_h1[AROWS], a_w1[AROWS];
  bool a_ok[AROWS];
#pragma unroll
  for (int r = 0; r < AROWS; ++r) {
    const int m = m0 + row0 + RPP * r;
    a_ok[r] = m < M;
    const int mm = a_ok[r] ? m : 0;
    const int wo = mm % d.Wo;
    const int t2 = mm / d.Wo;
    const int ho = t2 % d.Ho;
    a_img[r] = t2 / d.Ho;
    a_hb[r] = ho * d.s0.sh - d.s0.ph;
    a_wb[r] = wo * d.s0.sw - d.s0.pw;
    if (S1) { a_h1[r] = ho * d.s1.sh; a_w1[r] = wo * d.s1.sw; }
  }
  const int K0 = d.s0.kh * d.s0.kw * d.s0.cin;

  // incremental (tap, channel) decomposition of this thread's k = kt*BK + kq*4
  int k_c = 0, k_ky = 0, k_kx = 0;
  {
    const int k = kt0 * BK + kq * 4;
    if (k < K0) {
      const int tap = k / d.s0.cin;
      k_c = k - tap * d.s0.cin;
      k_ky = tap / d.s0.kw;
      k_kx = tap - k_ky * d.s0.kw;
    } else {
      k_ky = d.s0.kh; k_c = k - K0;   // in s1 (or beyond K)
    }
  }

  f32x4 ra[AROWS], rb[BROWS];

  auto load_tile = [&](int kt) {
    const int k = kt * BK + kq * 4;
    // ---- A (implicit im2col; zero outside the image / beyond K)
    if (k_ky < d.s0.kh) {
      const bool pre = d.s0.pre_scale != nullptr;
      f32x4 psc = {1.f, 1.f, 1.f, 1.f}, psh = {0.f, 0.f, 0.f, 0.f};
      if (pre) {
        psc = *reinterpret_cast<const f32x4*>(d.s0.pre_scale + k_c);
        psh = *reinterpret_cast<const f32x4*>(d.s0.pre_shift + k_c);
      }
#pragma unroll
      for (int r = 0; r < AROWS; ++r) {
        int hi = a_hb[r] + k_ky * d.s0.dh;
        int wi = a_wb[r] + k_kx * d.s0.dw;
        if (d.s0.reflect) {
          hi = hi < 0 ? -hi : (hi >= d.s0.H ? 2 * d.s0.H - 2 - hi : hi);
          wi = wi < 0 ? -wi : (wi >= d.s0.W ? 2 * d.s0.W - 2 - wi : wi);
        }
        const bool ok = a_ok[r] && hi >= 0 && hi < d.s0.H && wi >= 0 && wi < d.s0.W;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
          const size_t pix = (size_t)(a_img[r] * d.s0.H + hi) * d.s0.W + wi;
          v = *reinterpret_cast<const f32x4*>(d.s0.p + pix * d.s0.ld + k_c);
          if (ADD) v += *reinterpret_cast<const f32x4*>(d.s0.p2 + pix * d.s0.ld2 + k_c);
          if (pre) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = fmaxf(fmaf(v[q], psc[q], psh[q]), 0.f);
          }
        }
        ra[r] = v;
      }
    } else if (S1 && k_c < d.s1.cin) {
#pragma unroll
      for (int r = 0; r < AROWS; ++r) {
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (a_ok[r]) {
          const size_t pix = (size_t)(a_img[r] * d.s1.H + a_h1[r]) * d.s1.W + a_w1[r];
          v = *reinterpret_cast<const f32x4*>(d.s1.p + pix * d.s1.ld + k_c);
        }
        ra[r] = v;
      }
    } else {
#pragma unroll
      for (int r = 0; r < AROWS; ++r) ra[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // advance (tap, c) by BK for the next tile
    if (k_ky < d.s0.kh) {
      k_c += BK;
      while (k_c >= d.s0.cin && k_ky < d.s0.kh) {
        k_c -= d.s0.cin;
        if (++k_kx == d.s0.kw) { k_kx = 0; ++k_ky; }
      }
    } else {
      k_c += BK;
    }
    // ---- B (packed weights [N][Kp])
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      const int nr = row0 + RPP * r;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (nr < BN && n0 + nr < d.N) v = *reinterpret_cast<const f32x4*>(d.w + (size_t)(n0 + nr) * d.Kp + k);
      rb[r] = v;
    }
  };

  auto store_tile = [&](int buf) {
    float* a = As + buf * BM * LDS_ROW;
    float* b = Bs + buf * BN * LDS_ROW;
#pragma unroll
    for (int r = 0; r < AROWS; ++r) *reinterpret_cast<f32x4*>(a + (row0 + RPP * r) * LDS_ROW + kq * 4) = ra[r];
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      const int nr = row0 + RPP * r;
      if (nr < BN) *reinterpret_cast<f32x4*>(b + nr * LDS_ROW + kq * 4) = rb[r];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
      const int buf = (kt - kt0) & 1;
      if (kt + 1 < kt1) load_tile(kt + 1);
      const float* a = As + buf * BM * LDS_ROW;
      const float* b = Bs + buf * BN * LDS_ROW;
      // lane half lh owns k = lh*HK + s of this tile (same permutation for A and B)
      f32x4 af[TM][FQ], bf[TN][FQ];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* p = a + (wm * WTM + i * 32 + li) * LDS_ROW + lh * HK;
#pragma unroll
        for (int q = 0; q < FQ; ++q) af[i][q] = *reinterpret_cast<const f32x4*>(p + 4 * q);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* p = b + (wn * WTN + j * 32 + li) * LDS_ROW + lh * HK;
#pragma unroll
        for (int q = 0; q < FQ; ++q) bf[j][q] = *reinterpret_cast<const f32x4*>(p + 4 * q);
      }
#pragma unroll
      for (int s = 0; s < HK; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s >> 2][s & 3], bf[j][s >> 2][s & 3],
                                                              acc[i][j], 0, 0, 0);
      if (kt + 1 < kt1) store_tile(buf ^ 1);
      __syncthreads();
    }
  }

  // ---- fused epilogue (conv_epilogue.h): output row m of local row r is m0 + wm*WTM + r
  epilogue_tiles<TM, TN>(d, lds, acc, wave, lane, n0 + wn * WTN, M, [&](int r) { return m0 + wm * WTM + r; });
}

// Split-K combine: out = epi(sum_z partial[z])   (fixed z order: deterministic)
__global__ void splitk_reduce_kernel(const ConvDesc d, int M) {
  const size_t total = (size_t)M * d.N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int m = e / d.N, n = e % d.N;
    float v = 0.f;
    for (int z = 0; z < d.ksplit; ++z) v += d.partial[(size_t)z * total + e];
    d.out[(size_t)m * d.ldo + n] = epilogue_elem(d, m, n, v);
  }
}

struct Cfg {
  int bm, bn, bk, wm, wn;
};

Cfg select_cfg(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int bk = d.Kp >= 256 ? 32 : 16;
  if (d.N <= 32) return {256, 32, bk, 8, 1};
  if (d.N <= 64) return {256, 64, bk, 4, 2};
  if (M <= 4096) return {64, 128, bk, 1, 4};
  // 128x128 at BK=32 still fits two blocks per CU (73.7 KB LDS): half the K-steps, twice
  // the loads in flight per step -- what the short-K 1x1 convs need
  return {128, 128, 32, 2, 4};
}

template <int BM, int BN, int BK, int WM, int WN>
hipError_t launch_cfg(const ConvDesc& d, hipStream_t s) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int nblk = ((M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  dim3 grid(nblk, 1, d.ksplit);
  dim3 block(64 * WM * WN);
  const bool s1 = d.s1.p != nullptr, add = d.s0.p2 != nullptr;
  if (s1 && add) return hipErrorInvalidValue;
  if (s1) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, true, false>), grid, block, 0, s, d);
  else if (add) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, false, true>), grid, block, 0, s, d);
  else hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, false, false>), grid, block, 0, s, d);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || d.ksplit <= 1) return e;
  const size_t total = (size_t)M * d.N;
  const int rb = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(rb), dim3(256), 0, s, d, M);
  return hipGetLastError();
}

template <int BK>
hipError_t launch_bk(const ConvDesc& d, const Cfg& c, hipStream_t s) {
  if (c.bn == 32) return launch_cfg<256, 32, BK, 8, 1>(d, s);
  if (c.bn == 64) return launch_cfg<256, 64, BK, 4, 2>(d, s);
  if (c.bm == 64) return launch_cfg<64, 128, BK, 1, 4>(d, s);
  return launch_cfg<128, 128, BK, 2, 4>(d, s);
}

}  // namespace

// Name of the kernel instantiation launch_conv() picks (matches rocprofv3 kernel names).
std::string conv_kernel_name(const ConvDesc& d) {
  if (halo_conv_supported(d)) return halo_kernel_name(d);
  const Cfg c = select_cfg(d);
  const bool s1 = d.s1.p != nullptr || d.s1.cin > 0, add = d.s0.p2 != nullptr || d.s0.ld2 > 0;
  return "conv_gemm_kernel<" + std::to_string(c.bm) + ", " + std::to_string(c.bn) + ", " + std::to_string(c.bk) + ", " +
         std::to_string(c.wm) + ", " + std::to_string(c.wn) + ", " + (s1 ? "true" : "false") + ", " +
         (add ? "true" : "false") + ">";
}

int conv_tile_blocks(const ConvDesc& d) {
  const Cfg c = select_cfg(d);
  const int M = d.nimg * d.Ho * d.Wo;
  return ((M + c.bm - 1) / c.bm) * ((d.N + c.bn - 1) / c.bn);
}

hipError_t launch_conv(const ConvDesc& d, hipStream_t s) {
  // host-side shape checks: every float4 access must stay aligned and in range
  if (d.s0.cin % 4 || d.s0.ld % 4 || (d.s0.p2 && d.s0.ld2 % 4) || d.Kp % KP_ALIGN || d.ldo < d.N ||
      (d.s1.p && (d.s1.cin % 4 || d.s1.ld % 4)) || d.N <= 0 || d.nimg <= 0 || d.Ho <= 0 || d.Wo <= 0 ||
      (reinterpret_cast<uintptr_t>(d.s0.p) & 15) || (reinterpret_cast<uintptr_t>(d.w) & 15) ||
      d.K > d.Kp || (d.ksplit > 1 && !d.partial))
    return hipErrorInvalidValue;
  if (halo_conv_supported(d)) return launch_conv3x3_halo(d, s);
  const Cfg c = select_cfg(d);
  return c.bk == 32 ? launch_bk<32>(d, c, s) : launch_bk<16>(d, c, s);
}

}  // namespace spk
