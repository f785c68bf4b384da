// Fused ERes2NetV2 Res2Net block (speakerlab/models/eres2net/ERes2NetV2.py:65-91) for the
// stage-1 blocks: one persistent kernel, fp16x3 MFMA, gfx950.  Two shapes: the identity-
// shortcut blocks (128 -> 128 channels) and the first block of the stage (64 -> 128, a 1x1
// projection shortcut + BN, ERes2NetV2.py:84-88), whose shortcut GEMM is K-concatenated
// with conv3 (K = 64 concat channels + 64 input channels, biases summed on the host).
//
// Unfused, a stage-1 block is four launches (conv1, two 3x3 convs, conv3 + residual) whose
// intermediates make full HBM round trips: ~2.5 KB per pixel for 0.5 KB of real input and
// output.  Here a workgroup owns an 8 x 16 output tile and keeps everything between the
// block input and the block output in LDS:
//   1. conv1 (1x1, C -> 2 x 32 channels incl. padding) + bn1 + Hardtanh on the 12 x 20
//      halo-2 region: slice 0 -> S0 (the first 3x3 conv's input, halo 2), slice 1 -> SP
//      (halo 1); the input is staged through two LDS chunk buffers 32 pixels at a time
//      (split into fp16 hi / lo planes on the way in), its global loads three chunks ahead;
//   2. convs.0 (3x3) + bn + Hardtanh on the 10 x 18 halo-1 region; sp = y0 + s1 is formed
//      in place in SP (torch: sp = sp + spx[1]), y0's centre goes to CAT;
//   3. convs.1 (3x3) + bn + Hardtanh on the 8 x 16 tile -> CAT;
//   4. conv3 (1x1, 64 -> CO) + bn3 + residual + Hardtanh -> HBM; with the projection
//      shortcut the tile's input pixels are staged into LDS (over the SP region, free
//      after convs.1) as conv3's second K half, and no residual is read.
// Halo recompute: conv1 runs on 240 pixels and convs.0 on 180 per 128 outputs.
//
// MFMA v_mfma_f32_16x16x32_f16 in the TRANSPOSED form out^T[n][px] = W[n][k] . In^T[k][px]:
// A = weights (rows = output channels), B = activations (lane l: pixel l & 15, channels
// 8(l >> 4) .. +7 = one 16-byte LDS read), so the accumulator gives each lane four
// consecutive output channels of one pixel: an 8-byte LDS write per plane (or a float4
// store for the block output).  fp16x3 numerics as conv_gemm.hip (hi*hi + 2^-11 (hi*lo +
// lo*hi), fp32 accumulate).  LDS rows are XOR-swizzled per 16-byte block so the B / A reads
// are bank-conflict free (32-channel rows: block ^ ((row >> 1) & 3); 64-channel CAT rows:
// block ^ (row & 7); the staged input rows are padded by 16 halves instead).
#include <algorithm>

#include "conv_epilogue.h"
#include "res2block.h"

#ifndef SPK_R2_RES_EARLY
#define SPK_R2_RES_EARLY 1   // the second half of conv3's residual requested before convs.1 too
#endif
#ifndef SPK_R2_PROF
#define SPK_R2_PROF 0
#endif

namespace spk {

#if SPK_R2_PROF
// diagnostic build only (tools/r2_prof.py): per-wave cycle counts of the kernel's phases,
// stored by every lane to its own slot (vector stores)
constexpr int R2P_PH = 8, R2P_BLK = 1024;
__device__ long long r2_prof_buf[R2P_BLK * 8 * R2P_PH * 64];
#endif

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int CI, int CO, bool PROJ>
struct R2 {
  static constexpr int NT = 512;
  static constexpr int TH = 8, TW = 16;
  static constexpr int RH = TH + 4, RW = TW + 4, NR = RH * RW;      // S0 region 12 x 20 = 240 px
  static constexpr int PH = TH + 2, PW = TW + 2, NP = PH * PW;      // SP region 10 x 18 = 180 px
  static constexpr int NO = TH * TW;                                // 128 output px
  static constexpr int XCH = 32;                                    // pixels per conv1 input chunk
  static constexpr int NCH = (NR + XCH - 1) / XCH;                  // 8 chunks
  static constexpr int XF = XCH * (CI / 4) / NT;                    // float4 staged per thread per chunk
  static constexpr int KS1 = CI / 32;                               // conv1 k-steps
  static constexpr int NT3 = CO / 128;                              // conv3 n-tiles per wave
  static constexpr int KS3 = PROJ ? 2 + CI / 32 : 2;                // conv3 k-steps (concat | input)
  static constexpr int K3 = 32 * KS3;                               // packed conv3 row length
  static constexpr int CSW = CI / 8 - 1 < 15 ? CI / 8 - 1 : 15;     // chunk-row swizzle mask
  static constexpr int XCEN_PL = NO * CI;                           // PROJ: staged input tile (halves)
  static constexpr int S0_PL = NR * 32, CAT_PL = NO * 64;           // plane sizes (halves)
  static constexpr int R0_PL = S0_PL > CAT_PL ? S0_PL : CAT_PL;
  static constexpr int SP_PL = NP * 32, XC_PL = XCH * CI, WC_PL = 2 * 32 * 288;
  static constexpr int OFF_SP = 2 * R0_PL, OFF_XC = OFF_SP + 2 * SP_PL, OFF_WC = OFF_XC + 4 * XC_PL;
  static constexpr int LDS_HALVES = OFF_WC + 2 * WC_PL;
  static_assert(CO % 128 == 0, "conv3 n-tiles are dealt 8 per wave round");
  static_assert(XCH * (CI / 4) % NT == 0, "input chunk must split evenly over the block");
  static_assert(PROJ ? (CI == 64 && OFF_SP + 2 * XCEN_PL <= OFF_WC) : CI == CO, "block shape");
  static_assert(!PROJ || NO * (CI / 4) == 4 * NT, "PROJ: the input tile is four float4 per thread");
  static_assert(NCH >= 4, "the chunk ring assumes at least four chunks");
};

__device__ __forceinline__ int swz4(int row) { return (row >> 1) & 3; }
__device__ __forceinline__ float htanh(float v) { return fminf(fmaxf(v, 0.0f), 20.0f); }
__device__ __forceinline__ f32x4 mfma16(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <int CI, int CO, bool PROJ>
__global__ void __launch_bounds__(512, 1)
res2_block_kernel(const Res2Desc d) {
  using G = R2<CI, CO, PROJ>;
  __shared__ __attribute__((aligned(16))) _Float16 lds[G::LDS_HALVES];
  _Float16* const S0h = lds;                  // S0 region, then (aliased) CAT
  _Float16* const S0l = lds + G::S0_PL;
  _Float16* const CATh = lds;
  _Float16* const CATl = lds + G::CAT_PL;
  _Float16* const SPh = lds + G::OFF_SP;
  _Float16* const SPl = SPh + G::SP_PL;
  _Float16* const XCh = lds + G::OFF_XC;     // two chunk buffers: hi planes, then lo planes
  _Float16* const XCl = XCh + 2 * G::XC_PL;
  _Float16* const WCh = lds + G::OFF_WC;
  _Float16* const WCl = WCh + G::WC_PL;
  _Float16* const XNh = lds + G::OFF_SP;      // PROJ: the tile's input pixels (over SP + XC)
  _Float16* const XNl = XNh + G::XCEN_PL;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, lq = lane >> 4;
  const int H = d.H, W = d.W;
  const int ntx = (W + G::TW - 1) / G::TW, nty = (H + G::TH - 1) / G::TH;
  const int ntiles = d.nimg * ntx * nty;
#if SPK_R2_PROF
  long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  long long tl = __builtin_amdgcn_s_memtime();
#define R2_STAMP(i) do { const long long now_ = __builtin_amdgcn_s_memtime(); tp[i] += now_ - tl; tl = now_; } while (0)
#else
#define R2_STAMP(i) do {} while (0)
#endif

  // ---- once per block: both 3x3 weight matrices -> LDS, conv1 / conv3 A fragments -> VGPRs
  for (int i = tid; i < 2 * 32 * 36; i += G::NT) {
    const int kb = i % 36, n = (i / 36) % 32, cv = i / (36 * 32);
    const uint16_t* sh = cv ? d.wbh : d.wah;
    const uint16_t* sl = cv ? d.wbl : d.wal;
    const u32x4 h = *reinterpret_cast<const u32x4*>(sh + n * 288 + kb * 8);
    const u32x4 l = *reinterpret_cast<const u32x4*>(sl + n * 288 + kb * 8);
    const int dst = cv * 32 * 288 + n * 288 + 8 * ((kb & ~3) + ((kb & 3) ^ swz4(n)));
    *reinterpret_cast<u32x4*>(WCh + dst) = h;
    *reinterpret_cast<u32x4*>(WCl + dst) = l;
  }
  const int nt1 = wave & 3;                   // conv1: 16-channel tile of the 64 (slice = nt1 >> 1)
  f16x8 a1h[G::KS1], a1l[G::KS1];
#pragma unroll
  for (int ks = 0; ks < G::KS1; ++ks) {
    const size_t o = (size_t)(16 * nt1 + l16) * CI + 32 * ks + 8 * lq;
    a1h[ks] = *reinterpret_cast<const f16x8*>(d.w1h + o);
    a1l[ks] = *reinterpret_cast<const f16x8*>(d.w1l + o);
  }
  f16x8 a3h[G::NT3][G::KS3], a3l[G::NT3][G::KS3];
  f32x4 b3v[G::NT3];
#pragma unroll
  for (int j = 0; j < G::NT3; ++j) {
    const int n = 16 * (wave + 8 * j);
#pragma unroll
    for (int ks = 0; ks < G::KS3; ++ks) {
      const size_t o = (size_t)(n + l16) * G::K3 + 32 * ks + 8 * lq;
      a3h[j][ks] = *reinterpret_cast<const f16x8*>(d.w3h + o);
      a3l[j][ks] = *reinterpret_cast<const f16x8*>(d.w3l + o);
    }
    b3v[j] = *reinterpret_cast<const f32x4*>(d.b3 + n + 4 * lq);
  }
  const f32x4 b1v = *reinterpret_cast<const f32x4*>(d.b1 + 16 * nt1 + 4 * lq);
  const int ntc = wave & 1;                   // 3x3 convs: 16-channel tile of the 32
  const f32x4 bav = *reinterpret_cast<const f32x4*>(d.ba + 16 * ntc + 4 * lq);
  const f32x4 bbv = *reinterpret_cast<const f32x4*>(d.bb + 16 * ntc + 4 * lq);
  constexpr float kLo = 1.0f / 2048.0f;

  // ---- persistent walk: the tiles of one XCD's contiguous share go to that XCD's blocks,
  //      so neighbouring tiles (which re-read each other's halo) share an L2
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int per = (ntiles + 7) / 8;
  const int t_lo = xcd * per, t_hi = min(ntiles, t_lo + per);
  // conv1 input chunk ch of a tile: 32 region pixels x C channels, XF float4 per thread
  auto load_chunk = [&](int ch, f32x4 (&v)[G::XF], int ty0, int tx0, const float* im) {
#pragma unroll
    for (int j = 0; j < G::XF; ++j) {
      const int i = tid + G::NT * j;
      const int px = ch * G::XCH + i / (CI / 4), q = i % (CI / 4);
      const int gy = min(max(ty0 - 2 + px / G::RW, 0), H - 1);
      const int gx = min(max(tx0 - 2 + px % G::RW, 0), W - 1);
      v[j] = *reinterpret_cast<const f32x4*>(im + ((size_t)gy * W + gx) * CI + 4 * q);
    }
  };
  auto store_chunk = [&](const f32x4 (&v)[G::XF], int buf) {
#pragma unroll
    for (int j = 0; j < G::XF; ++j) {
      const int i = tid + G::NT * j;
      const int px = i / (CI / 4), q = i % (CI / 4);
      const int a = buf * G::XC_PL + px * CI + 8 * ((q >> 1) ^ (px & G::CSW)) + 4 * (q & 1);
      h16x4 h, l;
      split_x3(v[j], h, l);
      *reinterpret_cast<h16x4*>(XCh + a) = h;
      *reinterpret_cast<h16x4*>(XCl + a) = l;
    }
  };
  auto tile_origin = [&](int tt, int& im, int& ty0, int& tx0) {
    im = tt / (ntx * nty);
    ty0 = ((tt / ntx) % nty) * G::TH;
    tx0 = (tt % ntx) * G::TW;
  };
  f32x4 pf[3][G::XF];
  if (t_lo + slot < t_hi) {
    int im, ty0, tx0;
    tile_origin(t_lo + slot, im, ty0, tx0);
    const float* p0 = d.x + (size_t)im * H * W * CI;
    load_chunk(0, pf[0], ty0, tx0, p0);
    load_chunk(1, pf[1], ty0, tx0, p0);
    load_chunk(2, pf[2], ty0, tx0, p0);
  }
  for (int t = t_lo + slot; t < t_hi; t += nslot) {
    int img, y0, x0;
    tile_origin(t, img, y0, x0);
    const float* const xim = d.x + (size_t)img * H * W * CI;

    // ================= 1. conv1 on the S0 region, 32 pixels per chunk: chunks are staged
    //   through two LDS buffers (fp16 hi / lo, rows swizzled block ^ (px & 15)), their global
    //   loads run three chunks ahead in a register ring (the first three were requested
    //   during the previous tile's conv3), one barrier per chunk
#pragma unroll
    for (int ch = 0; ch < G::NCH; ++ch) {
      if (ch == 0) {
        store_chunk(pf[0], 0);
        load_chunk(3, pf[0], y0, x0, xim);
      }
      __syncthreads();
      R2_STAMP(0);
      if (ch + 1 < G::NCH) {
        store_chunk(pf[(ch + 1) % 3], (ch + 1) & 1);
        if (ch + 4 < G::NCH) load_chunk(ch + 4, pf[(ch + 1) % 3], y0, x0, xim);
      }
      R2_STAMP(1);
      const _Float16* xh = XCh + (ch & 1) * G::XC_PL;
      const _Float16* xl = XCl + (ch & 1) * G::XC_PL;
      const int pxl = 16 * (wave >> 2) + l16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < G::KS1; ++ks) {
        const int a = pxl * CI + 8 * ((4 * ks + lq) ^ (pxl & G::CSW));
        const f16x8 bh = *reinterpret_cast<const f16x8*>(xh + a);
        const f16x8 bl = *reinterpret_cast<const f16x8*>(xl + a);
        acc = mfma16(a1h[ks], bh, acc);
        accx = mfma16(a1h[ks], bl, accx);
        accx = mfma16(a1l[ks], bh, accx);
      }
      const int rpx = ch * G::XCH + pxl;     // S0-region pixel of this lane's column
      if (rpx < G::NR) {
        const int r = rpx / G::RW, c = rpx % G::RW;
        const int gy = y0 - 2 + r, gx = x0 - 2 + c;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;   // conv padding: zero outside
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = in ? htanh(acc[e] + accx[e] * kLo + b1v[e]) : 0.f;
        h16x4 h, l;
        split_x3(v, h, l);
        const int cc = 16 * (nt1 & 1) + 4 * lq;                   // channel within the slice
        const int kb = cc >> 3, sub = cc & 7;
        if (nt1 < 2) {
          const int a = rpx * 32 + 8 * (kb ^ swz4(rpx)) + sub;
          *reinterpret_cast<h16x4*>(S0h + a) = h;
          *reinterpret_cast<h16x4*>(S0l + a) = l;
        } else if (r >= 1 && r <= G::PH && c >= 1 && c <= G::PW) {
          const int sp = (r - 1) * G::PW + (c - 1);
          const int a = sp * 32 + 8 * (kb ^ swz4(sp)) + sub;
          *reinterpret_cast<h16x4*>(SPh + a) = h;
          *reinterpret_cast<h16x4*>(SPl + a) = l;
        }
      }
      R2_STAMP(2);
    }
    __syncthreads();
    R2_STAMP(3);

    // ================= 2. convs.0 on the SP region (3 pixel tiles per wave)
    const int cc = 16 * ntc + 4 * lq, kbo = cc >> 3, subo = cc & 7;
    f32x4 y[3];
    {
      f32x4 acc[3], accx[3];
      int base[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        accx[i] = acc[i];
        const int p = min(16 * ((wave >> 1) + 4 * i) + l16, G::NP - 1);
        base[i] = (p / G::PW) * G::RW + p % G::PW;
      }
      const int nrow = 16 * ntc + l16;
      const _Float16* wa_h = WCh + nrow * 288;
      const _Float16* wa_l = WCl + nrow * 288;
      const int wq = (lq ^ swz4(nrow)) * 8;
#pragma unroll 3
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * G::RW + tap % 3;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(wa_h + 32 * tap + wq);
        const f16x8 al = *reinterpret_cast<const f16x8*>(wa_l + 32 * tap + wq);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const int px = base[i] + toff;
          const int a = px * 32 + 8 * (lq ^ swz4(px));
          const f16x8 bh = *reinterpret_cast<const f16x8*>(S0h + a);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(S0l + a);
          acc[i] = mfma16(ah, bh, acc[i]);
          accx[i] = mfma16(ah, bl, accx[i]);
          accx[i] = mfma16(al, bh, accx[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int p = 16 * ((wave >> 1) + 4 * i) + l16;
        const int gy = y0 - 1 + p / G::PW, gx = x0 - 1 + p % G::PW;
        const bool in = p < G::NP && gy >= 0 && gy < H && gx >= 0 && gx < W;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[i][e] = in ? htanh(acc[i][e] + accx[i][e] * kLo + bav[e]) : 0.f;
      }
    }
    __syncthreads();                          // S0 reads done: the region becomes CAT
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = 16 * ((wave >> 1) + 4 * i) + l16;
      if (p >= G::NP) continue;
      const int a = p * 32 + 8 * (kbo ^ swz4(p)) + subo;
      const h16x4 sh = *reinterpret_cast<const h16x4*>(SPh + a);
      const h16x4 sl = *reinterpret_cast<const h16x4*>(SPl + a);
      f32x4 sp;
#pragma unroll
      for (int e = 0; e < 4; ++e) sp[e] = y[i][e] + ((float)sh[e] + (float)sl[e] * kLo);
      h16x4 h, l;
      split_x3(sp, h, l);
      *reinterpret_cast<h16x4*>(SPh + a) = h;
      *reinterpret_cast<h16x4*>(SPl + a) = l;
      const int r = p / G::PW - 1, c = p % G::PW - 1;
      if (r >= 0 && r < G::TH && c >= 0 && c < G::TW) {
        const int o = r * G::TW + c;
        const int ao = o * 64 + 8 * (kbo ^ (o & 7)) + subo;
        split_x3(y[i], h, l);
        *reinterpret_cast<h16x4*>(CATh + ao) = h;
        *reinterpret_cast<h16x4*>(CATl + ao) = l;
      }
    }
    __syncthreads();
    R2_STAMP(4);

    // residual of the first half of the conv3 pixel tiles (PROJ: the tile's input pixels,
    // conv3's second operand): requested now, in flight during convs.1
    f32x4 res_a[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      if constexpr (PROJ) {
        const int i = tid + G::NT * pt, o = i / (CI / 4), q = i % (CI / 4);
        const int gy = min(y0 + o / G::TW, H - 1), gx = min(x0 + o % G::TW, W - 1);
        res_a[pt] = *reinterpret_cast<const f32x4*>(xim + ((size_t)gy * W + gx) * CI + 4 * q);
      } else {
        const int gy = min(y0 + pt, H - 1), gx = min(x0 + l16, W - 1);
        res_a[pt] = *reinterpret_cast<const f32x4*>(xim + ((size_t)gy * W + gx) * CI + 16 * wave + 4 * lq);
      }
    }

#if SPK_R2_RES_EARLY
    // the second half as well: requested before the first MFMA of conv3 it would arrive an L2 /
    // HBM round trip after conv3's first four pixel tiles (phase stamps: conv3 8.8k cycles per
    // tile against 1.5k of MFMAs); the register ring is empty during convs.1, so the extra 16
    // VGPRs are free there
    f32x4 res_b[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int gy = min(y0 + 4 + pt, H - 1), gx = min(x0 + l16, W - 1);
      if constexpr (PROJ) res_b[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
      else res_b[pt] = *reinterpret_cast<const f32x4*>(xim + ((size_t)gy * W + gx) * CI + 16 * wave + 4 * lq);
    }
#endif
    // ================= 3. convs.1 on the output tile (2 pixel tiles per wave)
    {
      f32x4 acc[2], accx[2];
      int base[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        accx[i] = acc[i];
        const int o = 16 * ((wave >> 1) + 4 * i) + l16;
        base[i] = (o / G::TW) * G::PW + o % G::TW;
      }
      const int nrow = 16 * ntc + l16;
      const _Float16* wb_h = WCh + 32 * 288 + nrow * 288;
      const _Float16* wb_l = WCl + 32 * 288 + nrow * 288;
      const int wq = (lq ^ swz4(nrow)) * 8;
#pragma unroll 3
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * G::PW + tap % 3;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(wb_h + 32 * tap + wq);
        const f16x8 al = *reinterpret_cast<const f16x8*>(wb_l + 32 * tap + wq);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int px = base[i] + toff;
          const int a = px * 32 + 8 * (lq ^ swz4(px));
          const f16x8 bh = *reinterpret_cast<const f16x8*>(SPh + a);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(SPl + a);
          acc[i] = mfma16(ah, bh, acc[i]);
          accx[i] = mfma16(ah, bl, accx[i]);
          accx[i] = mfma16(al, bh, accx[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = 16 * ((wave >> 1) + 4 * i) + l16;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = htanh(acc[i][e] + accx[i][e] * kLo + bbv[e]);
        h16x4 h, l;
        split_x3(v, h, l);
        const int ao = o * 64 + 8 * ((4 + kbo) ^ (o & 7)) + subo;   // CAT channels 32..63
        *reinterpret_cast<h16x4*>(CATh + ao) = h;
        *reinterpret_cast<h16x4*>(CATl + ao) = l;
      }
    }
    __syncthreads();
    if constexpr (PROJ) {                     // SP / XC reads done: stage the input tile there
#pragma unroll
      for (int pt = 0; pt < 4; ++pt) {
        const int i = tid + G::NT * pt, o = i / (CI / 4), q = i % (CI / 4);
        const int a = o * CI + 8 * ((q >> 1) ^ (o & 7)) + 4 * (q & 1);
        h16x4 h, l;
        split_x3(res_a[pt], h, l);
        *reinterpret_cast<h16x4*>(XNh + a) = h;
        *reinterpret_cast<h16x4*>(XNl + a) = l;
      }
      __syncthreads();
    }
    R2_STAMP(5);

    // ================= 4. conv3 + bn3 + residual + Hardtanh -> out (8 pixel tiles per wave)
#if !SPK_R2_RES_EARLY
    // residual of the second half: requested before the first MFMA (the first half is in flight)
    f32x4 res_b[4];
#pragma unroll
    for (int pt = 0; pt < 4; ++pt) {
      const int gy = min(y0 + 4 + pt, H - 1), gx = min(x0 + l16, W - 1);
      if constexpr (PROJ) res_b[pt] = f32x4{0.f, 0.f, 0.f, 0.f};
      else res_b[pt] = *reinterpret_cast<const f32x4*>(xim + ((size_t)gy * W + gx) * CI + 16 * wave + 4 * lq);
    }
#endif
    // the next tile's first three input chunks, behind the residual (vmcnt retires in order,
    // so the epilogue's wait for the residual does not wait for these)
    // unconditional (the last tile re-reads its own chunks): a load on only some paths
    // leaves the compiler's wait counts unknown, and the residual waits below became
    // vmcnt(0), i.e. waits for these chunks too
    {
      int im, ty0, tx0;
      tile_origin(t + nslot < t_hi ? t + nslot : t, im, ty0, tx0);
      const float* pn = d.x + (size_t)im * H * W * CI;
      load_chunk(0, pf[0], ty0, tx0, pn);
      load_chunk(1, pf[1], ty0, tx0, pn);
      load_chunk(2, pf[2], ty0, tx0, pn);
    }
#pragma unroll
    for (int j = 0; j < G::NT3; ++j) {
      const int n = 16 * (wave + 8 * j) + 4 * lq;
#pragma unroll
      for (int pt = 0; pt < 8; ++pt) {
        const int o = 16 * pt + l16;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f}, accx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < G::KS3; ++ks) {
          f16x8 bh, bl;
          if (ks < 2) {
            const int a = o * 64 + 8 * ((4 * ks + lq) ^ (o & 7));
            bh = *reinterpret_cast<const f16x8*>(CATh + a);
            bl = *reinterpret_cast<const f16x8*>(CATl + a);
          } else {
            const int a = o * CI + 8 * ((4 * (ks - 2) + lq) ^ (o & 7));
            bh = *reinterpret_cast<const f16x8*>(XNh + a);
            bl = *reinterpret_cast<const f16x8*>(XNl + a);
          }
          acc = mfma16(a3h[j][ks], bh, acc);
          accx = mfma16(a3h[j][ks], bl, accx);
          accx = mfma16(a3l[j][ks], bh, accx);
        }
        const int gy = y0 + pt, gx = x0 + l16;
        if (gy < H && gx < W) {
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = PROJ ? 0.f : (pt < 4 ? res_a[pt][e] : res_b[pt - 4][e]);
            v[e] = htanh(acc[e] + accx[e] * kLo + b3v[j][e] + r);
          }
          block_store(reinterpret_cast<f32x4*>(d.out + (((size_t)img * H + gy) * W + gx) * CO + n), v);
        }
      }
    }
    R2_STAMP(6);
    __syncthreads();                          // CAT reads done before the next tile's conv1
    R2_STAMP(7);
  }
#if SPK_R2_PROF
  if (blockIdx.x < R2P_BLK)
    for (int i = 0; i < R2P_PH; ++i) r2_prof_buf[(((size_t)blockIdx.x * 8 + wave) * R2P_PH + i) * 64 + lane] = tp[i];
#endif
}

}  // namespace

bool res2_block_supported(const Res2Desc& d) {
  const int co = d.Cout ? d.Cout : d.C;
  const bool shape = d.stride == 1 && (!d.Hin || d.Hin == d.H) && (!d.Win || d.Win == d.W) &&
                     (d.proj ? (d.C == 64 && co == 128) : (d.C == 128 && co == 128));
  return conv_use_x3() && shape && d.width >= 1 && d.width <= 32 && d.nimg > 0 && d.H > 0 && d.W > 0 &&
         d.w1h && d.w1l && d.wah && d.wal && d.wbh && d.wbl && d.w3h && d.w3l && d.b1 && d.ba && d.bb && d.b3;
}

std::string res2_block_kernel_name(const Res2Desc& d) {
  return d.proj ? "res2_block_kernel<64, 128, true>" : "res2_block_kernel<128, 128, false>";
}

hipError_t launch_res2_block(const Res2Desc& d, hipStream_t s) {
  if (!res2_block_supported(d) || d.x == d.out) return hipErrorInvalidValue;
  const int ntiles = d.nimg * ((d.W + 15) / 16) * ((d.H + 7) / 8);
  int grid = std::min(device_cus(), (ntiles + 7) / 8 * 8);
  grid = std::max(8, grid / 8 * 8);
  if (d.proj) hipLaunchKernelGGL((res2_block_kernel<64, 128, true>), dim3(grid), dim3(512), 0, s, d);
  else hipLaunchKernelGGL((res2_block_kernel<128, 128, false>), dim3(grid), dim3(512), 0, s, d);
  return hipGetLastError();
}

}  // namespace spk

#if SPK_R2_PROF
extern "C" int spk_exp_res2_prof(long long* host, size_t n) {
  const size_t all = sizeof(spk::r2_prof_buf) / sizeof(long long);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(spk::r2_prof_buf), std::min(n, all) * sizeof(long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
