// Halo-tiled 3x3 / stride 1 / pad 1 convolution for small channel counts, fp32 MFMA, gfx950.
//
// Targets the Res2Net 3x3 convs of ERes2Net(V2) stages 1-2 (26 -> 26 and 52 -> 52
// channels, physical 28 / 52; ERes2Net-large 32 / 64) and CAM++'s FCM convs, where the
// generic implicit GEMM re-reads every input pixel nine times through L2 with 64-B
// im2col segments.  Here a block owns an output tile of PIX pixels (TH x TW, TW chosen
// per layer to minimise edge waste) and all NP output channels:
//   1. the (TH+2) x (TW+2) x CIN input halo is staged into LDS once (zero outside the
//      image, the Res2Net `sp + spx` addend summed on the way in);
//   2. the nine taps run as nine K-slices of CIN: A fragments are read straight out of the
//      halo at the tap offset, B (weights of one tap, [NP][CIN]) is double-buffered in LDS
//      and the next tap's slice is prefetched into registers during the current tap;
//   3. the fused epilogue (bias + Hardtanh / ReLU, strided write into a channel slice) is
//      the one of the implicit-GEMM kernel (conv_epilogue.h).
// MFMA v_mfma_f32_32x32x2_f32: lane half h owns channels [h*CIN/2, (h+1)*CIN/2) of every
// tap (same split for A and B), read as ds_read_b64 pairs.  LDS rows are CIN+2 floats:
// an odd number of 8-byte slots, so 32 lanes on 32 different pixels (or weight rows) hit
// distinct banks.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

#ifndef SPK_EXP
#define SPK_EXP 0
#endif
#ifndef SPK_HALO_M16
#define SPK_HALO_M16 1   // x3 kernel on v_mfma_f32_16x16x32_f16 (round 6; 0: 32x32x16)
#endif
#ifndef SPK_HALO_PF2
#define SPK_HALO_PF2 0   // two halos in flight: measured neutral on ERes2NetV2, slower on ERes2Net-large / CAM++
#endif

namespace spk {

namespace {


template <int CIN, int NP, int PIX, bool ADD>
struct HaloCfg {
  static constexpr int WN = NP / 32;
  static constexpr int TILES = (PIX / 32) * WN;           // 32x32 output tiles per block
  static constexpr int NW = TILES >= 8 ? 8 : TILES;       // waves
  static constexpr int WM = NW / WN;
  static constexpr int TM = (PIX / 32) / WM;              // 32-pixel tiles per wave
  static constexpr int CS = CIN + 2;                      // LDS row stride (floats)
  static constexpr int HC = CIN / 2;
  static constexpr int Q = CIN / 4;                       // float4 per pixel / weight row
  static constexpr int HALO_PIX = PIX == 256 ? 340 : 204;   // max (TH+2)(TW+2), TW in {8, 16, 32}
  static constexpr int HALO = HALO_PIX * CS;
  static constexpr int WBUF = NP * CS;
  static constexpr int STAGE = HALO + 2 * WBUF;
  static constexpr int EPI = NW * TM * 1024;
  static constexpr int LDS = STAGE > EPI ? STAGE : EPI;
  static constexpr int WPF = (NP * Q + 64 * NW - 1) / (64 * NW);   // weight float4 per thread
};

template <int CIN, int NP, int PIX, bool ADD>
__global__ void __launch_bounds__(512, 2)
conv3x3_halo_kernel(const ConvDesc d, int TW) {
  SPK_GATE(d.run_if);
  using C = HaloCfg<CIN, NP, PIX, ADD>;
  constexpr int NT = 64 * C::NW;
  __shared__ __attribute__((aligned(16))) float lds[C::LDS];
  float* halo = lds;
  float* wbuf = lds + C::HALO;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WN, wn = wave % C::WN;
  const int li = lane & 31, lh = lane >> 5;
  const int TH = PIX / TW, HW = TW + 2, HH = TH + 2;
  const int H = d.Ho, W = d.Wo;
  const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
  const int img = blockIdx.x / (ntx * nty);
  const int ty = (blockIdx.x / ntx) % nty, tx = blockIdx.x % ntx;
  const int y0 = ty * TH, x0 = tx * TW;

  // ---- 1. input halo -> LDS: batches of HB float4 per thread, every load of a batch in
  //         flight before the first LDS write (one memory round trip per batch)
  constexpr int HB = ADD ? 4 : 8;
  const int hq = HH * HW * C::Q;
  for (int base = 0; base < hq; base += NT * HB) {
    f32x4 v[HB];
#pragma unroll
    for (int r = 0; r < HB; ++r) {
      const int idx = base + tid + NT * r;
      v[r] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int q = idx % C::Q, p = idx / C::Q;
      const int gy = y0 - 1 + p / HW, gx = x0 - 1 + p % HW;
      if (idx < hq && gy >= 0 && gy < H && gx >= 0 && gx < W) {
        const size_t pix = (size_t)(img * H + gy) * W + gx;
        v[r] = *reinterpret_cast<const f32x4*>(d.s0.p + pix * d.s0.ld + 4 * q);
        if (ADD) v[r] += *reinterpret_cast<const f32x4*>(d.s0.p2 + pix * d.s0.ld2 + 4 * q);
      }
    }
#pragma unroll
    for (int r = 0; r < HB; ++r) {
      const int idx = base + tid + NT * r;
      if (idx < hq) {
        const int q = idx % C::Q, p = idx / C::Q;
        float2* dst = reinterpret_cast<float2*>(halo + p * C::CS + 4 * q);
        dst[0] = make_float2(v[r][0], v[r][1]);
        dst[1] = make_float2(v[r][2], v[r][3]);
      }
    }
  }
  // ---- 2. weights of tap 0 -> LDS buffer 0; later taps are prefetched through registers
  f32x4 wr[C::WPF];
  auto load_w = [&](int tap) {
#pragma unroll
    for (int r = 0; r < C::WPF; ++r) {
      const int idx = tid + NT * r;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const int n = idx / C::Q, q = idx % C::Q;
      if (idx < NP * C::Q && n < d.N) v = *reinterpret_cast<const f32x4*>(d.w + (size_t)n * d.Kp + tap * CIN + 4 * q);
      wr[r] = v;
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int r = 0; r < C::WPF; ++r) {
      const int idx = tid + NT * r;
      if (idx < NP * C::Q) {
        const int n = idx / C::Q, q = idx % C::Q;
        float2* dst = reinterpret_cast<float2*>(wbuf + buf * C::WBUF + n * C::CS + 4 * q);
        dst[0] = make_float2(wr[r][0], wr[r][1]);
        dst[1] = make_float2(wr[r][2], wr[r][3]);
      }
    }
  };
  load_w(0);
  store_w(0);
  __syncthreads();

  f32x16 acc[C::TM][1];
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][0][r] = 0.f;

  // per-wave pixel rows: local pixel p -> (p / TW, p % TW) of the tile
  int abase[C::TM];
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    const int p = (wm * C::TM + i) * 32 + li;
    abase[i] = ((p / TW) * HW + (p % TW)) * C::CS + lh * C::HC;
  }
  const int bbase = (wn * 32 + li) * C::CS + lh * C::HC;

  for (int tap = 0; tap < 9; ++tap) {
    if (tap + 1 < 9) load_w(tap + 1);
    const int toff = ((tap / 3) * HW + (tap % 3)) * C::CS;
    const float* wb = wbuf + (tap & 1) * C::WBUF + bbase;
#pragma unroll
    for (int s2 = 0; s2 < C::HC / 2; ++s2) {
      const float2 b = *reinterpret_cast<const float2*>(wb + 2 * s2);
#pragma unroll
      for (int i = 0; i < C::TM; ++i) {
        const float2 a = *reinterpret_cast<const float2*>(halo + abase[i] + toff + 2 * s2);
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, acc[i][0], 0, 0, 0);
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, acc[i][0], 0, 0, 0);
      }
    }
    if (tap + 1 < 9) store_w((tap + 1) & 1);
    __syncthreads();
  }

  const int M = d.nimg * H * W;
  epilogue_tiles<C::TM, 1>(d, lds, acc, wave, lane, wn * 32, M, [&](int r) {
    const int p = wm * C::TM * 32 + r;
    const int gy = y0 + p / TW, gx = x0 + p % TW;
    return (gy < H && gx < W) ? (img * H + gy) * W + gx : -1;
  });
}

// Persistent variant for <= 32 output channels (ERes2NetV2 / ERes2Net-large stage 1,
// CAM++ FCM): all nine taps of the weights stay resident in LDS for the life of the block,
// and the next tile's input halo is loaded into registers while the MFMAs of the current
// tile run, so HBM latency is hidden behind compute instead of being paid once per tile.
// Grid = min(tiles, 2 x CUs); tiles are dealt round-robin (block-uniform trip count).
template <int CIN, bool ADD>
struct PersistCfg {
  static constexpr int NP = 32, PIX = 256, NW = 8, NT = 512;
  static constexpr int CS = CIN + 2, HC = CIN / 2, Q = CIN / 4;
  static constexpr int HALO_PIX = 340;                              // (TH+2)(TW+2), TW in {8, 16, 32}
  static constexpr int HALO = HALO_PIX * CS;
  static constexpr int WRES = 9 * NP * CS;
  static constexpr int EPI = NW * 1024;                             // aliases the halo after the taps
  static constexpr int LDS = (HALO > EPI ? HALO : EPI) + WRES;
  static constexpr int PF = (HALO_PIX * Q + NT - 1) / NT;           // prefetch float4 per thread
};

template <int CIN, int TW, bool ADD>
__global__ void __launch_bounds__(512, 2)
conv3x3_halo_persistent_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
  using C = PersistCfg<CIN, ADD>;
  __shared__ __attribute__((aligned(16))) float lds[C::LDS];
  float* halo = lds;
  float* wres = lds + (C::HALO > C::EPI ? C::HALO : C::EPI);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  constexpr int TH = C::PIX / TW, HW = TW + 2, HH = TH + 2;   // compile-time: no integer divides
  constexpr int hq = HH * HW * C::Q;
  const int H = d.Ho, W = d.Wo;
  const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
  const int ntiles = d.nimg * ntx * nty;

  f32x4 pa[C::PF], pb[ADD ? C::PF : 1];
  // tile t's halo (or, with which = 1, its Res2Net addend) -> registers
  auto pf_load = [&](int t, int which) {
    const int img = t / (ntx * nty), ty = (t / ntx) % nty, tx = t % ntx;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const float* src = which ? d.s0.p2 : d.s0.p;
    const int ld = which ? d.s0.ld2 : d.s0.ld;
#pragma unroll
    for (int r = 0; r < C::PF; ++r) {
      const int idx = tid + C::NT * r;
      const int q = idx % C::Q, p = idx / C::Q;
      const int gy = y0 + p / HW, gx = x0 + p % HW;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (idx < hq && gy >= 0 && gy < H && gx >= 0 && gx < W)
        v = *reinterpret_cast<const f32x4*>(src + ((size_t)(img * H + gy) * W + gx) * ld + 4 * q);
      if (which) pb[r] = v;
      else pa[r] = v;
    }
  };
  auto pf_store = [&]() {
#pragma unroll
    for (int r = 0; r < C::PF; ++r) {
      const int idx = tid + C::NT * r;
      if (idx < hq) {
        f32x4 v = pa[r];
        if (ADD) v += pb[r];
        const int q = idx % C::Q, p = idx / C::Q;
        float2* dst = reinterpret_cast<float2*>(halo + p * C::CS + 4 * q);
        dst[0] = make_float2(v[0], v[1]);
        dst[1] = make_float2(v[2], v[3]);
      }
    }
  };

  int t = blockIdx.x;
  if (t < ntiles) {
    pf_load(t, 0);
    if (ADD) pf_load(t, 1);
  }
  // all nine taps of the weights -> LDS ([tap][n][CS]); rows n >= N are zero
  for (int idx = tid; idx < 9 * C::NP * C::Q; idx += C::NT) {
    const int q = idx % C::Q, n = (idx / C::Q) % C::NP, tap = idx / (C::Q * C::NP);
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (n < d.N) v = *reinterpret_cast<const f32x4*>(d.w + (size_t)n * d.Kp + tap * CIN + 4 * q);
    float2* dst = reinterpret_cast<float2*>(wres + (tap * C::NP + n) * C::CS + 4 * q);
    dst[0] = make_float2(v[0], v[1]);
    dst[1] = make_float2(v[2], v[3]);
  }
  if (t < ntiles) pf_store();
  __syncthreads();

  f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};               // loaded once: see epilogue_tiles pre_bias
  {
    const int n = (lane & 7) * 4;
    if (d.bias && n < d.N) bias4 = *reinterpret_cast<const f32x4*>(d.bias + n);
  }
  const int p_own = wave * 32 + li;                 // this lane's A row (pixel of the tile)
  const int abase = ((p_own / TW) * HW + (p_own % TW)) * C::CS + lh * C::HC;
  const int bbase = li * C::CS + lh * C::HC;
  for (; t < ntiles; t += gridDim.x) {
    const int tn = t + gridDim.x;
    if (tn < ntiles) pf_load(tn, 0);                // in flight during the taps below
    f32x16 acc[1][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const float* a = halo + abase + ((tap / 3) * HW + (tap % 3)) * C::CS;
      const float* b = wres + tap * C::NP * C::CS + bbase;
#pragma unroll
      for (int s2 = 0; s2 < C::HC / 2; ++s2) {
        const float2 av = *reinterpret_cast<const float2*>(a + 2 * s2);
        const float2 bv = *reinterpret_cast<const float2*>(b + 2 * s2);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc[0][0], 0, 0, 0);
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc[0][0], 0, 0, 0);
      }
    }
    if (ADD && tn < ntiles) pf_load(tn, 1);         // the addend: in flight during the epilogue
    __syncthreads();                                // halo reads done: the epilogue reuses it
    {
      const int img = t / (ntx * nty), ty = (t / ntx) % nty, tx = t % ntx;
      const int y0 = ty * TH, x0 = tx * TW;
      epilogue_tiles<1, 1, true>(d, lds, acc, wave, lane, 0, d.nimg * H * W, [&](int r) {
        const int p = wave * 32 + r;
        const int gy = y0 + p / TW, gx = x0 + p % TW;
        return (gy < H && gx < W) ? (img * H + gy) * W + gx : -1;
      }, &bias4);
    }
    __syncthreads();                                // epilogue LDS reads done
    if (tn < ntiles) pf_store();
    __syncthreads();
  }
}

// fp16x3 variant of the persistent kernel (conv_gemm.hip "fp16x3"): the halo and the
// resident weights are held as fp16 hi / lo planes, channels padded to CINP (a multiple of
// 16: one 16-deep k-step per 16 channels per tap), pixel rows of CINP + 8 halves
// (conflict-free ds_read_b128).  A block computes 32 output channels; with N > 32 the
// channel halves go to the blocks b and b + 8 (same XCD, so the second halo read of a
// tile is an L2 hit).  The halo loads are unconditional (clamped address, zero applied
// from a mask at staging) so they stay in flight across the taps.
//
// KS = 2 k-groups: the LDS (halo + all nine taps of the weights, ~140 KB) allows one block
// per CU, so with one wave per 32-pixel tile a SIMD would run a single wave and expose
// every LDS and barrier latency.  Instead a second group of NW waves computes the same
// output tiles over the other half of each tap's 16-deep k-steps; its partial sums meet
// the first group's in LDS before the epilogue (two waves per SIMD, half the MFMA chain
// per wave, halo staging spread over twice the threads).
// SH = 2: frequency (row) stride 2 (CAM++ FCM: the stride-(2, 1) 3x3 convs); an output
// tile of TH rows then reads 2 TH + 1 input rows.
template <int CIN, int PIX, int KS, int SH = 1>
struct HaloX3Cfg {
  static constexpr int NP = 32, NW = PIX / 32, NT = 64 * NW * KS;
  static constexpr int CINP = (CIN + 15) / 16 * 16, QP = CINP / 4, Q = CIN / 4;
  static constexpr int KSTEPS = CINP / 16, KSG = KSTEPS / KS;       // k-steps per tap / per group
  // 16x16x32 form where a group's tap is whole 32-deep steps (not the SH = 2 form, KSG = 1)
  // and two k-groups (52 / 64 channels): the one-group forms (28 / 32 channels) would need 92
  // instead of 76 KB of LDS for the wider rows, one block per CU instead of two (CAM++ FCM halo
  // launches 1.29 -> 1.76 ms, r06_ablation/halo_m16_ab.txt)
  static constexpr bool M16 = SPK_HALO_M16 != 0 && KSG % 2 == 0 && KS == 2;
  // pixel / weight rows: CINP + 8 halves (conflict-free for the 32x32x16 reads); the 16x16x32
  // reads (lane: row l & 15, 16-B block l >> 4; ds_read_b128 lane groups {0-3, 12-15, 20-27},
  // ...) need a row stride of 6 or 10 16-B units: CINP + 16 halves for CINP = 32 / 64
  static constexpr int ROW = M16 ? CINP + 16 : CINP + 8;
  static_assert(KSTEPS % KS == 0, "k-steps must split evenly over the groups");
  // max over TW in {8, 16, 32} of (SH (TH - 1) + 3)(TW + 2)
  static constexpr int HALO_PIX = SH == 1 ? (PIX == 256 ? 340 : 204) : (PIX == 256 ? 594 : 330);
  static constexpr int HALO_F = HALO_PIX * ROW;                     // floats = hi + lo halves
  static constexpr int WRES_F = 9 * NP * ROW;                       // floats = hi + lo halves
  static constexpr int SLAB = epi_slab_floats<M16>();               // one 32x32 tile's slab
  static constexpr int EPI = NW * SLAB * KS;                        // epilogue slabs + partner sums
  static constexpr int LDS = (HALO_F > EPI ? HALO_F : EPI) + WRES_F;
  static constexpr int PF = (HALO_PIX * QP + NT - 1) / NT;          // staged float4 per thread
};

// two k-groups where a tap has four k-steps (52 / 64 channels: -8 % per launch on
// ERes2NetV2 layer2); with two k-steps (28 / 32) measured neutral to +1 %, so one group
constexpr int halo_ks(int cin, int sh = 1) { return cin > 32 || sh == 2 ? 2 : 1; }
// (the frequency-strided form holds a 1.5x taller halo: one block per CU, so it takes the
// second k-group too, for two waves per SIMD)

template <int CIN, int TW, bool ADD, int PIX, int KS, bool PLAIN, int SH>
__global__ void __launch_bounds__(64 * (PIX / 32) * KS, 1)
conv3x3_halo_x3_kernel(const ConvDesc d, int nsplit) {
  SPK_GATE(d.run_if);
  using C = HaloX3Cfg<CIN, PIX, KS, SH>;
  // scaled split (common.h): operand x 2^-s at staging, accumulators x 2^s after the taps
  const float sc = range_scale_flat(d.range_in), back = pow2_div(sc, 0), back_x = pow2_div(sc, -11);
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) float lds[C::LDS];
  _Float16* hh = reinterpret_cast<_Float16*>(lds);                 // halo hi plane
  _Float16* hlo = hh + C::HALO_PIX * C::ROW;                        // halo lo plane
  _Float16* wh = reinterpret_cast<_Float16*>(lds + (C::HALO_F > C::EPI ? C::HALO_F : C::EPI));
  _Float16* wl = wh + 9 * C::NP * C::ROW;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  constexpr int TH = PIX / TW, HW = TW + 2, HH = SH * (TH - 1) + 3;
  constexpr int hq = HH * HW * C::QP;
  static_assert(HH * HW <= C::HALO_PIX, "halo buffer");
  const int H = d.Ho, W = d.Wo;                     // output
  const int Hin = d.s0.H, Win = d.s0.W;             // input (SH = 1: the same)
  const int ntx = (W + TW - 1) / TW, nty = (H + TH - 1) / TH;
  const int ntiles = d.nimg * ntx * nty;
  // channel slice: blocks b and b+8 (one XCD) share tiles, one per 32-channel slice
  const int b = blockIdx.x;
  const int slice = nsplit > 1 ? (b >> 3) % nsplit : 0;
  const int tbase = nsplit > 1 ? (b & 7) + 8 * (b / (8 * nsplit)) : b;
  const int tstride = gridDim.x / nsplit;
  const int n0 = slice * C::NP;

  // Halo element r of this thread: quad qq (the same for every r, NT % QP == 0) of halo
  // pixel p = tid / QP + (NT / QP) * r.  Its (row, column) in the halo is tile-invariant,
  // so it is computed once and kept packed (row << 16 | column); elements past the halo and
  // padding quads get a row no image has.  Per tile a load then costs an add, two unsigned
  // bounds compares and one buffer load through a per-image resource (out-of-range offsets
  // read zeros), instead of a divide chain and 64-bit address arithmetic.
  static_assert(C::NT % C::QP == 0, "halo quads must tile the block");
  const int qq = tid % C::QP;
  uint32_t hrc[C::PF];
#pragma unroll
  for (int r = 0; r < C::PF; ++r) {
    const int idx = tid + C::NT * r;
    const int p = idx / C::QP;
    hrc[r] = (idx < hq && qq < C::Q) ? ((uint32_t)(p / HW) << 16) | (uint32_t)(p % HW) : 0x7FFF0000u;
  }
  const size_t img_px = (size_t)Hin * Win;
  // SPK_HALO_PF2: two tiles' halos in flight (register sets 0 / 1, the loop unrolled by two so
  // the set is a compile-time index): a tile's halo is requested at the start of the tile two
  // ahead, i.e. a whole tile earlier than with one set
  constexpr int NSET = SPK_HALO_PF2 ? 2 : 1;
  f32x4 pa[NSET][C::PF], pb[NSET][ADD ? C::PF : 1];
  auto pf_load = [&](int t, auto setc) {
    constexpr int S = decltype(setc)::value;
    const int img = t / (ntx * nty), ty = (t / ntx) % nty, tx = t % ntx;
    const int y0 = ty * TH * SH - 1, x0 = tx * TW - 1;
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(d.s0.p + img * img_px * d.s0.ld);
    __amdgpu_buffer_rsrc_t r2;
    if (ADD) r2 = make_rsrc(d.s0.p2 + img * img_px * d.s0.ld2);
#pragma unroll
    for (int r = 0; r < C::PF; ++r) {
      const int gy = y0 + (int)(hrc[r] >> 16), gx = x0 + (int)(hrc[r] & 0xFFFFu);
      const bool ok = ((unsigned)gy < (unsigned)Hin) & ((unsigned)gx < (unsigned)Win);
      const uint32_t pix = (uint32_t)(gy * Win + gx);
      // offsets materialised in registers before the loads (the empty asm keeps the
      // compiler from turning the select into a branch around the load: a load on only
      // some paths leaves its wait count unknown, and every later wait becomes vmcnt(0))
      uint32_t oa = ok ? (pix * (uint32_t)d.s0.ld + 4u * qq) * 4u : BUF_OOB;
      asm volatile("" : "+v"(oa));
      pa[S][r] = buf_load4(r0, oa);
      if (ADD) {
        uint32_t ob = ok ? (pix * (uint32_t)d.s0.ld2 + 4u * qq) * 4u : BUF_OOB;
        asm volatile("" : "+v"(ob));
        pb[S][r] = buf_load4(r2, ob);
      }
    }
  };
  auto pf_store = [&](auto setc) {
    constexpr int S = decltype(setc)::value;
    split_pass(sc, [&](auto split) {                // scaled split (common.h) when the word is set
#pragma unroll
      for (int r = 0; r < C::PF; ++r) {
        const int idx = tid + C::NT * r;
        if (idx < hq) {
          f32x4 v = pa[S][r];
          if (ADD) v += pb[S][r];
          const int q = qq, p = idx / C::QP;
          f16x4 h, l;
          split(v, h, l);
          *reinterpret_cast<f16x4*>(hh + p * C::ROW + 4 * q) = h;
          *reinterpret_cast<f16x4*>(hlo + p * C::ROW + 4 * q) = l;
        }
      }
    });
  };
  using Set0 = std::integral_constant<int, 0>;
  using Set1 = std::integral_constant<int, NSET - 1>;

  // the epilogue's bias quad, loaded once, before the first halo prefetch so that
  // the first wait for the halo retires it too (otherwise the compiler keeps it pending and
  // waits vmcnt(0) at its use in every tile; see epilogue_tiles: with the next tile's halo in
  // flight, a per-tile bias load would wait for the whole prefetch)
  f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};
  {
    const int n = n0 + (lane & 7) * 4;
    if (d.bias && n < d.N) bias4 = *reinterpret_cast<const f32x4*>(d.bias + n);
  }
  int t = tbase;
  if (t < ntiles) pf_load(t, Set0{});
  // all nine taps of this slice's split weights -> LDS ([tap][n][ROW] hi / lo); zero padded
  for (int idx = tid; idx < 9 * C::NP * C::QP; idx += C::NT) {
    const int q = idx % C::QP, n = (idx / C::QP) % C::NP, tap = idx / (C::QP * C::NP);
    typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
    u16x4 h = {0, 0, 0, 0}, l = {0, 0, 0, 0};
    if (n0 + n < d.N && q < C::Q) {
      const size_t o = (size_t)(n0 + n) * d.Kp + tap * CIN + 4 * q;
      h = *reinterpret_cast<const u16x4*>(d.wh + o);
      l = *reinterpret_cast<const u16x4*>(d.wl + o);
    }
    *reinterpret_cast<u16x4*>(wh + (tap * C::NP + n) * C::ROW + 4 * q) = h;
    *reinterpret_cast<u16x4*>(wl + (tap * C::NP + n) * C::ROW + 4 * q) = l;
  }
  if (t < ntiles) pf_store(Set0{});
  if (NSET == 2 && t + tstride < ntiles) pf_load(t + tstride, Set1{});
  __syncthreads();

  const int kg = wave / C::NW, pw = wave % C::NW;                  // k-group, pixel wave
  const int p_own = pw * 32 + li;
  const int abase = ((p_own / TW) * SH * HW + (p_own % TW)) * C::ROW + 8 * lh + 16 * C::KSG * kg;
  const int bbase = li * C::ROW + 8 * lh + 16 * C::KSG * kg;
  // 16x16x32 form: pixel block q of the wave (pixels 16 q .. 16 q + 15), channel block q
  int abase16[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = pw * 32 + 16 * q + (lane & 15);
    abase16[q] = ((p / TW) * SH * HW + (p % TW)) * C::ROW + 8 * (lane >> 4) + 16 * C::KSG * kg;
  }
  const int bbase16 = (lane & 15) * C::ROW + 8 * (lane >> 4) + 16 * C::KSG * kg;
  // one tile; S = the register set this tile's successor-but-one is loaded into
  auto tile = [&](int t, auto setc) {
    constexpr int S = decltype(setc)::value;
    const int tn = t + tstride;
#if SPK_EXP != 1
    if (NSET == 2) {                                // in flight during this tile and the next
      // unconditional (past the end: the last tile again), so the loads are on every path
      // and the wait for the older set is a count that leaves these in flight
      pf_load(min(tn + tstride, ntiles - 1), setc);
    } else if (tn < ntiles) {                       // in flight during the taps and epilogue
      pf_load(tn, setc);
    }
#endif
    f32x16 acc[1][1];
    if constexpr (C::M16) {
      // 16x16x32 form: a tap's KSG 16-deep steps are KSG / 2 32-deep ones; the wave's 32
      // pixels x 32 channels are 2 x 2 blocks of 16 (lane l: pixel / channel l & 15 of a
      // block, k 8 (l >> 4) .. +7), two accumulator sets as before (hi x hi; the cross terms)
      f32x4 a4[2][2], x4[2][2];
#pragma unroll
      for (int pb = 0; pb < 2; ++pb)
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          a4[pb][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
          x4[pb][cb] = a4[pb][cb];
        }
#pragma unroll 3
      for (int tap = 0; tap < (SPK_EXP == 3 ? 0 : 9); ++tap) {
        const int toff = ((tap / 3) * HW + (tap % 3)) * C::ROW;
#pragma unroll
        for (int s = 0; s < C::KSG / 2; ++s) {
          f16x8 ah[2], al[2], bh[2], bl[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int ao = abase16[q] + toff + 32 * s;
            ah[q] = *reinterpret_cast<const f16x8*>(hh + ao);
            al[q] = *reinterpret_cast<const f16x8*>(hlo + ao);
            const int bo = tap * C::NP * C::ROW + bbase16 + q * 16 * C::ROW + 32 * s;
            bh[q] = *reinterpret_cast<const f16x8*>(wh + bo);
            bl[q] = *reinterpret_cast<const f16x8*>(wl + bo);
          }
#pragma unroll
          for (int pb = 0; pb < 2; ++pb)
#pragma unroll
            for (int cb = 0; cb < 2; ++cb) {
              a4[pb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[pb], bh[cb], a4[pb][cb], 0, 0, 0);
              x4[pb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[pb], bl[cb], x4[pb][cb], 0, 0, 0);
              x4[pb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[pb], bh[cb], x4[pb][cb], 0, 0, 0);
            }
        }
      }
      // quadrant q = 2 pb + cb at elements 4q .. 4q + 3 (epilogue_tiles L16 layout)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc[0][0][4 * q + e] = a4[q >> 1][q & 1][e] * back + x4[q >> 1][q & 1][e] * back_x;
    } else {
      f32x16 accx;
#pragma unroll
      for (int r = 0; r < 16; ++r) { acc[0][0][r] = 0.f; accx[r] = 0.f; }
#pragma unroll 3
      for (int tap = 0; tap < (SPK_EXP == 3 ? 0 : 9); ++tap) {
        const int aoff = abase + ((tap / 3) * HW + (tap % 3)) * C::ROW;
        const int boff = tap * C::NP * C::ROW + bbase;
#pragma unroll
        for (int s = 0; s < C::KSG; ++s) {
          const f16x8 ah = *reinterpret_cast<const f16x8*>(hh + aoff + 16 * s);
          const f16x8 al = *reinterpret_cast<const f16x8*>(hlo + aoff + 16 * s);
          const f16x8 bh = *reinterpret_cast<const f16x8*>(wh + boff + 16 * s);
          const f16x8 bl = *reinterpret_cast<const f16x8*>(wl + boff + 16 * s);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, acc[0][0], 0, 0, 0);
          accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, accx, 0, 0, 0);
          accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, accx, 0, 0, 0);
        }
      }
      acc[0][0] = acc[0][0] * back + accx * back_x;
    }
    __syncthreads();                                // halo reads done: the epilogue reuses it
    const int img = t / (ntx * nty), ty = (t / ntx) % nty, tx = t % ntx;
    const int y0 = ty * TH, x0 = tx * TW;
    if constexpr (KS > 1 && PLAIN) {
      // balanced epilogue: both k-groups' partial sums go to LDS (MFMA C layout, rows =
      // pixels), then every wave finishes half the rows of its pixel tile (group kg: rows
      // 16 kg .. 16 kg + 15) -- bias, activation, two row-quad stores per lane -- so all
      // eight waves store (one group used to idle through the epilogue) and every wave issues
      // the same stores, which keeps the next halos' wait counts exact
      constexpr int SROW = epi_srow<C::M16>();
      float* slab = lds + (kg * C::NW + pw) * C::SLAB;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if constexpr (C::M16)
          slab[(16 * (r >> 3) + 4 * (lane >> 4) + (r & 3)) * SROW + 16 * ((r >> 2) & 1) + (lane & 15)] = acc[0][0][r];
        else
          slab[((r & 3) + 8 * (r >> 2) + 4 * lh) * SROW + li] = acc[0][0][r];
      }
      __syncthreads();
      const float* s0 = lds + pw * C::SLAB;
      const float* s1 = lds + (C::NW + pw) * C::SLAB;
      const int c4 = (lane & 7) * 4, n = n0 + c4, M = d.nimg * H * W;
      float amax = 0.f;
      f32x4 o[2];
      int mq[2];
      auto act_rows = [&](auto actc) {
        constexpr int A = decltype(actc)::value;   // -1: general
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rl = 16 * kg + 8 * q + (lane >> 3);
          const int p = pw * 32 + rl;
          const int gy = y0 + p / TW, gx = x0 + p % TW;
          mq[q] = (gy < H && gx < W) ? (img * H + gy) * W + gx : -1;
          // group 0's partial + group 1's, then the bias: the order the two-step form used
          o[q] = *reinterpret_cast<const f32x4*>(s0 + rl * SROW + c4) + *reinterpret_cast<const f32x4*>(s1 + rl * SROW + c4) +
                 bias4;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (A >= 0) o[q][e] = apply_act(o[q][e], A);
            else o[q][e] = apply_act(apply_act(o[q][e], d.act), d.act2);
          }
        }
      };
      if (d.act2 == ACT_NONE && d.act == ACT_HTANH) act_rows(std::integral_constant<int, ACT_HTANH>{});
      else if (d.act2 == ACT_NONE && d.act == ACT_RELU) act_rows(std::integral_constant<int, ACT_RELU>{});
      else act_rows(std::integral_constant<int, -1>{});
#if SPK_EXP != 2
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if (n < d.N && mq[q] >= 0 && mq[q] < M) {
          amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[q][0]), fabsf(o[q][1])), fmaxf(fabsf(o[q][2]), fabsf(o[q][3]))));
          *reinterpret_cast<f32x4*>(d.out + (size_t)mq[q] * d.ldo + n) = o[q];
        }
      }
      range_note(d.range_flag, amax);
#else
      if (o[0][0] == 12345.f) d.out[img + y0 + x0] = 1.f;
#endif
    } else {
      if constexpr (KS > 1) {                       // group 1's partial sums -> group 0
        float* part = lds + (C::NW + pw) * C::SLAB;
        if (kg == 1) {
#pragma unroll
          for (int r = 0; r < 16; ++r) part[r * 64 + lane] = acc[0][0][r];
        }
        __syncthreads();
        if (kg == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[0][0][r] += part[r * 64 + lane];
        }
      }
      if (kg == 0) {
#if SPK_EXP != 2
        epilogue_tiles<1, 1, true, PLAIN, false, C::M16>(d, lds, acc, pw, lane, n0, d.nimg * H * W, [&](int r) {
          const int p = pw * 32 + r;
          const int gy = y0 + p / TW, gx = x0 + p % TW;
          return (gy < H && gx < W) ? (img * H + gy) * W + gx : -1;
        }, &bias4);
#else
        if (acc[0][0][0] == 12345.f) d.out[img + y0 + x0] = 1.f;
#endif
      }
    }
    __syncthreads();                                // epilogue LDS reads done
    if (tn < ntiles) pf_store(std::integral_constant<int, NSET == 2 ? 1 - S : 0>{});
    __syncthreads();
  };
  if constexpr (NSET == 2) {
    for (; t < ntiles; t += 2 * tstride) {
      tile(t, Set0{});
      if (t + tstride < ntiles) tile(t + tstride, Set1{});
    }
  } else {
    for (; t < ntiles; t += tstride) tile(t, Set0{});
  }
}

// resident blocks per CU of a kernel (persistent grids must not exceed what is co-resident)
template <class K>
int resident_blocks(K kernel, int threads) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, threads, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}

template <int CIN, int TW, int PIX, bool ADD, bool PLAIN, int SH = 1>
hipError_t launch_halo_x3_k(const ConvDesc& d, int nsplit, int tiles, hipStream_t s) {
  constexpr int NT = HaloX3Cfg<CIN, PIX, halo_ks(CIN, SH), SH>::NT;
  auto k = conv3x3_halo_x3_kernel<CIN, TW, ADD, PIX, halo_ks(CIN, SH), PLAIN, SH>;
  static const int per_cu = resident_blocks(k, NT);
  // nsplit blocks per tile group of 8; a multiple of 8 * nsplit (or everything when small)
  const int slots = per_cu * device_cus();
  const int g = std::min((tiles + 7) / 8 * 8, std::max(8, slots / nsplit / 8 * 8));
  hipLaunchKernelGGL(k, dim3(g * nsplit), dim3(NT), 0, s, d, nsplit);
  return hipGetLastError();
}

// PLAIN: no residual / post-affine / ragged mask, so the epilogue issues no load behind
// the next tile's halo prefetch (conv_epilogue.h); the common case (every Res2Net 3x3)
template <int CIN, int TW, int PIX>
hipError_t launch_halo_x3_tw(const ConvDesc& d, hipStream_t s) {
  constexpr int TH = PIX / TW;
  const int tiles = d.nimg * ((d.Ho + TH - 1) / TH) * ((d.Wo + TW - 1) / TW);
  const int nsplit = (d.N + 31) / 32;
  const bool plain = !d.res && !d.post_scale && !d.rowlen && !d.osplit &&
                     ((double)d.nimg * d.Ho * d.Wo * d.ldo + d.N) * 4.0 < 0x7FFFFFF0;
  if constexpr (CIN == 32) {   // CAM++ FCM: frequency-strided 3x3 (halo_conv_supported)
    if (d.s0.sh == 2)
      return plain ? launch_halo_x3_k<CIN, TW, PIX, false, true, 2>(d, nsplit, tiles, s)
                   : launch_halo_x3_k<CIN, TW, PIX, false, false, 2>(d, nsplit, tiles, s);
  }
  if (d.s0.p2)
    return plain ? launch_halo_x3_k<CIN, TW, PIX, true, true>(d, nsplit, tiles, s)
                 : launch_halo_x3_k<CIN, TW, PIX, true, false>(d, nsplit, tiles, s);
  return plain ? launch_halo_x3_k<CIN, TW, PIX, false, true>(d, nsplit, tiles, s)
               : launch_halo_x3_k<CIN, TW, PIX, false, false>(d, nsplit, tiles, s);
}

template <int CIN, int PIX>
hipError_t launch_halo_x3(const ConvDesc& d, int TW, hipStream_t s) {
  if (TW == 8) return launch_halo_x3_tw<CIN, 8, PIX>(d, s);
  if (TW == 16) return launch_halo_x3_tw<CIN, 16, PIX>(d, s);
  return launch_halo_x3_tw<CIN, 32, PIX>(d, s);
}

template <int CIN, int TW>
hipError_t launch_halo_persistent_tw(const ConvDesc& d, hipStream_t s) {
  constexpr int TH = 256 / TW;
  const int tiles = d.nimg * ((d.Ho + TH - 1) / TH) * ((d.Wo + TW - 1) / TW);
  if (d.s0.p2) {
    auto k = conv3x3_halo_persistent_kernel<CIN, TW, true>;
    static const int per_cu = resident_blocks(k, 512);
    hipLaunchKernelGGL(k, dim3(std::min(tiles, per_cu * device_cus())), dim3(512), 0, s, d);
  } else {
    auto k = conv3x3_halo_persistent_kernel<CIN, TW, false>;
    static const int per_cu = resident_blocks(k, 512);
    hipLaunchKernelGGL(k, dim3(std::min(tiles, per_cu * device_cus())), dim3(512), 0, s, d);
  }
  return hipGetLastError();
}

template <int CIN>
hipError_t launch_halo_persistent(const ConvDesc& d, int TW, hipStream_t s) {
  if (TW == 8) return launch_halo_persistent_tw<CIN, 8>(d, s);
  if (TW == 16) return launch_halo_persistent_tw<CIN, 16>(d, s);
  return launch_halo_persistent_tw<CIN, 32>(d, s);
}

template <int CIN, int NP, int PIX>
hipError_t launch_halo_t(const ConvDesc& d, int TW, hipStream_t s) {
  using C = HaloCfg<CIN, NP, PIX, false>;
  const int TH = PIX / TW;
  const int blocks = d.nimg * ((d.Ho + TH - 1) / TH) * ((d.Wo + TW - 1) / TW);
  if (d.s0.p2)
    hipLaunchKernelGGL((conv3x3_halo_kernel<CIN, NP, PIX, true>), dim3(blocks), dim3(64 * C::NW), 0, s, d, TW);
  else
    hipLaunchKernelGGL((conv3x3_halo_kernel<CIN, NP, PIX, false>), dim3(blocks), dim3(64 * C::NW), 0, s, d, TW);
  return hipGetLastError();
}

// pixel tile size + width with the least edge waste for an H x W image
void pick_tile(int H, int W, int np, int* pix, int* tw) {
  double best = 1e30;
  for (int P : {256, 128}) {
    if (np == 32 && P == 128) continue;   // 4-wave blocks: keep 256-pixel tiles
    for (int t : {8, 16, 32}) {   // TW = 64 would need a larger halo buffer (occupancy)
      const int th = P / t;
      if (th < 2) continue;
      const double cover = (double)((H + th - 1) / th) * th * ((W + t - 1) / t) * t;
      const double cost = cover / ((double)H * W) + (P == 128 ? 0.04 : 0.0);   // small-tile halo tax
      if (cost < best - 1e-9) { best = cost; *pix = P; *tw = t; }
    }
  }
}

}  // namespace

// the x3 kernel: lean epilogue (conv_epilogue.h), <= 64 output channels as 32-channel slices
bool x3_halo_ok(const ConvDesc& d) {
  return conv_use_x3() && d.wh && d.wl && d.N <= 64 && d.N % 4 == 0 && d.ldo % 4 == 0 &&
         (!d.res || d.ldr % 4 == 0) && !d.affx && !d.gate && !d.rowbias && d.ksplit == 1;
}

// tile width for a fixed pixel count: least edge waste
int pick_tw(int H, int W, int P) {
  double best = 1e30;
  int tw = 16;
  for (int t : {8, 16, 32}) {
    const int th = P / t;
    const double cover = (double)((H + th - 1) / th) * th * ((W + t - 1) / t) * t;
    if (cover < best - 1e-9) { best = cover; tw = t; }
  }
  return tw;
}

// the persistent kernel: <= 32 output channels and the lean epilogue (conv_epilogue.h)
bool persistent_ok(const ConvDesc& d) {
  return d.N <= 32 && (d.s0.cin == 28 || d.s0.cin == 32) && d.N % 4 == 0 && d.ldo % 4 == 0 &&
         (!d.res || d.ldr % 4 == 0) && !d.affx && !d.gate && !d.rowbias && d.ksplit == 1;
}

bool halo_conv_supported(const ConvDesc& d) {
  static const int off = [] {   // SPK_NO_HALO=1|28|52...: route those convs to the implicit GEMM (experiments)
    const char* e = std::getenv("SPK_NO_HALO");
    return e ? std::atoi(e) : 0;
  }();
  const ConvSrc& s = d.s0;
  if (off == 1 || (off > 1 && off == s.cin)) return false;
  if (s.vlen) return false;   // masked (pre-activated) inputs take the implicit GEMM
  // frequency stride 2: the x3 kernel's SH = 2 form, 32 input channels (CAM++ FCM)
  const bool geom = s.sh == 1 ? (d.Ho == s.H && d.Wo == s.W)
                              : (s.sh == 2 && s.cin == 32 && !s.p2 && s.ld2 == 0 && x3_halo_ok(d) &&
                                 d.Ho == (s.H - 1) / 2 + 1 && d.Wo == s.W);
  return !d.kcb && s.kh == 3 && s.kw == 3 && s.sw == 1 && s.ph == 1 && s.pw == 1 && s.dh == 1 && s.dw == 1 &&
         !s.reflect && !s.pre_scale && !d.s1.p && d.s1.cin == 0 && d.ksplit == 1 && d.N <= 64 &&
         (s.cin == 28 || s.cin == 32 || s.cin == 52 || s.cin == 64) && geom &&
         d.Kp >= 9 * s.cin && s.ld % 4 == 0 && (!s.p2 || s.ld2 % 4 == 0) &&
         // the x3 kernel addresses one image through a buffer resource (32-bit offsets)
         (double)s.H * s.W * std::max(s.ld, s.p2 ? s.ld2 : 0) * 4.0 < 0x7FFFFFF0 - 64;
}

std::string halo_kernel_name(const ConvDesc& d) {
  const int np = d.N <= 32 ? 32 : 64;
  int pix = 256, tw = 16;
  pick_tile(d.Ho, d.Wo, np, &pix, &tw);
  const bool add = d.s0.p2 != nullptr || d.s0.ld2 > 0;
  if (x3_halo_ok(d)) {
    const int px = 128;
    return "conv3x3_halo_x3_kernel<" + std::to_string(d.s0.cin) + ", " + std::to_string(pick_tw(d.Ho, d.Wo, px)) +
           ", " + (add ? "true" : "false") + ", " + std::to_string(px) + ", " + std::to_string(halo_ks(d.s0.cin, d.s0.sh)) + ", " +
           ((!d.res && d.ldr == 0 && !d.post_scale && !d.rowlen && !d.osplit &&
             ((double)d.nimg * d.Ho * d.Wo * d.ldo + d.N) * 4.0 < 0x7FFFFFF0) ? "true" : "false") + ", " +
           std::to_string(d.s0.sh) + ">";
  }
  if (persistent_ok(d))
    return "conv3x3_halo_persistent_kernel<" + std::to_string(d.s0.cin) + ", " + std::to_string(tw) + ", " +
           (add ? "true" : "false") + ">";
  return "conv3x3_halo_kernel<" + std::to_string(d.s0.cin) + ", " + std::to_string(np) + ", " + std::to_string(pix) +
         ", " + (add ? "true" : "false") + ">";
}

hipError_t launch_conv3x3_halo(const ConvDesc& d, hipStream_t s) {
  if (!halo_conv_supported(d)) return hipErrorInvalidValue;
  const int np = d.N <= 32 ? 32 : 64;
  int pix = 256, tw = 16;
  pick_tile(d.Ho, d.Wo, np, &pix, &tw);
#define SPK_HALO_CASE(CI)                                                               \
  if (d.s0.cin == CI) {                                                                 \
    if (np == 32) return launch_halo_t<CI, 32, 256>(d, tw, s);                          \
    return pix == 256 ? launch_halo_t<CI, 64, 256>(d, tw, s) : launch_halo_t<CI, 64, 128>(d, tw, s); \
  }
  if (x3_halo_ok(d)) {
    if (d.s0.cin == 28) return launch_halo_x3<28, 128>(d, pick_tw(d.Ho, d.Wo, 128), s);
    if (d.s0.cin == 32) return launch_halo_x3<32, 128>(d, pick_tw(d.Ho, d.Wo, 128), s);
    if (d.s0.cin == 52) return launch_halo_x3<52, 128>(d, pick_tw(d.Ho, d.Wo, 128), s);
    if (d.s0.cin == 64) return launch_halo_x3<64, 128>(d, pick_tw(d.Ho, d.Wo, 128), s);
  }
  if (persistent_ok(d) && d.s0.cin == 28) return launch_halo_persistent<28>(d, tw, s);
  if (persistent_ok(d) && d.s0.cin == 32) return launch_halo_persistent<32>(d, tw, s);
  SPK_HALO_CASE(28)
  SPK_HALO_CASE(32)
  SPK_HALO_CASE(52)
  SPK_HALO_CASE(64)
#undef SPK_HALO_CASE
  return hipErrorInvalidValue;
}

}  // namespace spk
