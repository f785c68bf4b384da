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
#include <cstdlib>
#include <string>
#include <type_traits>

#include "common.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

#ifndef SPK_GEXP
#define SPK_GEXP 0   // ablation builds only (tools/gemm_exp.sh): 6 no epilogue, 1 no MFMA, 2 no split, 3 no
                     // in-loop loads, 5 no in-loop LDS stores; 0 = the product kernel
#endif

namespace spk {

namespace {


constexpr int KP_ALIGN = 32;   // weights are packed with Kp a multiple of this

template <int BM, int BN, int BK, int WM, int WN, bool S1, bool ADD, bool PRE>
__global__ void __launch_bounds__(64 * WM * WN, 4)
conv_gemm_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
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

  // ---- A: asynchronous implicit-im2col loader (conv_loader.h); B rows clamped + masked
  const int kq = tid % QPR, row0 = tid / QPR;
  using AL = ALoader<AROWS, RPP, BK, S1, ADD, PRE>;
  AL al;
  al.init(d, m0, row0, kq, kt0);
  typename AL::Slot sa;
  f32x4 rb[BROWS];
  unsigned bok = 0;

  auto load_tile = [&](int kt) {
    al.load(d, sa);
    const int k = kt * BK + kq * 4;
    bok = 0;
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      const int nr = row0 + RPP * r;
      const bool ok = nr < BN && n0 + nr < d.N;
      const int n = ok ? n0 + nr : 0;
      rb[r] = *reinterpret_cast<const f32x4*>(d.w + (size_t)n * d.Kp + k);
      if (ok) bok |= 1u << r;
    }
  };

  auto store_tile = [&](int buf) {
    float* a = As + buf * BM * LDS_ROW;
    float* b = Bs + buf * BN * LDS_ROW;
#pragma unroll
    for (int r = 0; r < AROWS; ++r)
      *reinterpret_cast<f32x4*>(a + (row0 + RPP * r) * LDS_ROW + kq * 4) = al.value(sa, r);
#pragma unroll
    for (int r = 0; r < BROWS; ++r) {
      const int nr = row0 + RPP * r;
      if (nr < BN)
        *reinterpret_cast<f32x4*>(b + nr * LDS_ROW + kq * 4) = ((bok >> r) & 1) ? rb[r] : f32x4{0.f, 0.f, 0.f, 0.f};
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

// ---------------------------------------------------------------------------------------
// fp16x3: fp32-accurate GEMM on the fp16 matrix cores (v_mfma_f32_32x32x16_f16, 16x the
// fp32 MFMA's work per cycle).  Every operand x is split as hi = fp16(x) and
// lo = fp16((x - hi) * 2^11) (the 2^11 keeps lo out of the fp16 subnormal range), and
//   x * w  ~=  2^-11 * (hi_x * (2^11 hi_w)  +  hi_x * lo_w  +  lo_x * hi_w)
// with products exact and sums in fp32 (one accumulator); the dropped lo*lo term is
// 2^-22 relative.  Embeddings stay within the reference's own fp32-vs-fp64 noise
// (DESIGN.md §4).  Weights are split once at model creation (misc.hip split_f16);
// activations are split while they are staged into LDS (packed round-toward-zero
// conversions here: fewer VALU, lo still holds the remainder exactly to fp16 precision), so
// HBM traffic is unchanged (fp32 in, fp32 out).
//
// LDS per buffer: A hi / A lo / B hi / B lo planes, rows of BK = 32 halves padded to 40
// (80 B: the same conflict-free ds_read_b128 pattern as the fp32 kernel's 20-float rows).
// Lane half h owns k = 16h .. 16h+15 of the tile: k-step s reads halves 16h + 8s .. +7
// for both operands (a k permutation shared by A and B, so the products pair up).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));


template <int BM, int BN, int WM, int WN, bool X1 = false>
struct X3Cfg {
  static constexpr int BK = 32, NT = 64 * WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  static constexpr int QPR = BK / 4, RPP = NT / QPR, AROWS = BM / RPP;             // A: fp32 quads
  // B: 16-B chunks, four per 32-half row and plane; x3 spreads the block over both planes
  static constexpr int CPR = X1 ? 4 : 8, RPPB = NT / CPR, BROWS = (BN + RPPB - 1) / RPPB;
  static constexpr int LROW = BK + 8;                                               // halves
  static constexpr int PA = BM * LROW, PB = BN * LROW;
  static constexpr int NPL = X1 ? 1 : 2;               // planes per operand (hi, lo)
  static constexpr int STAGE = NPL * (PA + PB);        // halves per buffer = floats for both buffers
  static constexpr int LDS_EPI = WM * WN * TM * TN * 1024;
  static constexpr int LDS_FLOATS = STAGE > LDS_EPI ? STAGE : LDS_EPI;
};

// X1 = the single-product variant (C3's reduced-precision mode, spk_model_config_t
// precision = SPK_PRECISION_FP16): operands rounded to fp16 (round to nearest), one MFMA
// per product, fp32 accumulation; only the hi planes are staged.
template <int BM, int BN, int WM, int WN, bool S1, bool ADD, bool PRE, bool BUF, bool X1, bool SC>
__device__ __forceinline__ void conv_gemm_f16_body(const ConvDesc& d, float* lds, float sc_arg) {
  using C = X3Cfg<BM, BN, WM, WN, X1>;
  constexpr int BK = C::BK, TM = C::TM, TN = C::TN, RPP = C::RPP, AROWS = C::AROWS;
  static_assert(TM >= 1 && TN >= 1 && BM % RPP == 0, "tile shape");
  _Float16* hl = reinterpret_cast<_Float16*>(lds);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + BN - 1) / BN;
  const int nM = (M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, nM * nN);
  const int mt = lid / nN, nt = lid % nN;
  const int m0 = mt * BM, n0 = nt * BN;

  // scaled split (common.h): operand x 2^-s at staging, accumulator x 2^s before the epilogue
  // (SC = false: the in-range instance, scale 1 at compile time)
  const float sc = SC ? sc_arg : 1.0f;
  const auto split = [sc](const f32x4& v, h16x4& h, h16x4& l) {
    if constexpr (SC) split_x3s(v, sc, h, l);
    else split_x3(v, h, l);
  };
  const int nkt_all = d.Kp / BK;
  const int per = (nkt_all + d.ksplit - 1) / d.ksplit;
  const int kt0 = blockIdx.z * per;
  const int kt1 = min(nkt_all, kt0 + per);

  // ---- A: asynchronous implicit-im2col loader (conv_loader.h): the buffer-resource form
  // wherever the layer allows it (BUF), else the generic one (reflect padding, cin < 32)
  const int kq = tid % C::QPR, row0 = tid / C::QPR;
  using AL = typename std::conditional<BUF, BufALoader<AROWS, RPP, BK, S1, ADD, PRE>,
                                       ALoader<AROWS, RPP, BK, S1, ADD, PRE>>::type;
  AL al;
  al.init(d, m0, row0, kq, kt0);
  // ---- B chunk geometry: the first half of the block loads the hi plane, the second the
  // lo plane (wave-uniform, so each wave reads through one buffer resource); a thread owns
  // one 16-B quarter of a 32-half weight row.  Rows past N read zeros (offset past range).
  const int plane = X1 ? 0 : __builtin_amdgcn_readfirstlane(tid / (C::NT / 2));
  const int bq = tid & 3, brow0 = X1 ? tid >> 2 : (tid % (C::NT / 2)) >> 2;
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(plane ? d.wl : d.wh);
  uint32_t boff[C::BROWS];
#pragma unroll
  for (int r = 0; r < C::BROWS; ++r) {
    const int nr = brow0 + C::RPPB * r;
    boff[r] = (nr < BN && n0 + nr < d.N) ? ((uint32_t)(n0 + nr) * d.Kp + bq * 8) * 2u : BUF_OOB;
  }

  // two register sets: the loads of K-tile kt+2 are issued before the MFMAs of tile kt, so
  // every load has two K-steps of compute to land (prefetch distance 2, LDS double buffer)
  struct Set {
    typename AL::Slot a;
    u32x4 b[C::BROWS];
  };
  Set set0, set1;

  auto load_tile = [&](int kt, Set& st) {
    al.load(d, st.a);
    const int koff = __builtin_amdgcn_readfirstlane(kt * BK * 2);   // uniform: no waterfall (T20)
#pragma unroll
    for (int r = 0; r < C::BROWS; ++r) st.b[r] = __builtin_amdgcn_raw_buffer_load_b128(brs, (int)boff[r], koff, 0);
  };

  auto store_tile = [&](int buf, const Set& st) {
    _Float16* ahi = hl + buf * C::STAGE;
    _Float16* alo = ahi + C::PA;
    _Float16* bpl = ahi + C::NPL * C::PA + plane * C::PB;
    // packed round-toward-zero split (conv_epilogue.h split_x3; measured -0.3 ms per ERes2NetV2
    // forward against per-element round-to-nearest conversions), or the scaled split
    {
#pragma unroll
      for (int r = 0; r < AROWS; ++r) {
        const f32x4 v = al.value(st.a, r);
        const int off = (row0 + RPP * r) * C::LROW + kq * 4;
        if constexpr (X1) {
          *reinterpret_cast<f16x4*>(ahi + off) = __builtin_convertvector(v * sc, f16x4);
        } else {
          f16x4 h, l;
#if SPK_GEXP == 2
          h = __builtin_convertvector(v, f16x4);
          l = h;
#else
          split(v, h, l);
#endif
          *reinterpret_cast<f16x4*>(ahi + off) = h;
          *reinterpret_cast<f16x4*>(alo + off) = l;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < C::BROWS; ++r) {
      const int nr = brow0 + C::RPPB * r;
      if (nr < BN) *reinterpret_cast<u32x4*>(bpl + nr * C::LROW + bq * 8) = st.b[r];
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
  auto compute = [&](int buf) {
    const _Float16* ahi = hl + buf * C::STAGE;
    const _Float16* bhi = ahi + C::NPL * C::PA;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const _Float16* p = ahi + (wm * C::WTM + i * 32 + li) * C::LROW + lh * 16 + 8 * s;
        ah[i] = *reinterpret_cast<const f16x8*>(p);
        if constexpr (!X1) al[i] = *reinterpret_cast<const f16x8*>(p + C::PA);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const _Float16* p = bhi + (wn * C::WTN + j * 32 + li) * C::LROW + lh * 16 + 8 * s;
        bh[j] = *reinterpret_cast<const f16x8*>(p);
        if constexpr (!X1) bl[j] = *reinterpret_cast<const f16x8*>(p + C::PB);
      }
      // single accumulator: the hi x hi product takes the weights' hi plane scaled by 2^11
      // (exact: a power of two, |w| < 31.5 is checked on the host -- ConvDesc::wbig), so all
      // three products carry the same 2^11 and sum into one accumulator, scaled back once in
      // the epilogue (half the accumulator registers of a two-accumulator form; measured
      // -24 % on the 128x128 tiles, which then keep two blocks per CU)
      f16x8 bh2[TN];
      if constexpr (!X1) {
#pragma unroll
        for (int j = 0; j < TN; ++j) bh2[j] = bh[j] * (_Float16)2048.0f;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#if SPK_GEXP == 1
          acc[i][j][0] += (float)ah[i][0] + (float)bh[j][0] + (float)al[i][1] + (float)bl[j][1];
#else
          if constexpr (!X1) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh2[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          } else {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
#endif
        }
    }
  };
  if (kt0 < kt1) {
    load_tile(kt0, set0);
    load_tile(min(kt0 + 1, kt1 - 1), set1);
    store_tile(0, set0);
    __syncthreads();
    // The prefetches are unconditional (past the last K-tile they re-read it): a load that
    // only some paths issue makes the compiler's wait counting assume the short path and
    // wait for ALL loads (vmcnt(0)) before the LDS store, i.e. for the tile just issued.
    // Without a second operand the LDS store of the next tile is unconditional (past the
    // last tile it rewrites the idle buffer), so loads, MFMAs and stores share one basic
    // block and the compiler interleaves them (measured: -3% on the deep-K layers; with
    // the extra operand registers of S1/ADD the same change spills).
    constexpr bool UNCOND = !S1 && !ADD;
    for (int kt = kt0; kt < kt1; kt += 2) {
      // even step: LDS buffer 0 holds kt, set 1 holds kt+1 (in flight), set 0 is free
#if SPK_GEXP != 3
      load_tile(min(kt + 2, kt1 - 1), set0);
#endif
      compute(0);
#if SPK_GEXP != 5
      if (UNCOND || kt + 1 < kt1) store_tile(1, set1);
#endif
      __syncthreads();
      if (kt + 1 >= kt1) break;
      // odd step: buffer 1 holds kt+1, set 0 holds kt+2 (in flight), set 1 is free
#if SPK_GEXP != 3
      load_tile(min(kt + 3, kt1 - 1), set1);
#endif
      compute(1);
#if SPK_GEXP != 5
      if (UNCOND || kt + 2 < kt1) store_tile(0, set0);
#endif
      __syncthreads();
    }
  }
  {
    const float back = pow2_div(sc, X1 ? 0 : -11);   // 2^(-11) / sc, exact
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] *= back;
  }
#if SPK_GEXP == 6
  {   // ablation: no epilogue (every accumulator kept live through one conditional store)
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += acc[i][j][r];
    if (sum == 1234.5f) d.out[tid] = sum;
  }
#else
  epilogue_tiles<TM, TN>(d, lds, acc, wave, lane, n0 + wn * C::WTN, M, [&](int r) { return m0 + wm * C::WTM + r; });
#endif
}

// A 128-VGPR budget (4 waves per SIMD) for the <= 128x128 tiles: the in-range instance fits
// it without spills (125 VGPRs); a budget of 256 let the compiler take 160+ VGPRs and measured
// 16-23 % slower on every launch with more than one block per CU (ECAPA / CAM++ layers), even
// though the 80 KB of LDS allows two blocks per CU either way.  The scaled instance spills
// under this budget -- it runs only while the range word is set.
#ifndef SPK_X3_LB
#define SPK_X3_LB 4
#endif
// The body twice behind one uniform branch on the range word: the in-range instance is the
// unscaled kernel exactly (a scale threaded through one shared K loop measured +25 % on the
// 128x128 tiles: an extra VALU per value pair, and register copies of the accumulators where
// two loop copies merged), the scaled one (common.h scaled split) runs only when the word is set.
template <int BM, int BN, int WM, int WN, bool S1, bool ADD, bool PRE, bool BUF, bool X1>
__device__ __forceinline__ void conv_gemm_f16_entry(const ConvDesc& d) {
  SPK_GATE(d.run_if);
  __shared__ __attribute__((aligned(16))) float lds[X3Cfg<BM, BN, WM, WN, X1>::LDS_FLOATS];
  const float sc = range_scale(d.range_in);
  if (sc == 1.0f) conv_gemm_f16_body<BM, BN, WM, WN, S1, ADD, PRE, BUF, X1, false>(d, lds, 1.0f);
  else conv_gemm_f16_body<BM, BN, WM, WN, S1, ADD, PRE, BUF, X1, true>(d, lds, sc);
}

template <int BM, int BN, int WM, int WN, bool S1, bool ADD, bool PRE, bool BUF>
__global__ void __launch_bounds__(64 * WM * WN, (BM * BN <= 128 * 128) ? SPK_X3_LB : 1)
conv_gemm_x3_kernel(const ConvDesc d) {
  conv_gemm_f16_entry<BM, BN, WM, WN, S1, ADD, PRE, BUF, false>(d);
}

template <int BM, int BN, int WM, int WN, bool S1, bool ADD, bool PRE>
__global__ void __launch_bounds__(64 * WM * WN, (BM * BN <= 128 * 128) ? 2 : 1)
conv_gemm_x1_kernel(const ConvDesc d) {
  conv_gemm_f16_entry<BM, BN, WM, WN, S1, ADD, PRE, true, true>(d);
}

#ifndef SPK_CG_PART
// Split-K combine: out = epi(sum_z partial[z])   (fixed z order: deterministic)
__global__ void splitk_reduce_kernel(const ConvDesc d, int M) {
  SPK_GATE(d.run_if);
  const size_t total = (size_t)M * d.N;
  float amax = 0.f;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int m = e / d.N, n = e % d.N;
    float v = 0.f;
    for (int z = 0; z < d.ksplit; ++z) v += d.partial[(size_t)z * total + e];
    const float o = epilogue_elem(d, m, n, v);
    amax = fmaxf(amax, fabsf(o));
    *out_at(d, m, n) = o;
  }
  range_note(d.range_flag, amax);
}
#endif

}  // namespace

#ifndef SPK_CG_PART
// split-K combine of the partial slabs a GEMM launch left in d.partial (ksplit > 1)
hipError_t launch_splitk_reduce(const ConvDesc& d, hipStream_t s) {
  const int M = d.nimg * d.Ho * d.Wo;
  const size_t total = (size_t)M * d.N;
  const int rb = (int)std::min<size_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(rb), dim3(256), 0, s, d, M);
  return hipGetLastError();
}
#endif

namespace {

// fp16x3 split-precision MFMA (default) or exact fp32 MFMA (SPK_CONV_MFMA=f32)
bool use_x3() {
  static const bool x3 = [] {
    const char* e = std::getenv("SPK_CONV_MFMA");
    return !(e && std::string(e) == "f32");
  }();
  return x3;
}

// x3 tile override for experiments: SPK_X3_TILE=128x128 | 256x128 | 128x256 | 64x128
int x3_tile() {
  static const int t = [] {
    const char* e = std::getenv("SPK_X3_TILE");
    if (!e) return 0;
    const std::string v(e);
    return v == "256x128" ? 1 : v == "128x256" ? 2 : v == "128x128" ? 3 : v == "64x128" ? 4 : 0;
  }();
  return t;
}

struct Cfg {
  int bm, bn, bk, wm, wn;
};

#ifndef SPK_DEEP_K
#define SPK_DEEP_K 4096   // K from which the 256x128 tile is used
#endif

Cfg select_cfg(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int bk = d.Kp >= 256 ? 32 : 16;
  // N <= 32 (CAM++'s CAM local convs, 128 -> 32 at M = 25,344): 256-row tiles give 99 blocks
  // for 256 CUs; 64-row tiles (two waves) spread the same work over every CU
  if (d.N <= 32) return (M + 255) / 256 >= 512 ? Cfg{256, 32, bk, 8, 1} : Cfg{64, 32, bk, 2, 1};
  if (d.N <= 64) return {256, 64, bk, 4, 2};
  if (M <= 4096) return {64, 128, bk, 1, 4};
  if (use_x3() && d.wh && !d.wbig) {
    const int t = x3_tile();
    if (t == 1) return {256, 128, 32, 4, 2};
    if (t == 2) return {128, 256, 32, 2, 4};
    if (t == 3) return {128, 128, 32, 2, 4};
    if (t == 4) return {64, 128, 32, 1, 4};
    // measured per layer (tools/tile_exp.sh, round 3): with one accumulator the 128x128 tile
    // keeps two blocks (four waves per SIMD) per CU and is the fastest or within 2 % on every
    // x3 GEMM of ERes2NetV2 / ERes2Net-large (all-128x128 27.0 ms vs 28.6 for round 2's
    // per-layer mix); only the deepest K (the 4608-deep stage-3 downsample) keeps 256x128 (-5 %)
    if (d.Kp >= SPK_DEEP_K && d.N >= 512) return {256, 128, 32, 4, 2};
  }
  // 128x128 at BK=32 still fits two blocks per CU (73.7 KB LDS): half the K-steps, twice
  // the loads in flight per step -- what the short-K 1x1 convs need
  return {128, 128, 32, 2, 4};
}

// the fp16x3 / fp16 kernels of one tile (launch_tile decides that they apply: f16_path)
template <int BM, int BN, int WM, int WN>
hipError_t launch_f16(const ConvDesc& d, hipStream_t s) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int nblk = ((M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  dim3 grid(nblk, 1, d.ksplit);
  dim3 block(64 * WM * WN);
  const bool s1 = d.s1.p != nullptr, add = d.s0.p2 != nullptr, pre = d.s0.pre_scale != nullptr;
  if (d.x1 && d.wh && conv_buf_loader_ok(d, BM)) {
    if (s1) hipLaunchKernelGGL((conv_gemm_x1_kernel<BM, BN, WM, WN, true, false, false>), grid, block, 0, s, d);
    else if (add) hipLaunchKernelGGL((conv_gemm_x1_kernel<BM, BN, WM, WN, false, true, false>), grid, block, 0, s, d);
    else if (pre) hipLaunchKernelGGL((conv_gemm_x1_kernel<BM, BN, WM, WN, false, false, true>), grid, block, 0, s, d);
    else hipLaunchKernelGGL((conv_gemm_x1_kernel<BM, BN, WM, WN, false, false, false>), grid, block, 0, s, d);
  } else if (conv_buf_loader_ok(d, BM)) {
    if (s1) hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, true, false, false, true>), grid, block, 0, s, d);
    else if (add) hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, false, true, false, true>), grid, block, 0, s, d);
    else if (pre) hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, false, false, true, true>), grid, block, 0, s, d);
    else hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, false, false, false, true>), grid, block, 0, s, d);
  } else if (s1 || pre) {
    return hipErrorInvalidValue;   // no generic-loader instantiation (conv_buf_loader_ok)
  } else if (add) {
    hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, false, true, false, false>), grid, block, 0, s, d);
  } else {
    hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN, WM, WN, false, false, false, false>), grid, block, 0, s, d);
  }
  return hipGetLastError();
}

// the exact fp32 MFMA kernels of one tile
template <int BM, int BN, int BK, int WM, int WN>
hipError_t launch_f32(const ConvDesc& d, hipStream_t s) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int nblk = ((M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  dim3 grid(nblk, 1, d.ksplit);
  dim3 block(64 * WM * WN);
  const bool s1 = d.s1.p != nullptr, add = d.s0.p2 != nullptr, pre = d.s0.pre_scale != nullptr;
  if (s1) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, true, false, false>), grid, block, 0, s, d);
  else if (add) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, false, true, false>), grid, block, 0, s, d);
  else if (pre) hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, false, false, true>), grid, block, 0, s, d);
  else hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, BK, WM, WN, false, false, false>), grid, block, 0, s, d);
  return hipGetLastError();
}

template <int BK>
hipError_t launch_f32_bk(const ConvDesc& d, int bm, int bn, hipStream_t s) {
  if (bn == 32) return bm == 64 ? launch_f32<64, 32, BK, 2, 1>(d, s) : launch_f32<256, 32, BK, 8, 1>(d, s);
  if (bn == 64) return launch_f32<256, 64, BK, 4, 2>(d, s);
  if (bm == 64) return launch_f32<64, 128, BK, 1, 4>(d, s);
  if (bm == 256) return launch_f32<256, 128, BK, 4, 2>(d, s);
  if (bn == 256) return launch_f32<128, 256, BK, 2, 4>(d, s);
  return launch_f32<128, 128, BK, 2, 4>(d, s);
}

}  // namespace

// Build split: the launch paths (their kernel instantiations are most of this file's compile
// time, the fp16x3 ones doubled by the scaled-split instances) are compiled from this file as
// four more objects, -DSPK_CG_PART=0..3 (Makefile), in parallel; the part-less object holds the
// dispatch below and calls them.
hipError_t conv_launch_part0(const ConvDesc& d, hipStream_t s, int bm, int bn);   // f16: 128x128
hipError_t conv_launch_part1(const ConvDesc& d, hipStream_t s, int bm, int bn);   // f16: 256x128, 128x256
hipError_t conv_launch_part2(const ConvDesc& d, hipStream_t s, int bm, int bn);   // f16: 256x32, 64x32, 256x64, 64x128
hipError_t conv_launch_part3(const ConvDesc& d, hipStream_t s, int bm, int bn, int bk);   // exact fp32, all tiles

#if defined(SPK_CG_PART) && SPK_CG_PART == 0
hipError_t conv_launch_part0(const ConvDesc& d, hipStream_t s, int, int) { return launch_f16<128, 128, 2, 4>(d, s); }
#elif defined(SPK_CG_PART) && SPK_CG_PART == 1
hipError_t conv_launch_part1(const ConvDesc& d, hipStream_t s, int bm, int) {
  return bm == 256 ? launch_f16<256, 128, 4, 2>(d, s) : launch_f16<128, 256, 2, 4>(d, s);
}
#elif defined(SPK_CG_PART) && SPK_CG_PART == 2
hipError_t conv_launch_part2(const ConvDesc& d, hipStream_t s, int bm, int bn) {
  if (bn == 32) return bm == 64 ? launch_f16<64, 32, 2, 1>(d, s) : launch_f16<256, 32, 8, 1>(d, s);
  if (bn == 64) return launch_f16<256, 64, 4, 2>(d, s);
  return launch_f16<64, 128, 1, 4>(d, s);
}
#elif defined(SPK_CG_PART) && SPK_CG_PART == 3
hipError_t conv_launch_part3(const ConvDesc& d, hipStream_t s, int bm, int bn, int bk) {
  return bk == 32 ? launch_f32_bk<32>(d, bm, bn, s) : launch_f32_bk<16>(d, bm, bn, s);
}
#endif

#ifndef SPK_CG_PART
namespace {
hipError_t launch_tile(const ConvDesc& d, const Cfg& c, hipStream_t s) {
  const bool s1 = d.s1.p != nullptr, add = d.s0.p2 != nullptr, pre = d.s0.pre_scale != nullptr;
  if ((int)s1 + (int)add + (int)pre > 1) return hipErrorInvalidValue;
  const bool f16 = (d.x1 && d.wh && conv_buf_loader_ok(d, c.bm)) || (use_x3() && d.wh && d.wl && !d.wbig);
  hipError_t e;
  if (!f16) e = conv_launch_part3(d, s, c.bm, c.bn, c.bk);
  else if (c.bn == 32 || c.bn == 64 || c.bm == 64) e = conv_launch_part2(d, s, c.bm, c.bn);
  else if (c.bm == 256 || c.bn == 256) e = conv_launch_part1(d, s, c.bm, c.bn);
  else e = conv_launch_part0(d, s, c.bm, c.bn);
  if (e != hipSuccess || d.ksplit <= 1) return e;
  return launch_splitk_reduce(d, s);
}
}  // namespace

// Name of the kernel instantiation launch_conv() picks (matches rocprofv3 kernel names).
std::string conv_kernel_name(const ConvDesc& d) {
  if (halo_conv_supported(d)) return halo_kernel_name(d);
  if (use_x3() && pw_supported(d)) return pw_kernel_name(d);
  if (use_x3() && gemm_f_supported(d)) return gemm_f_kernel_name(d);
  const Cfg c = select_cfg(d);
  const bool s1 = d.s1.p != nullptr || d.s1.cin > 0, add = d.s0.p2 != nullptr || d.s0.ld2 > 0;
  const bool pre = d.s0.pre_scale != nullptr;
  const std::string tail = std::to_string(c.wm) + ", " + std::to_string(c.wn) + ", " + (s1 ? "true" : "false") + ", " +
                           (add ? "true" : "false") + ", " + (pre ? "true" : "false") + ">";
  if (d.x1 && d.wh && conv_buf_loader_ok(d, c.bm))
    return "conv_gemm_x1_kernel<" + std::to_string(c.bm) + ", " + std::to_string(c.bn) + ", " + tail;
  if (use_x3() && d.wh && d.wl && !d.wbig)
    return "conv_gemm_x3_kernel<" + std::to_string(c.bm) + ", " + std::to_string(c.bn) + ", " +
           tail.substr(0, tail.size() - 1) + (conv_buf_loader_ok(d, c.bm) ? ", true>" : ", false>");
  return "conv_gemm_kernel<" + std::to_string(c.bm) + ", " + std::to_string(c.bn) + ", " + std::to_string(c.bk) + ", " +
         tail;
}

int conv_tile_blocks(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  const Cfg c = select_cfg(d);
  return ((M + c.bm - 1) / c.bm) * ((d.N + c.bn - 1) / c.bn);
}

bool conv_use_x3() { return use_x3(); }

hipError_t launch_conv(const ConvDesc& dd, hipStream_t s) {
  ConvDesc d = dd;
  d.run_if = launch_gate();
  // host-side shape checks: every float4 access must stay aligned and in range
  if (d.s0.cin % 4 || d.s0.ld % 4 || (d.s0.p2 && d.s0.ld2 % 4) || d.Kp % KP_ALIGN || (d.osplit ? (d.osplit % 4 || d.ldo < d.osplit) : d.ldo < d.N) ||
      (d.s1.p && (d.s1.cin % 4 || d.s1.ld % 4)) || d.N <= 0 || d.nimg <= 0 || d.Ho <= 0 || d.Wo <= 0 ||
      (reinterpret_cast<uintptr_t>(d.s0.p) & 15) || (reinterpret_cast<uintptr_t>(d.w) & 15) ||
      d.K > d.Kp || (d.ksplit > 1 && !d.partial))
    return hipErrorInvalidValue;
  if (halo_conv_supported(d)) return launch_conv3x3_halo(d, s);
  if (use_x3() && pw_supported(d)) return launch_pw(d, s);
  if (use_x3() && gemm_f_supported(d)) return launch_gemm_f(d, s);
  return launch_tile(d, select_cfg(d), s);
}
#endif  // !SPK_CG_PART

}  // namespace spk
