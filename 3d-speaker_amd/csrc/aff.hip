// Fused AFF (fusion.py:8-28) on fp16x3 MFMA, gfx950:
//   h   = SiLU(BN(W1 · cat(x, y) + b1))          (local_att.0-2, K = 2C, N = C/4)
//   z   = BN(W2 · h + b2)                        (local_att.3-4, K = C/4, N = C)
//   out = x · (1 + tanh z) + y · (1 − tanh z)
// The two-conv form moves x and y through HBM twice and the bottleneck h once each way;
// here one wave owns 32 pixels end to end and nothing but x, y (once) and out touch HBM.
//
// Both GEMMs are computed transposed (pixels along the MFMA columns), so that stage 1's
// accumulator layout (lane = pixel, registers = bottleneck channels) is exactly the B
// operand layout stage 2 needs: no LDS round trip between the stages.
//   stage 1: hT[j][m] = sum_k W1[j][k] · xy[m][k]   A = W1 (rows j), B = xy^T (columns m)
//   stage 2: zT[n][m] = sum_j W2[n][j] · hT[j][m]   A = W2 (rows n), B = hT
// 32x32x16 MFMA C layout: lane l holds column l&31, rows (r&3) + 8(r>>2) + 4(l>>5), r < 16.
// For stage 2's k-step (t, s) lane half h therefore supplies bottleneck channels
// 32t + 16s + 4h + {0..3} and 32t + 16s + 8 + 4h + {0..3}, and its W2 fragments are read in
// the same order.  Stage 1 uses the k permutation of the conv GEMM (lane half h owns
// k0 + 16h .. +15 of a 32-deep step, the two 16-deep MFMA steps take 8 each), so every lane
// reads 64 contiguous bytes of its pixel's [x | y] row per step.  The combine transposes z
// through a per-wave LDS slab, so its x / y loads and out stores are whole 128-B row
// segments (8 lanes per pixel row) instead of 32 rows per instruction.
// fp16x3 as in conv_gemm.hip: hi = fp16(v), lo = fp16((v − hi)·2^11), three products.
#include <algorithm>
#include <cstdlib>

#include "aff.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

namespace spk {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split8(const f32x4 a, const f32x4 b, f16x8& hi, f16x8& lo) {
  h16x4 ha, la, hb, lb;
  split_x3(a, ha, la);
  split_x3(b, hb, lb);
  hi = f16x8{ha[0], ha[1], ha[2], ha[3], hb[0], hb[1], hb[2], hb[3]};
  lo = f16x8{la[0], la[1], la[2], la[3], lb[0], lb[1], lb[2], lb[3]};
}

__device__ __forceinline__ f16x8 ld_h8(const uint16_t* p) { return *reinterpret_cast<const f16x8*>(p); }
__device__ __forceinline__ f16x4 ld_h4(const uint16_t* p) { return *reinterpret_cast<const f16x4*>(p); }

constexpr int SLAB_LD = 36;   // LDS row stride of the per-wave 32 x 32 transpose slab (floats)

template <int MT>   // bottleneck tiles of 32 channels
__global__ void __launch_bounds__(256) aff_x3_kernel(const AffDesc a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int m0 = (blockIdx.x * 4 + wave) * 32;
  if (m0 >= a.M) return;                            // wave-uniform; no block barriers below
  extern __shared__ float aff_lds[];                // >= 4 waves x 32 x SLAB_LD floats (launch)
  float* slab = aff_lds + wave * 32 * SLAB_LD;
  const int m = min(m0 + li, a.M - 1);             // this lane's pixel (stage-1 B column)
  const float* xr = a.x + (size_t)m * a.ldx;
  const float* yr = a.y + (size_t)m * a.ldy;
  const int K = 2 * a.cp;

  float amax = 0.f;                                 // range guard (common.h) on the outputs
  // ---- stage 1
  f32x16 h[MT], hx[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) { h[t][r] = 0.f; hx[t][r] = 0.f; }
  // [x | y] loads run one 32-deep step ahead of the MFMAs (clamped in-row addresses,
  // zeroed past K when used, so the prefetch is unconditional)
  auto load_xy = [&](int k0, f32x4 (&v)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {                   // 8 channels each, from x or y (cp % 8 == 0)
      const int k = min(k0 + 16 * lh + 8 * s, K - 8);
      const float* src = k < a.cp ? xr + k : yr + (k - a.cp);
      v[s][0] = *reinterpret_cast<const f32x4*>(src);
      v[s][1] = *reinterpret_cast<const f32x4*>(src + 4);
    }
  };
  f32x4 vn[2][2];
  load_xy(0, vn);
  for (int k0 = 0; k0 < K; k0 += 32) {
    f32x4 v[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool kin = k0 + 16 * lh + 8 * s < K;
      v[s][0] = kin ? vn[s][0] : f32x4{0.f, 0.f, 0.f, 0.f};
      v[s][1] = kin ? vn[s][1] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    load_xy(min(k0 + 32, K - 8), vn);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int k = k0 + 16 * lh + 8 * s;
      f16x8 bh, bl;
      split8(v[s][0], v[s][1], bh, bl);
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        f16x8 ah = {}, al = {};
        if (k < K) {                                // k + 7 < K <= kp1: inside the packed row
          const size_t wo = (size_t)(t * 32 + li) * a.kp1 + k;
          ah = ld_h8(a.w1h + wo);
          al = ld_h8(a.w1l + wo);
        }
        h[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh, h[t], 0, 0, 0);
        hx[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl, hx[t], 0, 0, 0);
        hx[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh, hx[t], 0, 0, 0);
      }
    }
  }

  // ---- bias + SiLU, split: stage 2's B fragments straight from the accumulators
  f16x8 gh[MT][2], gl[MT][2];
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      float v = h[t][r] + hx[t][r] * (1.0f / 2048.0f) + a.b1[j];
      v = v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));   // SiLU (hardware reciprocal)
      const _Float16 vh = (_Float16)v;
      gh[t][r >> 3][r & 7] = vh;
      gl[t][r >> 3][r & 7] = (_Float16)((v - (float)vh) * 2048.0f);
    }

  // ---- stage 2 + AFF combine, 32 output channels at a time.  A chunk's operands -- the
  // x / y row segments of the combine and the W2 fragments -- are requested one chunk ahead
  // (clamped, unconditional: the last chunk re-reads itself), so each chunk's waits are
  // counts that leave the next chunk's loads in flight
  const int c4 = (lane & 7) * 4;
  const int nch = (a.cp + 31) / 32;                 // <= 7 (cp <= 208)
  struct Chunk {
    f32x4 xv[4], yv[4];
    f16x8 wh[MT][2], wl[MT][2];
    f32x4 b2;
  };
  auto load_chunk = [&](int c, Chunk& ck) {
    const int n0 = 32 * c;
    const int n = min(n0 + li, a.cp - 1);           // W2 row of this lane (A operand)
    const int cc = min(n0 + c4, a.cp - 4);
    ck.b2 = *reinterpret_cast<const f32x4*>(a.b2 + cc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mq = min(m0 + q * 8 + (lane >> 3), a.M - 1);
      ck.xv[q] = *reinterpret_cast<const f32x4*>(a.x + (size_t)mq * a.ldx + cc);
      ck.yv[q] = *reinterpret_cast<const f32x4*>(a.y + (size_t)mq * a.ldy + cc);
    }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const size_t wo = (size_t)n * a.kp2 + t * 32 + 16 * s + 4 * lh;
        const f16x4 h0 = ld_h4(a.w2h + wo), h1 = ld_h4(a.w2h + wo + 8);
        const f16x4 l0 = ld_h4(a.w2l + wo), l1 = ld_h4(a.w2l + wo + 8);
        ck.wh[t][s] = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
        ck.wl[t][s] = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
      }
  };
  auto chunk = [&](int c, const Chunk& ck) {
    const int n0 = 32 * c;
    const bool nok = n0 + li < a.cp;
    f32x16 z, zx;
#pragma unroll
    for (int r = 0; r < 16; ++r) { z[r] = 0.f; zx[r] = 0.f; }
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const f16x8 ah = nok ? ck.wh[t][s] : f16x8{}, al = nok ? ck.wl[t][s] : f16x8{};
        z = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gh[t][s], z, 0, 0, 0);
        zx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, gl[t][s], zx, 0, 0, 0);
        zx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, gh[t][s], zx, 0, 0, 0);
      }
    // transpose through the wave's LDS slab: MFMA C layout (lane = pixel) -> rows
#pragma unroll
    for (int r = 0; r < 16; ++r)
      slab[li * SLAB_LD + (r & 3) + 8 * (r >> 2) + 4 * lh] = z[r] + zx[r] * (1.0f / 2048.0f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const f32x4 bias = ck.b2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = q * 8 + (lane >> 3);
      const f32x4 zq = *reinterpret_cast<const f32x4*>(slab + p * SLAB_LD + c4);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // x(1 + tanh z) + y(1 - tanh z) = 2(y + s(x - y)), s = sigmoid(2z): one exp + rcp
        const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * (zq[e] + bias[e])));
        o[e] = 2.0f * fmaf(sg, ck.xv[q][e] - ck.yv[q][e], ck.yv[q][e]);
      }
      if (m0 + p < a.M && n0 + c4 < a.cp) {
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
        *reinterpret_cast<f32x4*>(a.out + (size_t)(m0 + p) * a.ldo + n0 + c4) = o;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // slab reads done before the next chunk
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  if constexpr (MT == 1) {
    Chunk ring[2];
    load_chunk(0, ring[0]);
#pragma unroll
    for (int c = 0; c < 7; ++c) {                   // unrolled: the set index is a constant
      if (c >= nch) break;
      load_chunk(min(c + 1, nch - 1), ring[(c + 1) & 1]);
      chunk(c, ring[c & 1]);
    }
  } else {                                          // two bottleneck tiles: no room for a
    Chunk ck;                                       // second set at two waves per SIMD
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      load_chunk(c, ck);
      chunk(c, ck);
    }
  }
  range_note(a.range_flag, amax);
}

// ---------------------------------------------------------------------------------------
// Persistent form for a 32-channel bottleneck and cp <= 128 (ERes2NetV2 / ERes2Net layer-3
// fusions), round 6.  The kernel above is latency-bound (2.2 TB/s, MFMA busy 0.05): each of
// its stage-1 k-steps waits for that step's [x | y] loads (one step ahead) and W1 fragment
// loads, and the combine re-reads x / y from L2.  Here
//   * W1 and W2 live in LDS (loaded once per block, fp16 hi / lo planes, rows padded to 40
//     halves: conflict-free ds_read_b128), so no global load sits inside the MFMA chains;
//   * a wave owns 16 pixels at a time on v_mfma_f32_16x16x32_f16 (transposed GEMMs, pixels
//     along the MFMA columns) and walks tiles with a stride of the grid; 16 waves per CU
//     (two 8-wave blocks) keep 16 tiles' x / y in flight;
//   * the K order of stage 1 is permuted so that lane (pixel l & 15, group g = l >> 4) loads,
//     for each 32-channel group c of x and of y, channels 32c + 4g .. +3 and 32c + 16 + 4g .. +3
//     -- exactly the channels stage 2's accumulators give that lane (n = 16 nb + 4g + e), so the
//     combine takes x and y from the same registers: HBM traffic is x, y and out once each;
//   * stage 1's accumulators (lane: pixel, j = 16 jb + 4g + e) are stage 2's B operand under
//     the matching permutation of W2's columns (k slot 8g + e <-> j = 4g + e, 16 + 4g + e - 4).
// fp16x3 products and the two-accumulator order as aff_x3_kernel.
constexpr int AP_ROW = 48;   // halves per LDS weight row (96 B: the 16x16x32 fragment reads of one ds_read_b128
                             // lane group land on distinct banks, conv_gemm_f.hip FCfg::LROW)

// CX 32-channel groups of x (and of y), the last one with LH valid 16-channel halves:
// cp <= 32 (CX - 1) + 16 LH (ERes2NetV2 layer 3: cp = 104, CX = 4, LH = 1)
template <int CX, int LH>
__global__ void __launch_bounds__(512, 4) aff_x3p_kernel(const AffDesc a) {   // 4 waves per SIMD
  constexpr int KS1 = 2 * CX;                       // stage-1 k-steps (x groups, then y groups)
  constexpr int NB = 2 * (CX - 1) + LH;             // stage-2 16-channel output blocks
  extern __shared__ float aff_lds[];
  _Float16* const w1h = reinterpret_cast<_Float16*>(aff_lds);          // [KS1][32][AP_ROW]
  _Float16* const w1l = w1h + KS1 * 32 * AP_ROW;
  _Float16* const w2h = w1l + KS1 * 32 * AP_ROW;                      // [16 NB][AP_ROW]
  _Float16* const w2l = w2h + NB * 16 * AP_ROW;
  float* const b2s = reinterpret_cast<float*>(w2l + NB * 16 * AP_ROW);        // [16 NB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int cp = a.cp;

  // ---- weights -> LDS in the permuted K orders (zeros past cp / nmid).  Slot kk = 8 gg + e of
  // a 32-deep step holds channel 4 gg + e (e < 4) or 16 + 4 gg + e - 4: two 4-half runs, each
  // one 8-byte load; every load of the staging is issued before the first LDS store (a
  // load-store loop paid one L2 round trip per element at kernel start: ~30 us per launch)
  typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
  {
    constexpr int N1 = KS1 * 32 * 8;                // W1 runs: (step c, row j, run r = 2 gg + half)
    constexpr int N2 = NB * 16 * 8;                 // W2 runs: (row n, run)
    constexpr int R1 = (N1 + 511) / 512, R2 = (N2 + 511) / 512;
    u16x4 h1[R1], l1[R1], h2[R2], l2[R2];
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int i = tid + 512 * r;
      const int run = i & 7, j = (i >> 3) & 31, c = min(i >> 8, KS1 - 1);
      const int ch = 32 * (c % CX) + (run & 1) * 16 + 4 * (run >> 1);
      const bool ok = i < N1 && ch < cp;
      const size_t o = (size_t)j * a.kp1 + (c < CX ? 0 : cp) + (ok ? ch : 0);
      h1[r] = *reinterpret_cast<const u16x4*>(a.w1h + o);
      l1[r] = *reinterpret_cast<const u16x4*>(a.w1l + o);
      if (!ok) h1[r] = l1[r] = u16x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      const int i = tid + 512 * r;
      const int run = i & 7, n = min(i >> 3, NB * 16 - 1);
      const int jj = (run & 1) * 16 + 4 * (run >> 1);
      const bool ok = i < N2 && n < cp;
      const size_t o = (size_t)(ok ? n : 0) * a.kp2 + jj;
      h2[r] = *reinterpret_cast<const u16x4*>(a.w2h + o);
      l2[r] = *reinterpret_cast<const u16x4*>(a.w2l + o);
      if (!ok) h2[r] = l2[r] = u16x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int r = 0; r < R1; ++r) {
      const int i = tid + 512 * r;
      if (i >= N1) continue;
      const int run = i & 7, j = (i >> 3) & 31, c = i >> 8;
      const int kk = 8 * (run >> 1) + 4 * (run & 1);
      *reinterpret_cast<u16x4*>(w1h + (c * 32 + j) * AP_ROW + kk) = h1[r];
      *reinterpret_cast<u16x4*>(w1l + (c * 32 + j) * AP_ROW + kk) = l1[r];
    }
#pragma unroll
    for (int r = 0; r < R2; ++r) {
      const int i = tid + 512 * r;
      if (i >= N2) continue;
      const int run = i & 7, n = i >> 3;
      const int kk = 8 * (run >> 1) + 4 * (run & 1);
      *reinterpret_cast<u16x4*>(w2h + n * AP_ROW + kk) = h2[r];
      *reinterpret_cast<u16x4*>(w2l + n * AP_ROW + kk) = l2[r];
    }
  }
  for (int i = tid; i < NB * 16; i += 512) b2s[i] = i < cp ? a.b2[i] : 0.f;
  // stage-1 bias of this lane's bottleneck channels j = 4g + e and 16 + 4g + e
  const f32x4 b1a = *reinterpret_cast<const f32x4*>(a.b1 + 4 * g);
  const f32x4 b1b = *reinterpret_cast<const f32x4*>(a.b1 + 16 + 4 * g);
  __syncthreads();

  const int ntiles = (a.M + 15) / 16;
  const int wstride = gridDim.x * 8;
  const int t0 = blockIdx.x * 8 + wave;
  // x / y quads of a tile: [c][h] = channels 32c + 16h + 4g .. +3 of pixel 16 t + l16 (clamped
  // row, clamped in-row column: every load unconditional; channels past cp meet zero weights
  // and are never stored)
  struct XY {
    f32x4 x[CX][2], y[CX][2];
  };
  auto load = [&](int t, XY& v) {
    const int m = min(16 * t + l16, a.M - 1);
    const float* xr = a.x + (size_t)m * a.ldx;
    const float* yr = a.y + (size_t)m * a.ldy;
#pragma unroll
    for (int c = 0; c < CX; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (c == CX - 1 && h >= LH) {               // past cp for every lane: not loaded
          v.x[c][h] = v.y[c][h] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        const int ch = min(32 * c + 16 * h + 4 * g, cp - 4);
        v.x[c][h] = *reinterpret_cast<const f32x4*>(xr + ch);
        v.y[c][h] = *reinterpret_cast<const f32x4*>(yr + ch);
      }
  };
  float amax = 0.f;
  auto tile = [&](int t, const XY& v) {
    // stage 1: hT[j][m] over K = [x | y] (permuted), two 16-row j blocks
    f32x4 h[2], hx[2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) { h[jb] = f32x4{0.f, 0.f, 0.f, 0.f}; hx[jb] = h[jb]; }
#pragma unroll
    for (int c = 0; c < KS1; ++c) {
      const int cc = c % CX;
      const bool isx = c < CX;
      f32x4 q0 = isx ? v.x[cc][0] : v.y[cc][0], q1 = isx ? v.x[cc][1] : v.y[cc][1];
      // channels past cp: zero (their W1 columns are zero too, but the clamped load may hold
      // finite garbage from the row's tail -- keep the products exactly zero)
      if (32 * cc + 4 * g >= cp) q0 = f32x4{0.f, 0.f, 0.f, 0.f};
      if (32 * cc + 16 + 4 * g >= cp) q1 = f32x4{0.f, 0.f, 0.f, 0.f};
      h16x4 h0, l0, h1, l1;
      split_x3(q0, h0, l0);
      split_x3(q1, h1, l1);
      const f16x8 bh = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
      const f16x8 bl = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const int o = (c * 32 + 16 * jb + l16) * AP_ROW + 8 * g;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(w1h + o);
        const f16x8 al = *reinterpret_cast<const f16x8*>(w1l + o);
        h[jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, h[jb], 0, 0, 0);
        hx[jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, hx[jb], 0, 0, 0);
        hx[jb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, hx[jb], 0, 0, 0);
      }
    }
    // bias + SiLU, split: stage 2's B operand (k slot 8g + e: j = 4g + e, then 16 + 4g + e)
    f16x8 gh, gl;
#pragma unroll
    for (int jb = 0; jb < 2; ++jb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float z = h[jb][e] + hx[jb][e] * (1.0f / 2048.0f) + (jb ? b1b[e] : b1a[e]);
        z = z * __builtin_amdgcn_rcpf(1.0f + __expf(-z));   // SiLU (hardware reciprocal)
        const _Float16 zh = (_Float16)z;
        gh[4 * jb + e] = zh;
        gl[4 * jb + e] = (_Float16)((z - (float)zh) * 2048.0f);
      }
    // stage 2 + combine, one 16-channel output block at a time
    const int m = 16 * t + l16;
    // stores through a resource based at the tile's first row: a lane past M or cp gets an
    // offset the buffer unit drops, so no store (and no load) sits behind a branch
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.out + (size_t)16 * t * a.ldo);
    const uint32_t orow = m < a.M ? (uint32_t)l16 * (uint32_t)a.ldo * 4u : BUF_OOB;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int o = (nb * 16 + l16) * AP_ROW + 8 * g;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(w2h + o);
      const f16x8 al = *reinterpret_cast<const f16x8*>(w2l + o);
      f32x4 z = {0.f, 0.f, 0.f, 0.f}, zx = z;
      z = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gh, z, 0, 0, 0);
      zx = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, gl, zx, 0, 0, 0);
      zx = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, gh, zx, 0, 0, 0);
      const int n = 16 * nb + 4 * g;                  // this lane's four output channels
      const f32x4 xv = v.x[nb >> 1][nb & 1], yv = v.y[nb >> 1][nb & 1];
      const f32x4 b2 = *reinterpret_cast<const f32x4*>(b2s + n);
      f32x4 out;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // x(1 + tanh z) + y(1 - tanh z) = 2(y + s(x - y)), s = sigmoid(2z): one exp + rcp
        const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * (z[e] + zx[e] * (1.0f / 2048.0f) + b2[e])));
        out[e] = 2.0f * fmaf(sg, xv[e] - yv[e], yv[e]);
      }
      const bool ok = n < cp && orow != BUF_OOB;
      if (ok) amax = fmaxf(amax, fmaxf(fmaxf(fabsf(out[0]), fabsf(out[1])), fmaxf(fabsf(out[2]), fabsf(out[3]))));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, out), ro, ok ? (int)(orow + 4u * n) : (int)BUF_OOB, 0, 0);
    }
  };
  // persistent walk; one register set per wave (a second one, for a prefetch of the next
  // tile, spills at CX = 4): the memory parallelism comes from 16 waves per CU instead
  for (int t = t0; t < ntiles; t += wstride) {
    XY v;
    load(t, v);
    // all of the tile's loads issued before any use (left to itself the scheduler sank them
    // next to their uses, one vmcnt(0) round trip per load)
    __builtin_amdgcn_sched_barrier(0);
    tile(t, v);
  }
  range_note(a.range_flag, amax);
}

}  // namespace

bool aff_x3_supported(int cp, int nmid) {
  static const bool off = [] {   // SPK_NO_AFF_FUSED=1: the two-conv form (experiments)
    const char* e = std::getenv("SPK_NO_AFF_FUSED");
    return e && std::atoi(e) != 0;
  }();
  // cp <= 208: past that (ERes2Net-large fuse_mode12, 256 channels at 40 x T/2) the rows of
  // the pixels in flight no longer stay in L2 and the two-conv form is faster (measured)
  return !off && conv_use_x3() && (nmid == 32 || nmid == 64) && cp % 8 == 0 && cp >= 8 && cp <= 208;
}

// the persistent form (aff_x3p_kernel): a 32-channel bottleneck, cp <= 128;
// SPK_AFF_P=0 keeps aff_x3_kernel (A/B runs)
bool aff_p_ok(int cp, int nmid) {
  static const bool off = [] {
    const char* e = std::getenv("SPK_AFF_P");
    return e && std::atoi(e) == 0;
  }();
  return !off && nmid == 32 && cp <= 128 && cp % 8 == 0;
}

std::string aff_x3_kernel_name(int cp, int nmid) {
  if (aff_p_ok(cp, nmid)) {
    const int cx = (cp + 31) / 32;
    return "aff_x3p_kernel<" + std::to_string(cx) + ", " + (cp - 32 * (cx - 1) <= 16 ? "1" : "2") + ">";
  }
  return "aff_x3_kernel<" + std::to_string(nmid / 32) + ">";
}

hipError_t launch_aff_x3(const AffDesc& a, hipStream_t s) {
  // host-side shape checks: every vector access stays aligned and inside its row
  if (!aff_x3_supported(a.cp, a.nmid) || a.M <= 0 || !a.w1h || !a.w1l || !a.w2h || !a.w2l || !a.b1 || !a.b2 ||
      a.kp1 < 2 * a.cp || a.kp1 % 8 || a.kp2 < a.nmid || a.kp2 % 4 || a.ldx % 4 || a.ldy % 4 || a.ldo % 4 ||
      a.ldx < a.cp || a.ldy < a.cp || a.ldo < a.cp ||
      (reinterpret_cast<uintptr_t>(a.x) & 15) || (reinterpret_cast<uintptr_t>(a.y) & 15) ||
      (reinterpret_cast<uintptr_t>(a.out) & 15) || (reinterpret_cast<uintptr_t>(a.w1h) & 15) ||
      (reinterpret_cast<uintptr_t>(a.w1l) & 15))
    return hipErrorInvalidValue;
  const dim3 grid((a.M + 127) / 128), block(256);
  // The combine re-reads the x / y rows stage 1 streamed; with every block slot filled the
  // rows of the pixels in flight overflow the XCD's 4 MB L2 before they are re-read.  A
  // 60 KB LDS reservation caps residency at 2 blocks (8 waves) per CU, which keeps them in
  // L2 (measured: layer3 fusions 1.08 -> 0.97 ms per ERes2NetV2 forward; 1 block per CU
  // is slower again).  SPK_AFF_LDS_KB overrides it for experiments.
  static const size_t lds_pad = [] {
    const char* e = std::getenv("SPK_AFF_LDS_KB");
    return std::max((size_t)(e ? std::atoi(e) : 60) * 1024, (size_t)4 * 32 * SLAB_LD * sizeof(float));
  }();
  if (aff_p_ok(a.cp, a.nmid)) {
    const int cx = (a.cp + 31) / 32;
    const size_t lds = ((size_t)2 * cx * 32 * AP_ROW * 2 + (size_t)2 * cx * 16 * AP_ROW * 2) * sizeof(_Float16) +
                       (size_t)2 * cx * 16 * sizeof(float);
    const int ntiles = (a.M + 15) / 16;
    const int blocks = std::max(1, std::min((ntiles + 7) / 8, 2 * device_cus()));
    const int lh = a.cp - 32 * (cx - 1) <= 16 ? 1 : 2;
#define SPK_AFFP(CX, LH) if (cx == CX && lh == LH) hipLaunchKernelGGL((aff_x3p_kernel<CX, LH>), dim3(blocks), dim3(512), lds, s, a)
    SPK_AFFP(1, 1); SPK_AFFP(1, 2); SPK_AFFP(2, 1); SPK_AFFP(2, 2);
    SPK_AFFP(3, 1); SPK_AFFP(3, 2); SPK_AFFP(4, 1); SPK_AFFP(4, 2);
#undef SPK_AFFP
    return hipGetLastError();
  }
  if (a.nmid == 32) hipLaunchKernelGGL(aff_x3_kernel<1>, grid, block, lds_pad, s, a);
  else hipLaunchKernelGGL(aff_x3_kernel<2>, grid, block, lds_pad, s, a);
  return hipGetLastError();
}

}  // namespace spk
