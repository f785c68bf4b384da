// Implicit-GEMM convolution on fp16x3 MFMA with an LDS-DMA ring for BOTH operands (gfx950).
//
// Replaces the register-staged tiled GEMM (conv_gemm.hip) on the plain large layers: there,
// every K-tile goes global -> VGPR -> split -> ds_write, and ablation builds put 32 % of the
// kernel's time in those in-loop LDS stores and the waits they carry.  Here:
//   * 256 x 128 block tile, 8 waves (2 per SIMD): wave w owns output pixels 32w .. 32w+31
//     and all 128 output channels, so every activation element is split into its fp16 hi / lo
//     halves exactly once, by the one wave that uses it;
//   * the MFMA is transposed (srcA = weights, srcB = activations, D[channel][pixel]): a lane
//     ends with 4 consecutive channels of one pixel per register quad, so the fused epilogue
//     reads its operands and stores the outputs as float4 straight from the accumulators --
//     no LDS round trip, no LDS reserved for it;
//   * K-tile of 32, three LDS stages of 48 KB, each filled by `buffer_load_dwordx4 ... lds`
//     (no VGPR destination, no ds_write): A = fp32 activations [256 pixels][128 B] (one
//     8-pixel x 128-B block of full lines per wave-instruction), B = the packed fp16 hi / lo
//     weight planes [plane][128 channels][64 B].  The DMA destination is lane-linear, so the
//     XOR swizzles that make the fragment reads bank-conflict free go on the SOURCE address:
//     A chunk c of pixel row r sits in slot c ^ ((r >> 1) & 7), B chunk c of channel n in slot
//     c ^ ((n >> 2) & 3) (cdna_hip_programming.md §5, rule 21);
//   * one raw s_barrier per K-tile with a counted vmcnt: the DMA of K-tile kt+2 is issued
//     right after the barrier of kt (which is also the WAR barrier of the stage it refills),
//     one K-tile of DMA stays in flight across it; no ordinary global load in the loop (a
//     VGPR-destination load next to LDS-DMA makes hipcc drain vmcnt(0) at its use);
//   * out-of-image taps, pixels past M and channels past N read offset BUF_OOB: the buffer
//     unit returns zeros and the DMA writes them.
// Numerics are those of conv_gemm.hip's fp16x3 kernels, with two accumulators (hi x hi, and
// the cross terms at 2^11):  x * w ~= hi_x hi_w + 2^-11 (hi_x lo_w + lo_x hi_w), products exact,
// fp32 sums.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "common.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

#ifndef SPK_REXP
#define SPK_REXP 0   // ablation builds only (tools/ring_exp.sh): 1 no MFMA, 2 no in-loop DMA,
                     // 3 no epilogue stores, 4 no split, 5 = 1 + 2 + 3, 6 empty kernel of the
                     // same resources; 0 = the product kernel
#endif

namespace spk {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int RBM = 256, RBN = 128, RBK = 32, RNW = 8, RNT = 64 * RNW, RNS = 3;
constexpr int RA_STAGE = RBM * RBK * 4;            // bytes: fp32 [256 pixels][128 B]
constexpr int RB_PLANE = RBN * RBK * 2;            // bytes: fp16 [128 channels][64 B]
constexpr int RB_STAGE = 2 * RB_PLANE;             // hi, lo
constexpr int RSTAGE = RA_STAGE + RB_STAGE;        // 48 KB
constexpr int RDMA = RBM / (8 * RNW) + RB_STAGE / (1024 * RNW);   // DMA instructions per wave per K-tile (4 + 2)

__device__ __forceinline__ int aswz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int bswz(int n) { return (n >> 2) & 3; }

// fp16x3 split of 8 fp32 values: hi = fp16(v) (round toward zero, packed), lo = fp16((v - hi) 2^11).
// lo is formed by v_fma_mixlo / v_fma_mixhi_f16 from the packed fp16 hi and 2^11 v (exact):
// one rounding, 2.5 VALU per value.  Inline asm because hipcc's SLP vectoriser otherwise turns
// the remainder into unpack + v_pk_fma_f32 + repack (3 per value, packed fp32 beside MFMAs).
__device__ __forceinline__ uint32_t split_lo2(uint32_t hp, float v0, float v1) {
  uint32_t r;
  const float m = -2048.0f;
  asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, %2, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(hp), "s"(m), "v"(v0 * 2048.0f), "v"(v1 * 2048.0f));
  return r;
}

__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, f16x8& h, f16x8& l) {
  typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
  u32x4v hv, lv;
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    hv[i] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v[2 * i], v[2 * i + 1]));
    lv[i] = split_lo2(hv[i], v[2 * i], v[2 * i + 1]);
  }
  h = __builtin_bit_cast(f16x8, hv);
  l = __builtin_bit_cast(f16x8, lv);
}

__global__ void __launch_bounds__(RNT, 2)
conv_gemm_ring_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
  __shared__ __attribute__((aligned(16))) float lds[RNS * RSTAGE / 4];   // the only LDS object
  char* const lb = reinterpret_cast<char*>(lds);
#if SPK_REXP == 6
  if (d.N > 0) {   // launch-cost probe: same resources, no work
    if (threadIdx.x == 1000) lds[0] = 0.f;
    return;
  }
#endif

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + RBN - 1) / RBN;
  const int nM = (M + RBM - 1) / RBM;
  const int ntile = nM * nN;
  const int nkt = d.Kp / RBK;

  // ---- tiles of this block.  One tile per block when the grid covers them (XCD remap: the N
  // tiles of one M tile on one XCD, their A in its L2); otherwise persistent: the tiles are
  // split into 8 contiguous ranges, one per XCD (blocks b and b + 8 share an XCD), and the
  // XCD's blocks take its range round-robin, so the blocks running together on an XCD work
  // on neighbouring tiles (same M tile, consecutive N tiles) and sweep M together.
  const int G = gridDim.x;
  int tbase, tstep, ntb;
  if (G >= ntile) {
    tbase = xcd_remap(blockIdx.x, ntile);
    tstep = 1;
    ntb = blockIdx.x < ntile ? 1 : 0;
  } else {
    const int x = blockIdx.x & 7, j = blockIdx.x >> 3, nper = G >> 3;   // G % 8 == 0 (host)
    const int q = ntile >> 3, r = ntile & 7;
    const int cnt = q + (x < r ? 1 : 0);
    tbase = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + j;
    tstep = nper;
    ntb = j < cnt ? (cnt - j + nper - 1) / nper : 0;
  }
  if (ntb == 0) return;
  const int total = ntb * nkt;

  // ---- A DMA: instruction j of wave w fills pixel rows 64 j + 8 w .. +7 (8 rows x 128 B);
  // lane p -> row 64 j + 8 w + (p >> 3), LDS slot p & 7, i.e. source k-quad
  // (p & 7) ^ aswz(row) = (p & 7) ^ ((4 w + (p >> 4)) & 7): the same quad for all four rows
  const int aq = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
  using AL = BufALoader<4, 64, RBK, false, false, false>;
  AL al;
  const int a_dst = (8 * wave) * 128;          // + 64 rows (8 KB) per instruction j
  // ---- B DMA: instruction i = 2 w + j (j = 0, 1) fills plane i >> 3 (hi / lo), channels
  // 16 (i & 7) .. +15; lane p -> channel 16 (i & 7) + (p >> 2), slot p & 3, source chunk
  // (p & 3) ^ bswz(channel) = (p & 3) ^ ((p >> 4) & 3).  Channels past N read zeros.
  const int plane = wave >> 2;
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(plane ? d.wl : d.wh);
  const int cq = (lane & 3) ^ ((lane >> 4) & 3);
  uint32_t boff[2];
  const int b_dst = RA_STAGE + plane * RB_PLANE + ((2 * wave) & 7) * 1024;   // + 1 KB per j

  // issue cursor (tile ii of this block, K-tile ik): runs two K-tiles ahead of the compute
  // cursor, across tile boundaries, so a tile's first K-tiles land during the previous
  // tile's last K-tiles and epilogue
  int ii = 0, ik = 0;
  auto set_issue_tile = [&](int i) {
    const int lid = tbase + i * tstep;
    const int m0 = (lid / nN) * RBM, n0 = (lid % nN) * RBN;
    al.init(d, m0, 8 * wave + (lane >> 3), aq, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 16 * ((2 * wave + j) & 7) + (lane >> 2);
      boff[j] = n < d.N ? ((uint32_t)n * d.Kp + cq * 8) * 2u : BUF_OOB;
    }
  };
  auto issue_next = [&](int stage) {
    uint32_t ao[4];
    al.offsets(d, ao);
    char* const sb = lb + stage * RSTAGE;
    const int koff = __builtin_amdgcn_readfirstlane(ik * RBK * 2);   // K-tile byte offset in a weight row
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(al.r0, (lds_ptr_t)(sb + a_dst + j * 8192), 16, (int)ao[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (lds_ptr_t)(sb + b_dst + j * 1024), 16, (int)boff[j], koff, 0, 0);
    if (++ik == nkt) {
      ik = 0;
      if (++ii < ntb) set_issue_tile(ii);
    }
  };

  // two accumulators per tile: hi_x hi_w, and the 2^11-scaled cross terms hi_x lo_w + lo_x hi_w
  // (no per-fragment rescaling of the weights in the loop, no weight-range restriction)
  f32x16 acc[4], accx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = accx[j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  const int arow = 32 * wave + li;
  const int af = aswz(arow);
  // fragment reads of substep s (k = 16 s .. 16 s + 15 of the K-tile; lane half lh holds
  // k = 16 s + 8 lh .. +7 for both operands): A = pixel arow, fp32 quads 4 s + 2 lh (+1);
  // B = channel 32 j + li, fp16 chunk 2 s + lh of each plane
  auto compute = [&](int stage) {
    const char* sb = lb + stage * RSTAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const char* ap = sb + arow * 128;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(ap + (((4 * s + 2 * lh) ^ af) << 4));
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(ap + (((4 * s + 2 * lh + 1) ^ af) << 4));
      f16x8 wh[4], wl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 32 * j + li;
        const char* bp = sb + RA_STAGE + n * 64 + (((2 * s + lh) ^ bswz(n)) << 4);
        wh[j] = *reinterpret_cast<const f16x8*>(bp);
        wl[j] = *reinterpret_cast<const f16x8*>(bp + RB_PLANE);
      }
      f16x8 xh, xl;
#if SPK_REXP == 4
      xh = __builtin_bit_cast(f16x8, a0);
      xl = __builtin_bit_cast(f16x8, a1);
#else
      split8(a0, a1, xh, xl);
#endif
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#if SPK_REXP == 1 || SPK_REXP >= 5
        acc[j][0] += (float)wh[j][0] * (float)xh[0] + (float)wl[j][1] * (float)xl[1];
        continue;
#endif
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[j], xh, acc[j], 0, 0, 0);
        accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wl[j], xh, accx[j], 0, 0, 0);
        accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wh[j], xl, accx[j], 0, 0, 0);
      }
    }
  };

  // ---- fused epilogue from the accumulators: lane (li, lh) holds pixel m of the wave, and in
  // register quad g of tile j the channels n = n0 + 32 j + 8 g + 4 lh .. +3 (MFMA D layout:
  // row = (r & 3) + 8 (r >> 2) + 4 lh, column = li)
  float amax = 0.f;
  auto epilogue = [&](int lid) {
    const int m0 = (lid / nN) * RBM, n0 = (lid % nN) * RBN;
    const int m = m0 + arow;
    const bool mok = m < M;
    const int mm = mok ? m : 0;
    const bool rowz = mok && row_masked(d, m);
    const int img = mm / (d.Ho * d.Wo), wo = mm % d.Wo;
    // one 32-channel tile at a time: its residual / AFF operand loads are all issued before use
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 ra[4], xa[4], ya[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + 32 * j + 8 * g + 4 * lh;
        const int nn = n < d.N ? n : 0;
        ra[g] = xa[g] = ya[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (d.res) ra[g] = *reinterpret_cast<const f32x4*>(d.res + (size_t)mm * d.ldr + nn);
        if (d.affx) {
          xa[g] = *reinterpret_cast<const f32x4*>(d.affx + (size_t)mm * d.ldx + nn);
          ya[g] = *reinterpret_cast<const f32x4*>(d.affy + (size_t)mm * d.ldy + nn);
        }
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + 32 * j + 8 * g + 4 * lh;
        if (!mok || n >= d.N) continue;
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = fmaf(accx[j][4 * g + e], 1.0f / 2048.0f, acc[j][4 * g + e]);
        if (d.bias) o += *reinterpret_cast<const f32x4*>(d.bias + n);
        if (d.rowbias) o += *reinterpret_cast<const f32x4*>(d.rowbias + (size_t)img * d.rowbias_ld + n);
        o += ra[g];
        if (d.affx) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float t = 1.0f + tanhf(o[e]);
            o[e] = xa[g][e] * t + ya[g][e] * (2.0f - t);
          }
        } else {
          f32x4 ps = {1.f, 1.f, 1.f, 1.f}, pt = {0.f, 0.f, 0.f, 0.f};
          if (d.post_scale) {
            ps = *reinterpret_cast<const f32x4*>(d.post_scale + n);
            pt = *reinterpret_cast<const f32x4*>(d.post_shift + n);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x = apply_act(o[e], d.act);
            if (d.post_scale) x = x * ps[e] + pt[e];
            o[e] = apply_act(x, d.act2);
          }
          if (d.gate)
            o *= *reinterpret_cast<const f32x4*>(d.gate + ((size_t)img * d.gate_nseg + wo / d.gate_seg) * d.gate_ld + n);
        }
        if (rowz) o = f32x4{0.f, 0.f, 0.f, 0.f};
        amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
#if SPK_REXP == 3 || SPK_REXP >= 5
        if (o[0] == 1234.5f)
#endif
        *reinterpret_cast<f32x4*>(out_at(d, m, n)) = o;
      }
    }
  };

  // prologue: the first two K-tiles of the block in flight
  set_issue_tile(0);
  issue_next(0);
  if (total > 1) issue_next(1);
  int st = 0, ci = 0, ck = 0;
  for (int it = 0; it < total; ++it) {
    // this wave's DMA of iteration `it` has landed (the RDMA of it+1 stay in flight); every
    // wave's fragment reads of the stage the next issue overwrites (read at it-1) are done
    if (it + 1 < total) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#if SPK_REXP != 2 && SPK_REXP < 5
    if (it + 2 < total) issue_next(st == 0 ? 2 : st - 1);
#endif
    compute(st);
    st = st == 2 ? 0 : st + 1;
    if (++ck == nkt) {
      epilogue(tbase + ci * tstep);
      ck = 0;
      ++ci;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = accx[j][r] = 0.f;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  range_note(d.range_flag, amax);
}

bool ring_enabled() {
  static const bool on = [] {
    // opt-in (SPK_RING=1): measured slower than the register-staged GEMM on every layer it
    // covers (ERes2NetV2 B=256 forward 24.9 -> 28.9 ms on MI355X)
    const char* e = std::getenv("SPK_RING");
    return e && std::string(e) == "1";
  }();
  return on;
}

}  // namespace

// The plain implicit GEMM (no K-concatenated second operand, no Res2Net addend, no BN-ReLU
// pre-activation, no split-K) of the fp16x3 path with N > 64 and M > 4096 rows, float4-aligned
// epilogue operands.
bool ring_supported(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  return ring_enabled() && conv_use_x3() && d.wh && d.wl && !d.x1 && !d.kcb && !d.s1.p && d.s1.cin == 0 &&
         !d.s0.p2 && d.s0.ld2 == 0 && !d.s0.pre_scale && d.ksplit <= 1 && d.N > 64 && M > 4096 && d.Kp % RBK == 0 &&
         d.N % 4 == 0 && d.ldo % 4 == 0 && (!d.res || d.ldr % 4 == 0) && (!d.affx || (d.ldx % 4 == 0 && d.ldy % 4 == 0)) &&
         (!d.gate || d.gate_ld % 4 == 0) && (!d.rowbias || d.rowbias_ld % 4 == 0) && conv_buf_loader_ok(d, RBM);
}

std::string ring_kernel_name(const ConvDesc&) { return "conv_gemm_ring_kernel"; }

int ring_tile_blocks(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  return ((M + RBM - 1) / RBM) * ((d.N + RBN - 1) / RBN);
}

// persistent grid: one block per CU (SPK_RING_GRID overrides; 0 = one block per tile)
static int ring_grid(int tiles) {
  static const int g = [] {
    const char* e = std::getenv("SPK_RING_GRID");
    if (e) return std::atoi(e);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
  }();
  if (g <= 0 || tiles <= g) return tiles;
  return std::max(8, g / 8 * 8);   // the tile split assumes whole groups of 8 (XCDs)
}

hipError_t launch_ring(const ConvDesc& d, hipStream_t s) {
  if (!ring_supported(d)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(conv_gemm_ring_kernel, dim3(ring_grid(ring_tile_blocks(d))), dim3(RNT), 0, s, d);
  return hipGetLastError();
}

}  // namespace spk
