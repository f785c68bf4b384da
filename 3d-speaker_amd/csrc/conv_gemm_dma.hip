// Implicit-GEMM convolution on fp16x3 MFMA with LDS-DMA staging (gfx950).
//
// The register-staged tiled GEMM (conv_gemm.hip) spends most of its time moving each K-tile
// global -> VGPR -> LDS: ablation builds (tools/gemm_exp.sh) took 26 % off its
// time without the in-loop LDS stores (and the load waits they carry) and only 7 % without
// the MFMAs.  Here both operands go global -> LDS by `buffer_load_dwordx4 ... lds` (no VGPR
// destination, no ds_write, no wait in the VALU stream), and the fp16x3 split of the fp32
// activations happens when the A fragments are read from LDS:
//   * 128 x 128 block tile, 256 threads: wave w owns output rows 32w .. 32w+31 and all 128
//     columns (four 32x32 MFMA tiles), so every A element is split exactly once per block;
//   * K-tile of 32, NS LDS stages of 32 KB (A: fp32 [k-half][row][16], B: fp16 hi / lo
//     planes [plane][col][32]), 64-B rows whose 16-B chunks are XOR-swizzled by
//     (row >> 2) & 3 -- the ds_read_b128 fragment reads are bank-conflict free and every
//     DMA lane keeps one fixed k-quad (the swizzle goes on the SOURCE address: the DMA
//     destination is lane-linear, cdna_hip_programming.md §5);
//   * NS = 3: the loads of K-tile kt+2 are issued right after the barrier of kt, which is
//     also the WAR barrier of the stage they overwrite -- one raw s_barrier per K-tile and a
//     counted vmcnt (one K-tile of DMA in flight across it; never __syncthreads(), whose
//     fence would drain the DMA, §5 "Pipelining across barriers");
//   * out-of-image taps, rows past M and K past the operand read offset BUF_OOB: the buffer
//     unit returns zeros and the DMA writes them (tests/test_gpu_lds_dma.py pins this);
//   * two accumulators (hi*hi, and hi*lo + lo*hi), no weight-range restriction.
// Numerics are those of conv_gemm.hip's fp16x3 kernels: x*w ~ hi_x hi_w + 2^-11 (hi_x lo_w +
// lo_x hi_w), products exact, fp32 accumulation.
#include <cstdlib>
#include <string>

#include "common.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

namespace spk {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int DBM = 128, DBN = 128, DBK = 32, DNT = 256;
constexpr int A_STAGE = DBM * DBK * 4;           // bytes: fp32 [2 k-halves][128 rows][64 B]
constexpr int B_STAGE = 2 * DBN * DBK * 2;       // bytes: fp16 [hi / lo][128 cols][64 B]
constexpr int STAGE = A_STAGE + B_STAGE;          // 32 KB

__device__ __forceinline__ int swz(int row) { return (row >> 2) & 3; }

// the fp16x3 split of 8 staged fp32 values (conv_epilogue.h split_x3, twice)
__device__ __forceinline__ void split8(const f32x4& a, const f32x4& b, f16x8& h, f16x8& l) {
  h16x4 h0, l0, h1, l1;
  split_x3(a, h0, l0);
  split_x3(b, h1, l1);
  h = f16x8{h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
  l = f16x8{l0[0], l0[1], l0[2], l0[3], l1[0], l1[1], l1[2], l1[3]};
}

template <int NS>
__global__ void __launch_bounds__(DNT, NS <= 2 ? 2 : 1)
conv_gemm_dma_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
  constexpr int LDS_EPI = 4 * 4 * 1024 * 4;     // epilogue: every accumulator of the block (bytes)
  constexpr int LDS_BYTES = NS * STAGE > LDS_EPI ? NS * STAGE : LDS_EPI;
  __shared__ __attribute__((aligned(16))) float lds[LDS_BYTES / 4];   // the only LDS object
  char* const lb = reinterpret_cast<char*>(lds);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + DBN - 1) / DBN;
  const int nM = (M + DBM - 1) / DBM;
  const int lid = xcd_remap(blockIdx.x, nM * nN);
  const int mt = lid / nN, nt = lid % nN;
  const int m0 = mt * DBM, n0 = nt * DBN;

  const int nkt_all = d.Kp / DBK;
  const int per = (nkt_all + d.ksplit - 1) / d.ksplit;
  const int kt0 = blockIdx.z * per;
  const int kt1 = min(nkt_all, kt0 + per);

  // ---- DMA geometry.  A: wave w fills k-half kh = w >> 1, row blocks 4(w & 1) + j
  // (j = 0..3, 16 rows x 64 B = one 1 KB wave-instruction each); lane -> row (lane >> 2) of the
  // block, LDS chunk slot lane & 3, i.e. source k-quad 4 kh + ((lane & 3) ^ swz(row)).
  const int kh = wave >> 1;
  const int cq = (lane & 3) ^ ((lane >> 4) & 3);   // swz(16 rb + (lane >> 2)) = (lane >> 4) & 3
  using AL = BufALoader<4, 16, DBK, false, false, false>;
  AL al;
  al.init(d, m0, 64 * (wave & 1) + (lane >> 2), 4 * kh + cq, kt0);
  // B: wave w fills plane w >> 1 (hi / lo), column blocks 4(w & 1) + j; columns past N read
  // zeros (offset past the range)
  const __amdgpu_buffer_rsrc_t brs = make_rsrc((wave >> 1) ? d.wl : d.wh);
  uint32_t boff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = 16 * (4 * (wave & 1) + j) + (lane >> 2);
    boff[j] = (n0 + n < d.N) ? ((uint32_t)(n0 + n) * d.Kp + cq * 8) * 2u : BUF_OOB;
  }
  const int a_dst = kh * (A_STAGE / 2) + 4 * (wave & 1) * 1024;     // + 1 KB per j
  const int b_dst = A_STAGE + (wave >> 1) * (B_STAGE / 2) + 4 * (wave & 1) * 1024;

  auto issue = [&](int kt, int stage) {
    uint32_t ao[4];
    al.offsets(d, ao);
    char* const sb = lb + stage * STAGE;
    const int koff = __builtin_amdgcn_readfirstlane(kt * DBK * 2);   // B: K-tile byte offset in a row
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(al.r0, (lds_ptr_t)(sb + a_dst + j * 1024), 16, (int)ao[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (lds_ptr_t)(sb + b_dst + j * 1024), 16, (int)boff[j], koff, 0, 0);
  };

  f32x16 acc[4], accx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc[j][r] = 0.f; accx[j][r] = 0.f; }

  const int li = lane & 31, lh = lane >> 5;
  const int arow = 32 * wave + li;
  // fragment reads: A row arow, k-half s, fp32 quads 2 lh, 2 lh + 1; B column 32 j + li,
  // halves 16 s + 8 lh .. +7 (chunk 2 s + lh) of each plane
  auto compute = [&](int stage) {
    const char* sb = lb + stage * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const char* ap = sb + s * (A_STAGE / 2) + arow * 64;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(ap + ((2 * lh) ^ swz(arow)) * 16);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(ap + ((2 * lh + 1) ^ swz(arow)) * 16);
      f16x8 bh[4], bl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = 32 * j + li;
        const char* bp = sb + A_STAGE + n * 64 + ((2 * s + lh) ^ swz(n)) * 16;
        bh[j] = *reinterpret_cast<const f16x8*>(bp);
        bl[j] = *reinterpret_cast<const f16x8*>(bp + B_STAGE / 2);
      }
      f16x8 ah, alo;
      split8(a0, a1, ah, alo);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[j], acc[j], 0, 0, 0);
        accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[j], accx[j], 0, 0, 0);
        accx[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(alo, bh[j], accx[j], 0, 0, 0);
      }
    }
  };

  if (kt0 < kt1) {
    static_assert(NS >= 3, "one barrier per K-tile needs three stages or more");
    // prologue: K-tiles kt0 .. kt0+NS-2 in flight (clamped: past the last tile a stage is
    // refilled with it again, unread, so every iteration's wait count is the same)
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) issue(min(kt0 + i, kt1 - 1), i);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      // this wave's DMA of K-tile kt has landed (the 8 per later tile may stay in flight);
      // every wave's reads of the stage the next issue overwrites (read at kt-1) are done
      if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (NS == 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int st2 = st == 0 ? NS - 1 : st - 1;  // (kt + NS - 1) % NS
      issue(min(kt + NS - 1, kt1 - 1), st2);
      compute(st);
      st = st == NS - 1 ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] += accx[j] * (1.0f / 2048.0f);
  __syncthreads();   // every wave's fragment reads done before the epilogue reuses the stages
  f32x16 (&acc2)[1][4] = *reinterpret_cast<f32x16(*)[1][4]>(&acc);
  epilogue_tiles<1, 4, false, false, true>(d, lds, acc2, wave, lane, n0, M, [&](int r) { return m0 + 32 * wave + r; });
}

bool dma_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("SPK_GEMM_DMA");
    return e && std::string(e) == "1";   // opt-in: measured slower
  }();
  return on;
}

}  // namespace

// The plain implicit GEMM (no K-concatenated second operand, no Res2Net addend, no
// BN-ReLU pre-activation) on the x3 path with N > 64 and M > 4096 rows: the shapes the
// register-staged kernel would run on 128-wide tiles.
bool gemm_dma_supported(const ConvDesc& d) {
  const int M = d.nimg * d.Ho * d.Wo;
  return dma_enabled() && conv_use_x3() && d.wh && d.wl && !d.x1 && !d.s1.p && d.s1.cin == 0 && !d.s0.p2 &&
         d.s0.ld2 == 0 && !d.s0.pre_scale && d.N > 64 && M > 4096 && d.Kp % DBK == 0 && conv_buf_loader_ok(d, DBM);
}

int dma_stages() {
  static const int ns = [] {
    const char* e = std::getenv("SPK_GEMM_DMA_NS");
    const int v = e ? std::atoi(e) : 4;
    return v >= 3 && v <= 5 ? v : 4;
  }();
  return ns;
}

std::string gemm_dma_kernel_name(const ConvDesc&) { return "conv_gemm_dma_kernel<" + std::to_string(dma_stages()) + ">"; }

hipError_t launch_gemm_dma(const ConvDesc& d, hipStream_t s) {
  if (!gemm_dma_supported(d)) return hipErrorInvalidValue;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nblk = ((M + DBM - 1) / DBM) * ((d.N + DBN - 1) / DBN);
  const dim3 grid(nblk, 1, d.ksplit);
  switch (dma_stages()) {
    case 3: hipLaunchKernelGGL((conv_gemm_dma_kernel<3>), grid, dim3(DNT), 0, s, d); break;
    case 5: hipLaunchKernelGGL((conv_gemm_dma_kernel<5>), grid, dim3(DNT), 0, s, d); break;
    default: hipLaunchKernelGGL((conv_gemm_dma_kernel<4>), grid, dim3(DNT), 0, s, d); break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess || d.ksplit <= 1) return e;
  return launch_splitk_reduce(d, s);
}

}  // namespace spk
