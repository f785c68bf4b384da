// fp16x3 implicit-GEMM convolution with fragment-packed weights streamed into LDS by
// LDS-DMA (gfx950).  The common layers of the ERes2Net(V2) stages 3-4 and every other plain
// conv the buffer-resource loader serves (conv_loader.h BufALoader conditions, no
// K-concatenated second operand, no BN-ReLU pre-activation).
//
// What differs from the register-staged kernel (conv_gemm.hip conv_gemm_x3_kernel):
//   * B (weights) never passes through VGPRs.  At model creation every packed weight matrix
//     is also laid out in MFMA fragment order (launch_pack_frag): per 32-deep K-tile, per
//     32-column n-tile, per 16-deep k-step, per plane (fp16 hi, fp16 lo) one 1-KB chunk whose
//     16-B lane slots are exactly the B operand of v_mfma_f32_32x32x16_f16.  A block's 16
//     chunks of a K-tile are contiguous; each wave moves two of them with
//     `buffer_load_dwordx4 ... lds` (no VGPR destination, no ds_write, no waits of its own)
//     and reads its fragments back with conflict-free ds_read_b128 (lane-linear 1-KB rows).
//   * A (fp32 activations) is staged through registers as before -- the fp16 hi / lo split
//     happens once per element, in the staging pass -- but the K walk is scalar: the K-tile
//     start (tap t0, channel c0) and the pixel deltas of taps t0 and t0 + 1 are wave-uniform
//     (SGPRs); a lane's quad is past the tap boundary or not (one compare, two selects), so
//     the loop body has no lane-divergent branch and no runtime-optional path (reflect padding,
//     channel-block K order, K-concatenated operands stay on the older kernel).
//   * The DMA is issued by inline asm, invisible to hipcc's wait counting: issued before the
//     K-tile's A loads, the compiler's counted wait for the previous A set also retires it
//     (vmcnt retires in order), and an explicit `s_waitcnt vmcnt(<A loads>)` before the
//     barrier makes that independent of the schedule.  (A DMA the compiler can see makes it
//     drain vmcnt(0) at every use of an ordinary load: cdna_hip_programming.md §5.)
// Numerics are those of the register-staged fp16x3 kernel (same split, same one-accumulator
// products, same K order): x w ~= 2^-11 (hi_x (2^11 hi_w) + hi_x lo_w + lo_x hi_w).
#include <cstdlib>
#include <string>
#include <type_traits>

#include "common.h"
#include "conv_epilogue.h"
#include "conv_loader.h"

#ifndef SPK_F_SCHED
#define SPK_F_SCHED 5   // loop schedule: 1 the one-set (256 x 256) loop splits + stores the next A
                        // set between its two k-steps (measured -5..-17 % on the N > 128 layers;
                        // 0: after both), 2 static priority for the second half of the waves
                        // (mixed, off), 4 the two-set loop splits between its k-steps too (0-3 %
                        // on the 128 x 128 layers)
#endif
#ifndef SPK_F_M16
#define SPK_F_M16 1   // 1: v_mfma_f32_16x16x32_f16 (round 6: 4-10 % faster per layer than 32x32x16, r06_ablation/m16_gemm.txt) (fragments packed for it, epilogue_tiles L16 layout)
#endif
#ifndef SPK_F_LPAD
#define SPK_F_LPAD (SPK_F_M16 ? 16 : 8)   // A row padding in halves (see FCfg::LROW)
#endif
#ifndef SPK_F_SKIP
#define SPK_F_SKIP 1   // M16: skip the MFMAs of 16-column blocks past N
#endif
#ifndef SPK_FEXP
#define SPK_FEXP 0   // ablation builds only (tools/fexp.sh), bit mask: 1 no MFMA, 2 no in-loop A loads,
                     // 4 no in-loop A split / stores, 8 no in-loop B DMA, 16 no epilogue (accumulators
                     // summed), 32 epilogue without its residual loads
#endif

namespace spk {

namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int FBK = 32;
constexpr int F_NPAD = 256;                          // packed N padded to the widest tile

// Tile geometry: BM x BN block tile, WM x WN waves, each wave TM x TN 32x32 accumulator tiles.
template <int BM, int BN, int WM, int WN>
struct FCfg {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  // A rows: 32 halves + 16 (96 B).  ds_read_b128 serves lanes in the groups {0-3, 12-15, 20-27}, {4-11, 16-19,
  // 28-31}, ... (MI355X_MICROARCH.md, LDS): with 16x16x32 fragments (lane: row l & 15, 16-B block l >> 4)
  // a 96-B row stride puts every group on 16 distinct 4-bank sets; the 80-B stride of the 32x32x16
  // form left 3 lanes per group 2-way conflicted (SQ_LDS_BANK_CONFLICT 42 % of the LDS cycles)
  static constexpr int LROW = FBK + SPK_F_LPAD;
  static constexpr int PA = BM * LROW;               // halves per A plane
  static constexpr int ASTAGE = 2 * PA * 2;          // bytes: A hi + lo
  static constexpr int CHUNKS = (BN / 32) * 2 * 2;   // B chunks per K-tile: n-tiles x k-steps x planes
  static constexpr int CPW = CHUNKS / (WM * WN);     // DMA chunks per wave per K-tile
  static constexpr int STAGE = ASTAGE + CHUNKS * 1024;
  // epilogue_tiles' slab: the whole wave tile when it fits next to nothing else (128 x 128),
  // else one row of accumulator tiles at a time
  static constexpr int SLAB = epi_slab_floats<SPK_F_M16 != 0>() * 4;   // bytes per 32x32 tile
  static constexpr int EPI_ALL = WM * WN * TM * TN * SLAB;
  static constexpr bool EPI_ONE = EPI_ALL <= 2 * STAGE;
  static constexpr int EPI = EPI_ONE ? EPI_ALL : WM * WN * TN * SLAB;
  static constexpr int LDS = 2 * STAGE > EPI ? 2 * STAGE : EPI;
  static constexpr int ROWS = BM / (NT / 8);         // A rows staged per thread
  static constexpr bool ONE_SET = TM * TN >= 8;     // 128 accumulator registers per wave
  static constexpr int WAVES_PER_EU = LDS <= 80 * 1024 ? 2 * WM * WN / 4 : WM * WN / 4;
  static_assert(TM >= 1 && TN >= 1 && CPW >= 1 && CHUNKS % (WM * WN) == 0 && BM % (NT / 8) == 0, "tile");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// LDS-DMA of one 16-B slot per lane: LDS[m0_base + 16 lane] = mem[rsrc + voff + soff].
// M0 is compiler-reserved: saved and restored inside the statement.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff, uint32_t lds_base) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %4\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(rs), "s"(soff), "s"(lds_base)
      : "memory");
}

template <int I, int E>
struct StaticFor {
  template <class F>
  __device__ __forceinline__ static void run(F& f) {
    f(std::integral_constant<int, I>{});
    StaticFor<I + 1, E>::run(f);
  }
};
template <int E>
struct StaticFor<E, E> {
  template <class F>
  __device__ __forceinline__ static void run(F&) {}
};

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// OP2: the second A operand -- 0 none, 1 the Res2Net addend (s0.p2, summed into A), 2 the
// K-concatenated 1x1 operand s1 (projection shortcut / AFF concat: K = taps * s0.cin + s1.cin)
template <int BM, int BN, int WM, int WN, int OP2>
__global__ void __launch_bounds__(64 * WM * WN, (FCfg<BM, BN, WM, WN>::WAVES_PER_EU))
conv_gemm_x3f_kernel(const ConvDesc d) {
  SPK_GATE(d.run_if);
  const float sc = range_scale_flat(d.range_in);            // scaled split: operand x 2^-s (common.h)
  using C = FCfg<BM, BN, WM, WN>;
  constexpr bool ADD = OP2 == 1, S1 = OP2 == 2;
  constexpr int TM = C::TM, TN = C::TN, ROWS = C::ROWS, NT = C::NT;
  constexpr int RPP = NT / 8;                          // rows per staging pass
  __shared__ __attribute__((aligned(16))) float lds[C::LDS / 4];
  char* const lb = reinterpret_cast<char*>(lds);
  const uint32_t lbase = lds_addr(lb);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int M = d.nimg * d.Ho * d.Wo;
  const int nN = (d.N + BN - 1) / BN;
  const int nM = (M + BM - 1) / BM;
  const int lid = xcd_remap(blockIdx.x, nM * nN);
  const int mt = lid / nN, nt = lid % nN;
  const int m0 = mt * BM, n0 = nt * BN;

  const int nkt_all = d.Kp / FBK;
  const int per = (nkt_all + d.ksplit - 1) / d.ksplit;
  const int kt0 = blockIdx.z * per;
  const int kt1 = min(nkt_all, kt0 + per);

  // ---- A: per-row constants (conv_loader.h BufALoader, without the reflect / kcb forms)
  const int kq = tid & 7, row0 = tid >> 3;            // thread: quad kq of rows row0 + RPP r
  const int img0 = m0 / (d.Ho * d.Wo);
  const size_t img_px = (size_t)d.s0.H * d.s0.W;
  const __amdgpu_buffer_rsrc_t r0 = make_rsrc(d.s0.p + (size_t)img0 * img_px * d.s0.ld);
  __amdgpu_buffer_rsrc_t r2;
  if (ADD) r2 = make_rsrc(d.s0.p2 + (size_t)img0 * img_px * d.s0.ld2);
  if (S1) r2 = make_rsrc(d.s1.p + (size_t)img0 * d.s1.H * d.s1.W * d.s1.ld);
  uint32_t roff[ROWS], roff2[OP2 ? ROWS : 1], rmask[ROWS];
  uint32_t rvalid = 0;                                // S1: bit r = row r < M
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int m = m0 + row0 + RPP * r;
    const bool valid = m < M;
    const int mm = valid ? m : m0;
    const int wo = mm % d.Wo, t2 = mm / d.Wo, ho = t2 % d.Ho, img = t2 / d.Ho;
    const int hb = ho * d.s0.sh - d.s0.ph, wb = wo * d.s0.sw - d.s0.pw;
    const int pix = ((img - img0) * d.s0.H + hb) * d.s0.W + wb;   // may be negative: masked
    roff[r] = (uint32_t)pix * (uint32_t)d.s0.ld * 4u;
    if (ADD) roff2[r] = (uint32_t)pix * (uint32_t)d.s0.ld2 * 4u;
    if (S1)
      roff2[r] = (uint32_t)((((img - img0) * d.s1.H + ho * d.s1.sh) * d.s1.W + wo * d.s1.sw) * d.s1.ld) * 4u;
    if (valid) rvalid |= 1u << r;
    const int wl = d.s0.vlen ? min(d.s0.W, d.s0.vlen[img]) : d.s0.W;
    uint32_t mk = 0;
    for (int ky = 0; ky < d.s0.kh; ++ky) {
      const int hi = hb + ky * d.s0.dh;
      if (hi < 0 || hi >= d.s0.H) continue;
      for (int x = 0; x < d.s0.kw; ++x) {
        const int wi = wb + x * d.s0.dw;
        if (wi >= 0 && wi < wl) mk |= 1u << (ky * d.s0.kw + x);
      }
    }
    rmask[r] = valid ? mk : 0u;   // bit `taps` (K padding past the last tap) is never set
  }

  // ---- scalar K walk: tile start (tap t0, channel c0), pixel deltas of taps t0 and t0 + 1
  // (past the last tap the walk stays at t0 = taps and c0 counts channels of s1)
  const int cin = d.s0.cin, kw = d.s0.kw, taps = d.s0.kh * d.s0.kw;
  const int dyW = d.s0.dh * d.s0.W, dx = d.s0.dw;
  int t0, c0, kyB, kxB, tdpA, tdpB;
  {
    const int k = kt0 * FBK;
    t0 = min(k / cin, taps);
    c0 = k - t0 * cin;
    const int ky = t0 / kw, kx = t0 - ky * kw;
    tdpA = ky * dyW + kx * dx;
    kxB = kx + 1;
    kyB = ky;
    if (kxB == kw) { kxB = 0; ++kyB; }
    tdpB = kyB * dyW + kxB * dx;
  }

  // ---- B: this wave's DMA chunks of a K-tile (chunk cb = CPW wave + j of the block's CHUNKS,
  // cb = (local n-tile) * 4 + k-step * 2 + plane)
  const int NJ = (d.N + F_NPAD - 1) / F_NPAD * (F_NPAD / 32);   // 32-column n-tiles of the packed matrix
  const __amdgpu_buffer_rsrc_t brs = make_rsrc(d.wf);
  const uint32_t bvoff = (uint32_t)lane * 16u;
  auto dma_b = [&](int kt, int buf) {
    if ((SPK_FEXP & 8) && kt != kt0) return;
#pragma unroll
    for (int j = 0; j < C::CPW; ++j) {
      const int cb = C::CPW * wave + j;
      const uint32_t soff = (uint32_t)(((kt * NJ + nt * (BN / 32)) * 4 + cb) * 1024);
      dma16(brs, bvoff, __builtin_amdgcn_readfirstlane(soff),
            __builtin_amdgcn_readfirstlane(lbase + buf * C::STAGE + C::ASTAGE + cb * 1024));
    }
  };

  struct ASet {
    f32x4 v[ROWS];
    f32x4 v2[OP2 ? ROWS : 1];
  };
  // issue the A loads of the K-tile at the walk position, then advance the walk by BK
  bool inloop = false;   // (ablation builds)
  auto load_a = [&](ASet& s) {
    const int c = c0 + 4 * kq;
    const bool sel = t0 < taps && c >= cin;            // this quad lies in tap t0 + 1 (or s1)
    const int cc = sel ? c - cin : c;
    const int t = min(t0 + (sel ? 1 : 0), 31);       // taps: past s0 (s1, or K padding: no mask bit)
    const int tdp = sel ? tdpB : tdpA;
    const uint32_t toff = (uint32_t)(tdp * d.s0.ld + cc) * 4u;
    const uint32_t toff2 = ADD ? (uint32_t)(tdp * d.s0.ld2 + cc) * 4u : (uint32_t)cc * 4u;
    const bool in1 = S1 && t == taps && cc < d.s1.cin;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
      const bool ok = (rmask[r] >> t) & 1u;
      if (!(SPK_FEXP & 2) || !inloop) {
        s.v[r] = buf_load4(r0, ok ? roff[r] + toff : BUF_OOB);
        if (ADD) s.v2[r] = buf_load4(r2, ok ? roff2[r] + toff2 : BUF_OOB);
        if (S1) s.v2[r] = buf_load4(r2, (in1 && ((rvalid >> r) & 1u)) ? roff2[r] + toff2 : BUF_OOB);
      }
    }
    c0 += FBK;
    if (t0 < taps && c0 >= cin) {                      // cin >= 32: one tap boundary per K-tile
      c0 -= cin;
      ++t0;
      tdpA = tdpB;
      if (++kxB == kw) { kxB = 0; ++kyB; }
      tdpB = kyB * dyW + kxB * dx;
    }
  };
  auto store_a = [&](int buf, const ASet& s, auto split) {
    if ((SPK_FEXP & 4) && inloop) return;
    _Float16* ahi = reinterpret_cast<_Float16*>(lb + buf * C::STAGE);
    _Float16* alo = ahi + C::PA;
    {
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        f32x4 v = s.v[r];
        if (OP2) v += s.v2[r];                         // addend, or s1 (exactly one of the two is nonzero)
        f16x4 h, l;
        split(v, h, l);
        const int off = (row0 + RPP * r) * C::LROW + kq * 4;
        *reinterpret_cast<f16x4*>(ahi + off) = h;
        *reinterpret_cast<f16x4*>(alo + off) = l;
      }
    }
  };

#if SPK_F_M16
  // 16x16x32 form: each 32x32 tile of the wave is four 16x16 accumulators; a K-tile is one
  // MFMA k-step (K = 32).  compute_s(buf, s) runs row half s (16-row blocks s*TM .. s*TM+TM-1)
  // of the wave tile; half 0 also reads the B fragments (kept in registers for half 1).
  // Fragment order (pack_frag_kernel M16): chunk (32-col tile j, 16-col half h, plane p) at
  // j * 4096 + (2 h + p) * 1024, lane l: column 16 h + (l & 15), k = 8 (l >> 4) + e.
  f32x4 acc[2 * TM][2 * TN];
#pragma unroll
  for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
    for (int j = 0; j < 2 * TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 bh[2 * TN], bl[2 * TN], bh2[2 * TN];
  // columns of the packed N (padded to 256) this wave's tile actually holds: the MFMAs of
  // 16-column blocks past N are skipped (N = 104 / 208 / 416 fill 81 % of their 128 / 256 tiles)
  const int ncols = __builtin_amdgcn_readfirstlane(d.N - (n0 + wn * TN * 32));
  auto compute_s = [&](int buf, int s) {
    const _Float16* ahi = reinterpret_cast<const _Float16*>(lb + buf * C::STAGE);
    if (s == 0) {
      const char* bb = lb + buf * C::STAGE + C::ASTAGE + wn * TN * 4096 + lane * 16;
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j) {
        bh[j] = *reinterpret_cast<const f16x8*>(bb + (j >> 1) * 4096 + (j & 1) * 2048);
        bl[j] = *reinterpret_cast<const f16x8*>(bb + (j >> 1) * 4096 + (j & 1) * 2048 + 1024);
        bh2[j] = bh[j] * (_Float16)2048.0f;   // exact (|w| < 31.5: ConvDesc::wbig)
      }
    }
#pragma unroll
    for (int ii = 0; ii < TM; ++ii) {
      const int i = s * TM + ii;
      const _Float16* p = ahi + (wm * TM * 32 + i * 16 + (lane & 15)) * C::LROW + 8 * (lane >> 4);
      const f16x8 ah = *reinterpret_cast<const f16x8*>(p);
      const f16x8 al = *reinterpret_cast<const f16x8*>(p + C::PA);
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j) {
#if SPK_F_SKIP
        if (j * 16 >= ncols) continue;                   // a 16-column block wholly past N (wave-uniform)
#endif
        if (SPK_FEXP & 1) {
          acc[i][j][0] += (float)ah[0] + (float)bh2[j][1] + (float)bl[j][2] + (float)al[3] + (float)bh[j][4];
          continue;
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh2[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[j], acc[i][j], 0, 0, 0);
      }
    }
  };
#else
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  // one 16-deep k-step of a K-tile (s = 0, 1)
  auto compute_s = [&](int buf, int s) {
    const _Float16* ahi = reinterpret_cast<const _Float16*>(lb + buf * C::STAGE);
    const char* bb = lb + buf * C::STAGE + C::ASTAGE + wn * TN * 4096 + lane * 16;
    {
      f16x8 ah[TM], al[TM], bh[TN], bl[TN], bh2[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const _Float16* p = ahi + (wm * TM * 32 + i * 32 + li) * C::LROW + lh * 16 + 8 * s;
        ah[i] = *reinterpret_cast<const f16x8*>(p);
        al[i] = *reinterpret_cast<const f16x8*>(p + C::PA);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const f16x8*>(bb + j * 4096 + s * 2048);
        bl[j] = *reinterpret_cast<const f16x8*>(bb + j * 4096 + s * 2048 + 1024);
        bh2[j] = bh[j] * (_Float16)2048.0f;   // exact (|w| < 31.5: ConvDesc::wbig)
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (SPK_FEXP & 1) {
            acc[i][j][0] += (float)ah[i][0] + (float)bh2[j][1] + (float)bl[j][2] + (float)al[i][3] + (float)bh[j][4];
            continue;
          }
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh2[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  };
#endif
  auto compute = [&](int buf) {
    compute_s(buf, 0);
    compute_s(buf, 1);
  };

  constexpr int ALOADS = ROWS * (OP2 ? 2 : 1);       // ordinary loads per A set
  // Pairs of K-tiles (even step: LDS buffer 0, odd step: buffer 1; A register sets 0 / 1 two
  // K-tiles ahead), an odd last K-tile peeled after the loop: the loop has one back edge, so
  // hipcc's wait counting sees the same loads in flight on both paths into its header (with a
  // `break` between the steps it merged two states and waited vmcnt(0) at the top).  Every
  // load and DMA in the loop is unconditional (clamped past the end: zeros, or a re-read of
  // the last tile into the idle buffer), so the body has no branch around a memory operation.
  // The whole K loop twice behind one uniform branch: the plain split while the range word is
  // clear, the scaled split (common.h) otherwise (a branch in the loop body would split the
  // basic block the sched_barrier placement relies on).
  split_pass(sc, [&](auto split) {
  if (C::ONE_SET && kt0 < kt1) {
    // one A register set (the 256 x 256 tile, whose accumulators take half the registers):
    // the loads of K-tile kt + 1 are issued right after the stores of kt, so they have the
    // whole next compute step (48 MFMAs per wave) to land
    ASet set;
    dma_b(kt0, 0);
    load_a(set);
    store_a(0, set, split);
    load_a(set);                                       // kt0 + 1
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALOADS) : "memory");   // B of kt0 landed
    __syncthreads();
    inloop = true;
#if SPK_F_SCHED & 2
    if (wave >= C::NT / 128) __builtin_amdgcn_s_setprio(1);   // the second-dispatched half of the waves
#endif
    for (int kt = kt0; kt < kt1; ++kt) {
      const int buf = (kt - kt0) & 1;
      dma_b(min(kt + 1, kt1 - 1), buf ^ 1);           // buffer buf ^ 1 was read before the last barrier
#if SPK_F_SCHED & 1
      // the A set's split + LDS stores between the two k-steps: its VALU / LDS work issues in
      // the gaps of the second k-step's MFMAs
      compute_s(buf, 0);
      __builtin_amdgcn_sched_barrier(0);
      store_a(buf ^ 1, set, split);
      load_a(set);
      compute_s(buf, 1);
#else
      compute(buf);
      // keep the split of the A set (loaded at the end of the previous step) behind the MFMAs:
      // hoisted to the top of the step it waited for those loads before any MFMA could issue
      __builtin_amdgcn_sched_barrier(0);
      store_a(buf ^ 1, set, split);                    // K-tile kt + 1 (past the end: unused)
      load_a(set);                                     // kt + 2
#endif
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALOADS) : "memory");   // B of kt + 1 landed
      __syncthreads();
    }
#if SPK_F_SCHED & 2
    __builtin_amdgcn_s_setprio(0);
#endif
  } else if (kt0 < kt1) {
    ASet set0, set1;
    dma_b(kt0, 0);
    load_a(set0);
    load_a(set1);                                      // kt0 + 1 (or past the end: unused)
    store_a(0, set0, split);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALOADS) : "memory");   // B of kt0 landed
    __syncthreads();
    inloop = true;
    int kt = kt0;
    for (; kt + 1 < kt1; kt += 2) {
      // even step: buffer 0 holds kt; set 1 holds kt + 1 (in flight)
      dma_b(kt + 1, 1);
      load_a(set0);                                    // kt + 2
#if SPK_F_SCHED & 4
      compute_s(0, 0);
      __builtin_amdgcn_sched_barrier(0);
      store_a(1, set1, split);
      compute_s(0, 1);
#else
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      store_a(1, set1, split);
#endif
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALOADS) : "memory");   // B of kt + 1 landed
      __syncthreads();
      // odd step: buffer 1 holds kt + 1; set 0 holds kt + 2 (in flight)
      dma_b(min(kt + 2, kt1 - 1), 0);
      load_a(set1);                                    // kt + 3
#if SPK_F_SCHED & 4
      compute_s(1, 0);
      __builtin_amdgcn_sched_barrier(0);
      store_a(0, set0, split);
      compute_s(1, 1);
#else
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      store_a(0, set0, split);
#endif
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ALOADS) : "memory");
      __syncthreads();
    }
    if (kt < kt1) {                                    // odd count: the last K-tile is in buffer 0
      compute(0);
      __syncthreads();                                 // the epilogue reuses the LDS
    }
  }
  });
  const float back = pow2_div(sc, -11);               // 2^(-11) / sc, exact
#if SPK_F_M16
  // the four 16x16 accumulators of 32x32 tile (i, j) as one f32x16 (epilogue_tiles L16)
#pragma unroll
  for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
    for (int j = 0; j < 2 * TN; ++j) acc[i][j] *= back;
  auto tile = [&](int i, int j) {
    f32x16 t;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[4 * q + e] = acc[2 * i + (q >> 1)][2 * j + (q & 1)][e];
    return t;
  };
  constexpr bool L16 = true;
#else
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] *= back;
  auto tile = [&](int i, int j) { return acc[i][j]; };
  constexpr bool L16 = false;
#endif
#if SPK_FEXP & 16
  {
    // every accumulator stays live (a test of two elements let the compiler drop the MFMAs of
    // all other tiles: the round-5 form of this ablation measured that, not the epilogue)
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x16 t = tile(i, j);
#pragma unroll
        for (int r = 0; r < 16; ++r) sum += t[r];
      }
    if (sum == 1234.5f) d.out[tid] = sum;
  }
#else
#if SPK_FEXP & 32
  ConvDesc dnores = d;                                   // ablation: epilogue without its residual loads
  dnores.res = nullptr;
#define d dnores
#endif
  // one row of accumulator tiles at a time through the wave's slab (TN x 4 KB): the whole
  // wave tile of a 256-wide block would not fit in LDS
  if constexpr (C::EPI_ONE) {
    f32x16 all[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) all[i][j] = tile(i, j);
    epilogue_tiles<TM, TN, false, false, false, L16>(d, lds, all, wave, lane, n0 + wn * TN * 32, M,
                                                     [&](int r) { return m0 + wm * TM * 32 + r; });
    return;
  }
  // compile-time row index (a runtime one, e.g. from a loop the compiler does not unroll around
  // the large inlined epilogue, puts the accumulators in scratch)
  auto epi_row = [&](auto ic) {
    constexpr int i = decltype(ic)::value;
    const int rb = m0 + wm * TM * 32 + i * 32;
    f32x16 row[1][TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) row[0][j] = tile(i, j);
    epilogue_tiles<1, TN, false, false, false, L16>(d, lds, row, wave, lane, n0 + wn * TN * 32, M,
                                                    [&](int r) { return rb + r; });
  };
  StaticFor<0, TM>::run(epi_row);
#if SPK_FEXP & 32
#undef d
#endif
#endif
}

// fragment order of one packed weight matrix (see the file comment):
// out[((kt * NJ + j) * 4 + s * 2 + p) * 512 + lane * 8 + e] = plane_p[n][k] with
// n = 32 j + (lane & 31), k = 32 kt + 16 (lane >> 5) + 8 s + e (zero for n >= N)
__global__ void pack_frag_kernel(const uint16_t* __restrict__ wh, const uint16_t* __restrict__ wl, int N, int Kp,
                                 int NJ, uint16_t* __restrict__ out) {
  const size_t total = (size_t)(Kp / 32) * NJ * 4 * 64;   // 16-B slots
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int lane = (int)(i & 63);
    const size_t ch = i >> 6;
    const int p = (int)(ch & 1), s = (int)((ch >> 1) & 1);
    const size_t kj = ch >> 2;
    const int j = (int)(kj % NJ), kt = (int)(kj / NJ);
#if SPK_F_M16
    // (s = the 16-column half) n = 32 j + 16 s + (lane & 15), k = 32 kt + 8 (lane >> 4) + e
    const int n = 32 * j + 16 * s + (lane & 15), k = 32 * kt + 8 * (lane >> 4);
#else
    const int n = 32 * j + (lane & 31), k = 32 * kt + 16 * (lane >> 5) + 8 * s;
#endif
    u32x4 v = {0u, 0u, 0u, 0u};
    if (n < N) v = *reinterpret_cast<const u32x4*>((p ? wl : wh) + (size_t)n * Kp + k);
    *reinterpret_cast<u32x4*>(out + i * 8) = v;
  }
}

}  // namespace

size_t frag_halves(int N, int Kp) { return (size_t)Kp * (size_t)((N + F_NPAD - 1) / F_NPAD * F_NPAD) * 2; }

hipError_t launch_pack_frag(const uint16_t* wh, const uint16_t* wl, int N, int Kp, uint16_t* out, hipStream_t s) {
  if (N <= 0 || Kp <= 0 || Kp % 32 || !wh || !wl || !out) return hipErrorInvalidValue;
  const int NJ = (N + F_NPAD - 1) / F_NPAD * (F_NPAD / 32);
  const size_t slots = (size_t)(Kp / 32) * NJ * 256;
  const int blocks = (int)std::min<size_t>((slots + 255) / 256, 4096);
  hipLaunchKernelGGL(pack_frag_kernel, dim3(blocks), dim3(256), 0, s, wh, wl, N, Kp, NJ, out);
  return hipGetLastError();
}

namespace {

struct FTile {
  int bm, bn;
};

// the two-operand forms (the naming probe of runtime.cpp sets the sizes without pointers)
bool has_add(const ConvDesc& d) { return d.s0.p2 != nullptr || d.s0.ld2 > 0; }
bool has_s1(const ConvDesc& d) { return d.s1.p != nullptr || d.s1.cin > 0; }

// tile per layer: SPK_GEMM_F_TILE=128x128 | 256x128 | 128x256 | 256x256 overrides (experiments)
FTile f_tile(const ConvDesc& d) {
  static const int forced = [] {
    const char* e = std::getenv("SPK_GEMM_F_TILE");
    if (!e) return 0;
    const std::string v(e);
    return v == "128x128" ? 1 : v == "256x128" ? 2 : v == "128x256" ? 3 : v == "256x256" ? 4 : 0;
  }();
  switch (forced) {
    case 1: return {128, 128};
    case 2: return {256, 128};
    case 3: return {128, 256};
    case 4: return (has_add(d) || has_s1(d)) ? FTile{128, 128} : FTile{256, 256};
    default: break;
  }
  // measured (tools/gemm_bench, ERes2NetV2 B = 256 layer shapes, round 5): the 256 x 256 tile
  // (8 waves of 128 x 64, one block per CU, half the LDS fragment reads per MFMA of the 64 x 32
  // wave tile) is fastest on every layer with N > 128, even where N = 208 / 416 leaves 19 % of
  // its columns empty (l3 conv1 313 -> 280 us, l4 conv1 275 -> 230, l4 3x3 215 -> 184, l3_ds
  // 2067 -> 1766); the 104-wide layers keep 128 x 128 at two blocks per CU
  // Two conditions keep a layer off it: a last round of blocks that leaves most CUs idle (one
  // block per CU: ECAPA's 1x1 convs at B = 256, 792 blocks = 3.1 rounds, 0.39 -> 0.55 ms), and
  // a short K with the AFF epilogue (fuse34's local_att.3, K = 256: its epilogue reads two
  // operands and is not overlapped by a second resident block, 0.22 -> 0.25 ms; the residual
  // conv3s of layer 3, K = 208, gain: 425 -> 396 us).
  const int M = d.nimg * d.Ho * d.Wo;
  if (d.N > 128 && M >= 16384 && !has_add(d) && !has_s1(d) && (d.Kp >= 512 || (!d.affx && !d.gate))) {
    const int cus = device_cus();
    const double rounds = (double)((M + 255) / 256) * ((d.N + 255) / 256) / cus;
    const double tail = rounds - (int)rounds;
    if (rounds >= 4.0 || tail == 0.0 || tail >= 0.6) return {256, 256};
  }
  return {128, 128};
}

template <int BM, int BN, int WM, int WN>
hipError_t launch_f_t(const ConvDesc& d, hipStream_t s) {
  const int M = d.nimg * d.Ho * d.Wo;
  const int nblk = ((M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
  dim3 grid(nblk, 1, d.ksplit);
  const dim3 blk(64 * WM * WN);
  if (d.s0.p2 || d.s1.p) {
    // f_tile: 128 x 128 for the two-operand forms (the 256 x 256 one spills)
    if constexpr (BM * BN >= 256 * 256) return hipErrorInvalidValue;
    else if (d.s0.p2) hipLaunchKernelGGL((conv_gemm_x3f_kernel<BM, BN, WM, WN, 1>), grid, blk, 0, s, d);
    else hipLaunchKernelGGL((conv_gemm_x3f_kernel<BM, BN, WM, WN, 2>), grid, blk, 0, s, d);
  } else {
    hipLaunchKernelGGL((conv_gemm_x3f_kernel<BM, BN, WM, WN, 0>), grid, blk, 0, s, d);
  }
  return hipGetLastError();
}

}  // namespace

bool gemm_f_supported(const ConvDesc& d) {
  static const bool off = [] {
    const char* e = std::getenv("SPK_GEMM_F");
    return e && std::string(e) == "0";
  }();
  const int M = d.nimg * d.Ho * d.Wo;
  const FTile t = f_tile(d);
  return !off && d.wf && d.wh && d.wl && !d.wbig && !d.x1 && !d.kcb && !d.s0.reflect && !d.s0.pre_scale &&
         d.N > 64 && M > 4096 && d.Kp % FBK == 0 && d.Kp >= d.K && !(has_add(d) && has_s1(d)) &&
         // K-concatenated s1: a 1x1 operand with the output's geometry (strided rows allowed)
         (!has_s1(d) || (d.s1.cin % 4 == 0 && d.s1.ld % 4 == 0 && d.K == d.s0.kh * d.s0.kw * d.s0.cin + d.s1.cin)) &&
         conv_buf_loader_ok(d, t.bm);
}

std::string gemm_f_kernel_name(const ConvDesc& d) {
  const bool add = d.s0.p2 != nullptr || d.s0.ld2 > 0, s1 = d.s1.p != nullptr || d.s1.cin > 0;
  const FTile t = f_tile(d);
  const int wm = t.bm == 256 && t.bn == 128 ? 4 : 2, wn = 8 / wm;
  return "conv_gemm_x3f_kernel<" + std::to_string(t.bm) + ", " + std::to_string(t.bn) + ", " + std::to_string(wm) +
         ", " + std::to_string(wn) + ", " + (add ? "1" : s1 ? "2" : "0") + ">";
}

hipError_t launch_gemm_f(const ConvDesc& d, hipStream_t s) {
  if (!gemm_f_supported(d)) return hipErrorInvalidValue;
  const FTile t = f_tile(d);
  hipError_t e;
  if (t.bm == 256 && t.bn == 256) e = launch_f_t<256, 256, 2, 4>(d, s);
  else if (t.bm == 256) e = launch_f_t<256, 128, 4, 2>(d, s);
  else if (t.bn == 256) e = launch_f_t<128, 256, 2, 4>(d, s);
  else e = launch_f_t<128, 128, 2, 4>(d, s);
  if (e != hipSuccess || d.ksplit <= 1) return e;
  return launch_splitk_reduce(d, s);
}

}  // namespace spk
