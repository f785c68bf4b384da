// Fused conv epilogue shared by the implicit-GEMM and the halo-tiled conv kernels.
#pragma once
#include <type_traits>

#include "common.h"

namespace spk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.0f);
    case ACT_HTANH: return fminf(fmaxf(v, 0.0f), 20.0f);
    case ACT_SILU: return v * __builtin_amdgcn_rcpf(1.0f + __expf(-v));   // v_rcp (1 ulp), no IEEE divide sequence
    case ACT_SIGMOID: return __builtin_amdgcn_rcpf(1.0f + __expf(-v));
    case ACT_TANH: return tanhf(v);
    default: return v;
  }
}

// AFF combine (fusion.py:26-28): x (1 + tanh v) + y (1 - tanh v) = 2 (y + sigmoid(2 v) (x - y))
// -- one exp and one reciprocal instead of tanhf's branches (aff.hip uses the same form)
__device__ __forceinline__ float aff_combine(float v, float x, float y) {
  const float sg = __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * v));
  return 2.0f * fmaf(sg, x - y, y);
}

// fp16x3 split of a staged fp32 quad (conv_gemm.hip "fp16x3"): hi = fp16(v) and
// lo = fp16((v - hi) * 2^11), with packed round-toward-zero conversions (two values per
// instruction, already packed; |v - hi| < ulp(hi) and lo keeps the remainder to 2^-22).
typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
#ifndef SPK_SPLIT_MIX
#define SPK_SPLIT_MIX 1   // 0: the round-3 form (cvt back to fp32, subtract, scale, cvt: 4 VALU per value)
#endif
// lo of two values from their packed hi: fp16(2^11 v - 2^11 hi) by v_fma_mix{lo,hi}_f16 (the
// hi operand read as fp16 from its packed half, 2^11 v exact), one rounding (to nearest) of an
// exact remainder: 2.5 VALU per value with the hi conversion.  Inline asm: hipcc otherwise
// unpacks hi and rebuilds the remainder in fp32.
__device__ __forceinline__ uint32_t split_lo2(uint32_t hp, float v0, float v1) {
  uint32_t r;
  const float m = -2048.0f;
  asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, %2, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(hp), "s"(m), "v"(v0 * 2048.0f), "v"(v1 * 2048.0f));
  return r;
}
__device__ __forceinline__ void split_x3(const f32x4 v, h16x4& h, h16x4& l) {
  typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
#if SPK_SPLIT_MIX
  const uint32_t h01 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v[0], v[1]));
  const uint32_t h23 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v[2], v[3]));
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  h = __builtin_bit_cast(h16x4, u32x2v{h01, h23});
  l = __builtin_bit_cast(h16x4, u32x2v{split_lo2(h01, v[0], v[1]), split_lo2(h23, v[2], v[3])});
#else
  const h16x2 h01 = __builtin_bit_cast(h16x2, __builtin_amdgcn_cvt_pkrtz(v[0], v[1]));
  const h16x2 h23 = __builtin_bit_cast(h16x2, __builtin_amdgcn_cvt_pkrtz(v[2], v[3]));
  const h16x2 l01 = __builtin_bit_cast(
      h16x2, __builtin_amdgcn_cvt_pkrtz((v[0] - (float)h01[0]) * 2048.0f, (v[1] - (float)h01[1]) * 2048.0f));
  const h16x2 l23 = __builtin_bit_cast(
      h16x2, __builtin_amdgcn_cvt_pkrtz((v[2] - (float)h23[0]) * 2048.0f, (v[3] - (float)h23[1]) * 2048.0f));
  h = h16x4{h01[0], h01[1], h23[0], h23[1]};
  l = h16x4{l01[0], l01[1], l23[0], l23[1]};
#endif
}

// split of sc * v (scaled split, common.h: sc = 2^-s, an SGPR) with the scale folded into
// the conversions, so the scaled quad is never materialised (a separate multiply measured
// +3 VGPRs and spills on the 128x128 tiled GEMM): hi = fp16(sc v) by v_fma_mix{lo,hi} (the
// product exact, one round to nearest), lo = fp16(2^11 sc v - 2^11 hi) as in split_lo2
__device__ __forceinline__ uint32_t split_hi2s(float v0, float v1, float sc) {
  uint32_t r;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %2, 0"
      : "=&v"(r)
      : "v"(v0), "v"(sc), "v"(v1));
  return r;
}
__device__ __forceinline__ uint32_t split_lo2s(uint32_t hp, float a0, float a1) {   // a = 2^11 sc v
  uint32_t r;
  const float m = -2048.0f;
  asm("v_fma_mixlo_f16 %0, %1, %2, %3 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, %2, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(hp), "s"(m), "v"(a0), "v"(a1));
  return r;
}
__device__ __forceinline__ void split_x3s(const f32x4 v, float sc, h16x4& h, h16x4& l) {
  typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
  const float c = pow2_mul(sc, 11);
  const uint32_t h01 = split_hi2s(v[0], v[1], sc);
  const uint32_t h23 = split_hi2s(v[2], v[3], sc);
  h = __builtin_bit_cast(h16x4, u32x2v{h01, h23});
  l = __builtin_bit_cast(h16x4, u32x2v{split_lo2s(h01, v[0] * c, v[1] * c), split_lo2s(h23, v[2] * c, v[3] * c)});
}

// One staging pass of A operands: `f(split)` stores the pass's rows through `split(v, h, l)`,
// instantiated twice behind one uniform branch -- the plain split while the range word is clear
// (sc == 1: the VALU count of the unscaled kernels; the folded scaled split costs one more VALU
// per value pair, measured +25 % on the VALU-bound 128x128 tiles), the scaled one otherwise.
template <class F>
__device__ __forceinline__ void split_pass(float sc, F&& f) {
  if (sc == 1.0f) f([](const f32x4& v, h16x4& h, h16x4& l) { split_x3(v, h, l); });
  else f([sc](const f32x4& v, h16x4& h, h16x4& l) { split_x3s(v, sc, h, l); });
}

// Output store of the fused blocks' conv3 (res2block*.hip).  SPK_NT_STORE=1 (experiment
// builds): non-temporal, so the block's output does not displace its input halo from L2.
#ifndef SPK_NT_STORE
#define SPK_NT_STORE 0
#endif
__device__ __forceinline__ void block_store(f32x4* p, const f32x4& v) {
#if SPK_NT_STORE
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One output element of the fused epilogue (everything after the K reduction).
__device__ __forceinline__ float epilogue_elem(const ConvDesc& d, int m, int n, float v) {
  if (d.bias) v += d.bias[n];
  if (d.rowbias) v += d.rowbias[(size_t)(m / (d.Ho * d.Wo)) * d.rowbias_ld + n];
  if (d.res) v += d.res[(size_t)m * d.ldr + n];
  if (d.affx) {
    const float t = 1.0f + tanhf(v);   // (scalar fallback: split-K reduce)
    return d.affx[(size_t)m * d.ldx + n] * t + d.affy[(size_t)m * d.ldy + n] * (2.0f - t);
  }
  v = apply_act(v, d.act);
  if (d.post_scale) v = v * d.post_scale[n] + d.post_shift[n];
  v = apply_act(v, d.act2);
  if (d.gate) {
    const int wo = m % d.Wo;
    const int img = m / (d.Wo * d.Ho);
    v *= d.gate[((size_t)img * d.gate_nseg + wo / d.gate_seg) * d.gate_ld + n];
  }
  return row_masked(d, m) ? 0.f : v;
}


// Runs the fused epilogue for a wave's TM x TN accumulator tiles (32x32 each, MFMA C
// layout).  `lds` must have TM*TN*1024 floats per wave free (all waves synchronised before
// the call); `nwave` is the first output column of the wave; rowmap(r) gives the output
// row m of the wave's local row r (0 .. 32*TM-1), or -1 when it is outside the output.
// LEAN = true compiles only the common-case path (bias / residual / act / post-affine,
// float4-aligned, no split-K); the caller guarantees those conditions on the host.
// `pre_bias` (optional, fast path): the lane's bias quads per tile, loaded by the caller
// ahead of time.  A persistent kernel with the next tile's loads in flight must pass it:
// vmcnt retires loads in order, so a bias load issued here would wait for all of them.
// PLAIN = true (implies LEAN): bias + activations only -- no residual, post-affine or
// ragged-row mask, i.e. no global load at all.  A persistent kernel with the next tile's
// loads in flight needs this: a load that may be issued here (even behind a branch the
// layer never takes) forces waits for everything issued before it (vmcnt counts in order).
// WIDE = true lets a wave with four accumulator tiles (the LDS-DMA GEMM's 32 x 128) take the
// one-round-trip paths too (16 residual / AFF quads in flight).
// `hook` (persistent GEMM): called once the epilogue's own global loads are all issued (fast
// paths) or done (the others), so loads it issues -- the next tile's first K-tiles -- are in
// flight during the epilogue without delaying its waits (vmcnt retires loads in order).
struct NoHook {
  __device__ void operator()() const {}
};
// L16 = true: each 32x32 tile holds four 16x16x32-MFMA accumulators (quadrant q = 2 a + b at
// elements 4 q .. 4 q + 3: row 16 a + 4 (lane >> 4) + e, column 16 b + (lane & 15)); the slab
// rows are then padded to 36 floats (the four lane groups of a store land 144 floats apart:
// distinct banks, where 128 apart would be a 4-way conflict).  epi_slab_floats() sizes it.
template <bool L16>
__host__ __device__ constexpr int epi_srow() { return L16 ? 36 : 32; }
template <bool L16>
__host__ __device__ constexpr int epi_slab_floats() { return 32 * epi_srow<L16>(); }
template <int TM, int TN, bool LEAN = false, bool PLAIN = false, bool WIDE = false, bool L16 = false, class RowMap,
          class Hook = NoHook>
__device__ __forceinline__ void epilogue_tiles(const ConvDesc& d, float* lds, f32x16 (&acc)[TM][TN], int wave,
                                               int lane, int nwave, int M, RowMap rowmap,
                                               const f32x4* pre_bias = nullptr, Hook hook = Hook{}) {
  const int li = lane & 31, lh = lane >> 5;
  constexpr int SROW = epi_srow<L16>(), SLAB = epi_slab_floats<L16>();
  // one 32x32 accumulator tile at a time through a per-wave LDS slab:
  // registers -> LDS in the MFMA C layout (col = lane&31, row = (r&3)+8(r>>2)+4(lane>>5)),
  // then each lane owns 4 consecutive columns of 4 rows (8 lanes = one 128-B output row):
  // every epilogue operand (residual, AFF inputs, bias, ...) is read as float4 and all of a
  // tile's loads are issued before the first use, so the fused epilogue costs one memory
  // round trip per tile instead of sixteen dependent scalar ones.
  // all of the wave's accumulators go to LDS first, so they are dead during the epilogue
  float* cw = lds + wave * (TM * TN * SLAB);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if constexpr (L16)
          cw[(i * TN + j) * SLAB + (16 * (r >> 3) + 4 * (lane >> 4) + (r & 3)) * SROW + 16 * ((r >> 2) & 1) + (lane & 15)] =
              acc[i][j][r];
        else
          cw[(i * TN + j) * SLAB + ((r & 3) + 8 * (r >> 2) + 4 * lh) * SROW + li] = acc[i][j][r];
      }
  wave_lds_sync();
  float* part = d.ksplit > 1 ? d.partial + (size_t)blockIdx.z * M * d.N : nullptr;
  const bool vec = (d.N % 4 == 0) && (d.ldo % 4 == 0) && (!d.res || d.ldr % 4 == 0) &&
                   (!d.affx || (d.ldx % 4 == 0 && d.ldy % 4 == 0)) && (!d.gate || d.gate_ld % 4 == 0) &&
                   (!d.rowbias || d.rowbias_ld % 4 == 0);
  // Common case (bias / residual / activations / post-affine only): every residual load of
  // the wave is issued before the first use, so the whole epilogue is one memory round trip.
  constexpr int NTL = TM * TN;
  float amax = 0.f;                            // range guard (common.h)
  if constexpr (NTL <= 2 || (WIDE && NTL <= 4)) {
    if (LEAN || PLAIN || (vec && !part && !d.affx && !d.gate && !d.rowbias)) {
      const int c4 = (lane & 7) * 4;
      f32x4 ra4[NTL][4], bias4[NTL], ps4[NTL], pt4[NTL];
#pragma unroll
      for (int tile = 0; tile < NTL; ++tile) {
        const int i = tile / TN, j = tile % TN;
        const int n = nwave + j * 32 + c4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          ra4[tile][q] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (!PLAIN && d.res && n < d.N) {
            const int m = max(0, min(rowmap(i * 32 + q * 8 + (lane >> 3)), M - 1));
            ra4[tile][q] = *reinterpret_cast<const f32x4*>(d.res + (size_t)m * d.ldr + n);
          }
        }
        // per-channel operands requested with the residual: one round trip for all of them
        bias4[tile] = f32x4{0.f, 0.f, 0.f, 0.f};
        ps4[tile] = f32x4{1.f, 1.f, 1.f, 1.f};
        pt4[tile] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (!PLAIN) {
          const int nn = n < d.N ? n : 0;
          if (pre_bias) bias4[tile] = pre_bias[tile];
          else if (d.bias) bias4[tile] = *reinterpret_cast<const f32x4*>(d.bias + nn);
          if (d.post_scale) {
            ps4[tile] = *reinterpret_cast<const f32x4*>(d.post_scale + nn);
            pt4[tile] = *reinterpret_cast<const f32x4*>(d.post_shift + nn);
          }
        }
      }
      hook();
#pragma unroll
      for (int tile = 0; tile < NTL; ++tile) {
        const int i = tile / TN, j = tile % TN;
        const int n = nwave + j * 32 + c4;
        if constexpr (PLAIN) {
          // No global load here at all (a load that may be issued, even behind a branch the
          // layer never takes, makes the compiler wait vmcnt(0) -- for every load issued
          // before it, i.e. the next tile's prefetch); all four rows are computed first and
          // stored back to back from distinct registers.
          const f32x4 bias = pre_bias[tile];
          const float* ct = cw + tile * SLAB;
          float* const ocol = d.out + n;
          f32x4 o[4];
          int mq[4];
          // the layer's activation resolved once per tile (compile-time forms for the common ones)
          auto act_rows = [&](auto actc) {
            constexpr int A = decltype(actc)::value;   // -1: general
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int rl = q * 8 + (lane >> 3);
              mq[q] = rowmap(i * 32 + rl);
              o[q] = *reinterpret_cast<const f32x4*>(ct + rl * SROW + c4) + bias;
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
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool ok = n < d.N && mq[q] >= 0 && mq[q] < M;
            if (ok) {
              amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[q][0]), fabsf(o[q][1])), fmaxf(fabsf(o[q][2]), fabsf(o[q][3]))));
              *reinterpret_cast<f32x4*>(ocol + (size_t)mq[q] * d.ldo) = o[q];
            }
          }
          continue;
        }
        if (n >= d.N) continue;
        float* const ocol = out_at(d, 0, n);   // plane / column split once per tile, not per row
        const f32x4 bias = bias4[tile], ps = ps4[tile], pt = pt4[tile];
        const float* ct = cw + tile * SLAB;
        // the rows of a tile with the layer's activation resolved once (not per element): the
        // common forms (one activation, no post-affine, no ragged mask) as compile-time
        // variants, everything else through the general form
        auto rows = [&](auto actc) {
          constexpr int A = decltype(actc)::value;   // -1: general
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int rl = q * 8 + (lane >> 3);
            const int m = rowmap(i * 32 + rl);
            if (m < 0 || m >= M) continue;
            f32x4 o = *reinterpret_cast<const f32x4*>(ct + rl * SROW + c4) + bias + ra4[tile][q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if constexpr (A >= 0) {
                o[e] = apply_act(o[e], A);
              } else {
                float x = apply_act(o[e], d.act);
                if (!PLAIN && d.post_scale) x = x * ps[e] + pt[e];
                o[e] = apply_act(x, d.act2);
              }
            }
            if constexpr (A < 0) {
              if (!PLAIN && row_masked(d, m)) o = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
            *reinterpret_cast<f32x4*>(ocol + (size_t)m * d.ldo) = o;
          }
        };
        const bool simple = !d.post_scale && d.act2 == ACT_NONE && !d.rowlen;
        if (simple && d.act == ACT_HTANH) rows(std::integral_constant<int, ACT_HTANH>{});
        else if (simple && d.act == ACT_RELU) rows(std::integral_constant<int, ACT_RELU>{});
        else if (simple && d.act == ACT_NONE) rows(std::integral_constant<int, ACT_NONE>{});
        else rows(std::integral_constant<int, -1>{});
      }
      range_note(d.range_flag, amax);
      return;
    }
    // AFF second conv (fusion.py:26-28): x*(1+tanh v) + y*(1-tanh v) replaces the
    // activations; both operands of every row of the wave are in flight before first use.
    if (!LEAN && vec && !part && d.affx && !d.res && !d.gate && !d.rowbias) {
      const int c4 = (lane & 7) * 4;
      f32x4 xa[NTL][4], ya[NTL][4];
#pragma unroll
      for (int tile = 0; tile < NTL; ++tile) {
        const int i = tile / TN, j = tile % TN;
        const int n = nwave + j * 32 + c4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          xa[tile][q] = f32x4{0.f, 0.f, 0.f, 0.f};
          ya[tile][q] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (n < d.N) {
            const int m = max(0, min(rowmap(i * 32 + q * 8 + (lane >> 3)), M - 1));
            xa[tile][q] = *reinterpret_cast<const f32x4*>(d.affx + (size_t)m * d.ldx + n);
            ya[tile][q] = *reinterpret_cast<const f32x4*>(d.affy + (size_t)m * d.ldy + n);
          }
        }
      }
      hook();   // (its bias loads below then wait for the hook's loads: no persistent grid here)
#pragma unroll
      for (int tile = 0; tile < NTL; ++tile) {
        const int i = tile / TN, j = tile % TN;
        const int n = nwave + j * 32 + c4;
        if (n >= d.N) continue;
        float* const ocol = out_at(d, 0, n);
        f32x4 bias = {0.f, 0.f, 0.f, 0.f};
        if (d.bias) bias = *reinterpret_cast<const f32x4*>(d.bias + n);
        const float* ct = cw + tile * SLAB;
        if constexpr (PLAIN) {
          // all four rows computed first, then four back-to-back stores from distinct
          // registers: a store whose source registers are reused right away makes the
          // compiler wait for it (vmcnt(0)), i.e. for every load issued before it
          f32x4 o[4];
          int mq[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int rl = q * 8 + (lane >> 3);
            mq[q] = rowmap(i * 32 + rl);
            o[q] = *reinterpret_cast<const f32x4*>(ct + rl * SROW + c4) + bias;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[q][e] = apply_act(apply_act(o[q][e], d.act), d.act2);
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[q][0]), fabsf(o[q][1])), fmaxf(fabsf(o[q][2]), fabsf(o[q][3]))));
          }
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (mq[q] >= 0 && mq[q] < M) *reinterpret_cast<f32x4*>(ocol + (size_t)mq[q] * d.ldo) = o[q];
          continue;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = q * 8 + (lane >> 3);
          const int m = rowmap(i * 32 + rl);
          if (m < 0 || m >= M) continue;
          f32x4 o = *reinterpret_cast<const f32x4*>(ct + rl * SROW + c4) + bias;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = aff_combine(o[e], xa[tile][q][e], ya[tile][q][e]);
          }
          if (row_masked(d, m)) o = f32x4{0.f, 0.f, 0.f, 0.f};
          amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
          *reinterpret_cast<f32x4*>(ocol + (size_t)m * d.ldo) = o;
        }
      }
      range_note(d.range_flag, amax);
      return;
    }
  }
  if constexpr (LEAN || PLAIN) {
    hook();
    return;
  }
#pragma unroll 1
  for (int tile = 0; tile < TM * TN; ++tile) {
    {
      const int i = tile / TN, j = tile % TN;
      const float* ct = cw + tile * SLAB;
      const int nbase = nwave + j * 32;
      if (vec) {
        const int c4 = (lane & 7) * 4;
        const int n = nbase + c4;
        float* const ocol = out_at(d, 0, n < d.N ? n : 0);
        f32x4 bias = {0.f, 0.f, 0.f, 0.f}, ps = {1.f, 1.f, 1.f, 1.f}, pt = {0.f, 0.f, 0.f, 0.f};
        if (!part && n < d.N) {
          if (d.bias) bias = *reinterpret_cast<const f32x4*>(d.bias + n);
          if (d.post_scale) {
            ps = *reinterpret_cast<const f32x4*>(d.post_scale + n);
            pt = *reinterpret_cast<const f32x4*>(d.post_shift + n);
          }
        }
        // two passes of two rows: operand loads of a pass are all in flight before use
#pragma unroll 1
        for (int half = 0; half < 2; ++half) {
          f32x4 v[2], ra4[2], xa4[2], ya4[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int rl = (half * 2 + q) * 8 + (lane >> 3);
            v[q] = *reinterpret_cast<const f32x4*>(ct + rl * SROW + c4);
            if (!part && n < d.N) {
              const int m = max(0, min(rowmap(i * 32 + rl), M - 1));
              if (d.res) ra4[q] = *reinterpret_cast<const f32x4*>(d.res + (size_t)m * d.ldr + n);
              if (d.affx) {
                xa4[q] = *reinterpret_cast<const f32x4*>(d.affx + (size_t)m * d.ldx + n);
                ya4[q] = *reinterpret_cast<const f32x4*>(d.affy + (size_t)m * d.ldy + n);
              }
            }
          }
          if (n >= d.N) continue;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int m = rowmap(i * 32 + (half * 2 + q) * 8 + (lane >> 3));
            if (m < 0 || m >= M) continue;
            if (part) {
              *reinterpret_cast<f32x4*>(part + (size_t)m * d.N + n) = v[q];
              continue;
            }
            f32x4 o = v[q] + bias;
            if (d.rowbias) o += *reinterpret_cast<const f32x4*>(d.rowbias + (size_t)(m / (d.Ho * d.Wo)) * d.rowbias_ld + n);
            if (d.res) o += ra4[q];
            if (d.affx) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                o[e] = aff_combine(o[e], xa4[q][e], ya4[q][e]);
              }
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                float x = apply_act(o[e], d.act);
                if (d.post_scale) x = x * ps[e] + pt[e];
                o[e] = apply_act(x, d.act2);
              }
              if (d.gate) {
                const int wo = m % d.Wo, img = m / (d.Wo * d.Ho);
                o *= *reinterpret_cast<const f32x4*>(d.gate + ((size_t)img * d.gate_nseg + wo / d.gate_seg) * d.gate_ld + n);
              }
            }
            if (row_masked(d, m)) o = f32x4{0.f, 0.f, 0.f, 0.f};
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3]))));
            *reinterpret_cast<f32x4*>(ocol + (size_t)m * d.ldo) = o;
          }
        }
      } else {
        const int n = nbase + li;
        float* const ocol = out_at(d, 0, n < d.N ? n : 0);
#pragma unroll 2
        for (int q = 0; q < 16; ++q) {
          const int rl = 2 * q + lh;
          const int m = rowmap(i * 32 + rl);
          if (m >= 0 && m < M && n < d.N) {
            const float v = ct[rl * SROW + li];
            if (part) {
              part[(size_t)m * d.N + n] = v;
            } else {
              const float o = epilogue_elem(d, m, n, v);
              amax = fmaxf(amax, fabsf(o));
              ocol[(size_t)m * d.ldo] = o;
            }
          }
        }
      }
    }
  }
  hook();   // the general path: its loads are all done
  range_note(d.range_flag, amax);
}

}  // namespace spk
