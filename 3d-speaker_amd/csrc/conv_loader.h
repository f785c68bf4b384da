// Implicit-im2col A-operand loader shared by the conv GEMM kernels (conv_gemm.hip).
//
// The loader is split into an issue half (`load`) and a consume half (`value`) so that the
// global loads of a K-tile stay in flight across the MFMAs of the previous tile: every load
// is unconditional (out-of-image taps, rows past M and K beyond the operands read a valid
// dummy address) and the zero-padding / Res2Net addend / CAM++ BN-ReLU are applied at
// consume time from a per-row mask.  A load guarded by a lane-divergent `if` would make the
// compiler wait for it right there (s_waitcnt vmcnt(0) at the branch merge), serialising
// the tile loads with the compute.
#pragma once
#include "common.h"
#include "conv_epilogue.h"

namespace spk {

// One thread's share of a BM x BK A tile: AROWS rows (RPP apart) x one float4 of k.
template <int AROWS, int RPP, int BK, bool S1, bool ADD, bool PRE>
struct ALoader {
  struct Slot {
    f32x4 v[AROWS];
    f32x4 v2[ADD ? AROWS : 1];
    f32x4 psc, psh;  // PRE: the BN-ReLU pre-activation of this thread's 4 channels
    unsigned ok;     // bit r: row r holds a real operand value (else zero)
    int pre;         // PRE: the K-tile lies in s0 (the pre-activation applies)
  };
  int img[AROWS], hb[AROWS], wb[AROWS], h1[AROWS], w1[AROWS];
  unsigned rok;
  int k_c, k_ky, k_kx;

  __device__ __forceinline__ void init(const ConvDesc& d, int m0, int row0, int kq, int kt0) {
    const int M = d.nimg * d.Ho * d.Wo;
    rok = 0;
#pragma unroll
    for (int r = 0; r < AROWS; ++r) {
      const int m = m0 + row0 + RPP * r;
      if (m < M) rok |= 1u << r;
      const int mm = m < M ? m : 0;
      const int wo = mm % d.Wo;
      const int t2 = mm / d.Wo;
      const int ho = t2 % d.Ho;
      img[r] = t2 / d.Ho;
      hb[r] = ho * d.s0.sh - d.s0.ph;
      wb[r] = wo * d.s0.sw - d.s0.pw;
      if (S1) { h1[r] = ho * d.s1.sh; w1[r] = wo * d.s1.sw; }
    }
    const int K0 = d.s0.kh * d.s0.kw * d.s0.cin;
    const int k = kt0 * BK + kq * 4;
    if (d.kcb) {   // channel-block-major K (common.h ConvDesc::kcb; BK == 32, checked on the host)
      const int taps = d.s0.kh * d.s0.kw;
      const int tap = kt0 % taps;
      k_c = (kt0 / taps) * BK + kq * 4;
      k_ky = k_c < d.s0.cin ? tap / d.s0.kw : d.s0.kh;
      k_kx = tap % d.s0.kw;
    } else if (k < K0) {
      const int tap = k / d.s0.cin;
      k_c = k - tap * d.s0.cin;
      k_ky = tap / d.s0.kw;
      k_kx = tap - k_ky * d.s0.kw;
    } else {
      k_ky = d.s0.kh; k_kx = 0; k_c = k - K0;   // in s1 (or beyond K)
    }
  }

  // issue the loads of the current K-tile into `s`, then advance (tap, c) by BK
  __device__ __forceinline__ void load(const ConvDesc& d, Slot& s) {
    const bool in0 = k_ky < d.s0.kh;
    const bool in1 = S1 && !in0 && k_c < d.s1.cin;
    if (PRE) {
      const int c = in0 ? k_c : 0;
      s.pre = in0;
      s.psc = *reinterpret_cast<const f32x4*>(d.s0.pre_scale + c);
      s.psh = *reinterpret_cast<const f32x4*>(d.s0.pre_shift + c);
    }
    s.ok = 0;
#pragma unroll
    for (int r = 0; r < AROWS; ++r) {
      int hi = hb[r] + k_ky * d.s0.dh;
      int wi = wb[r] + k_kx * d.s0.dw;
      if (d.s0.reflect) {
        hi = hi < 0 ? -hi : (hi >= d.s0.H ? 2 * d.s0.H - 2 - hi : hi);
        wi = wi < 0 ? -wi : (wi >= d.s0.W ? 2 * d.s0.W - 2 - wi : wi);
      }
      const bool ok0 = in0 && ((rok >> r) & 1) && hi >= 0 && hi < d.s0.H && wi >= 0 && wi < d.s0.W &&
                       (!d.s0.vlen || wi < d.s0.vlen[img[r]]);
      const bool ok1 = in1 && ((rok >> r) & 1);
      // offsets computed unconditionally and selected (branch-free)
      const long long pix0 = (long long)(img[r] * d.s0.H + hi) * d.s0.W + wi;
      const long long o0 = pix0 * d.s0.ld + k_c;
      long long off = ok0 ? o0 : 0;
      const float* base = d.s0.p;
      if (S1) {
        const long long o1 = ((long long)(img[r] * d.s1.H + h1[r]) * d.s1.W + w1[r]) * d.s1.ld + k_c;
        off = ok1 ? o1 : off;
        base = ok1 ? d.s1.p : base;
      }
      s.v[r] = *reinterpret_cast<const f32x4*>(base + off);
      if (ADD) {
        const long long o2 = ok0 ? pix0 * d.s0.ld2 + k_c : 0;
        s.v2[r] = *reinterpret_cast<const f32x4*>(d.s0.p2 + o2);
      }
      s.ok |= (ok0 || ok1) ? (1u << r) : 0u;
    }
    if (d.kcb) {   // next tap of the channel block; after its last tap the next block
      if (in0) {
        if (++k_kx == d.s0.kw) { k_kx = 0; ++k_ky; }
        if (k_ky == d.s0.kh) {
          k_c += BK;
          if (k_c < d.s0.cin) k_ky = 0;
        }
      }
    } else if (in0) {
      k_c += BK;
      while (k_c >= d.s0.cin && k_ky < d.s0.kh) {
        k_c -= d.s0.cin;
        if (++k_kx == d.s0.kw) { k_kx = 0; ++k_ky; }
      }
    } else {
      k_c += BK;
    }
  }

  // the operand value of row r (waits for that row's load)
  __device__ __forceinline__ f32x4 value(const Slot& s, int r) const {
    f32x4 v = s.v[r];
    if (ADD) v += s.v2[r];
    if (PRE && s.pre) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = fmaxf(fmaf(v[q], s.psc[q], s.psh[q]), 0.f);
    }
    const bool ok = (s.ok >> r) & 1;
    return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
};

// ---------------------------------------------------------------------------------------
// Buffer-resource form of the loader (the common case: zero padding, s0.cin >= BK,
// kh*kw <= 30 taps).  Everything that does not change along K is folded into per-row
// constants at init: the row's byte offset (relative to a block-uniform image base, so
// 32-bit offsets cover any batch) and a bit mask of the taps that land inside the image
// (and inside the utterance for ragged batches).  Per K-tile a row then costs one add and
// one mask test; an out-of-image tap gets an offset past the resource's range, which the
// buffer unit answers with zeros -- no select on the loaded value, no 64-bit address math.
// The tap walk (t, kx, pixel delta) is per thread because a 32-deep K-tile may straddle
// two taps when cin is not a multiple of 32 (ERes2NetV2 widths 104 / 208).
constexpr uint32_t BUF_RANGE = 0x7FFFFFF0u;   // resource size: every valid offset is below it
constexpr uint32_t BUF_OOB = 0x80000000u;     // an offset the buffer unit answers with zeros

// raw buffer resource on p (wave-uniform: built from readfirstlane'd halves, T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)BUF_RANGE, 0x00020000);
}

__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t r, uint32_t off, int soff = 0) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, soff, 0));
}

template <int AROWS, int RPP, int BK, bool S1, bool ADD, bool PRE>
struct BufALoader {
  struct Slot {
    f32x4 v[AROWS];
    f32x4 v2[(ADD || S1) ? AROWS : 1];   // Res2Net addend, or the K-concatenated s1 operand
    f32x4 psc, psh;
    unsigned ok;                         // PRE only: bit r = row r in bounds
    int pre;
  };
  __amdgpu_buffer_rsrc_t r0, r2, r1;
  uint32_t roff[AROWS], roff2[ADD ? AROWS : 1], roff1[S1 ? AROWS : 1];
  uint32_t rmask[AROWS];   // bit t: tap t in bounds; bit 31: row < M
  int wbr[AROWS];          // reflect padding (1-D, H = 1): the row's first tap column
  int c, t, kx, tdp;       // this thread's quad: channel within tap, tap, tap column, tap pixel delta

  __device__ __forceinline__ void init(const ConvDesc& d, int m0, int row0, int kq, int kt0) {
    const int M = d.nimg * d.Ho * d.Wo;
    const int img0 = m0 / (d.Ho * d.Wo);
    const size_t img_px = (size_t)d.s0.H * d.s0.W;
    r0 = make_rsrc(d.s0.p + (size_t)img0 * img_px * d.s0.ld);
    if (ADD) r2 = make_rsrc(d.s0.p2 + (size_t)img0 * img_px * d.s0.ld2);
    if (S1) r1 = make_rsrc(d.s1.p + (size_t)img0 * d.s1.H * d.s1.W * d.s1.ld);
#pragma unroll
    for (int r = 0; r < AROWS; ++r) {
      const int m = m0 + row0 + RPP * r;
      const bool valid = m < M;
      const int mm = valid ? m : m0;
      const int wo = mm % d.Wo;
      const int t2 = mm / d.Wo;
      const int ho = t2 % d.Ho;
      const int img = t2 / d.Ho;
      const int hb = ho * d.s0.sh - d.s0.ph, wb = wo * d.s0.sw - d.s0.pw;
      const int li = img - img0;
      const int pix = (li * d.s0.H + hb) * d.s0.W + wb;   // may be negative: masked
      roff[r] = (uint32_t)pix * (uint32_t)d.s0.ld * 4u;
      if (ADD) roff2[r] = (uint32_t)pix * (uint32_t)d.s0.ld2 * 4u;
      if (S1)
        roff1[r] = (uint32_t)(((li * d.s1.H + ho * d.s1.sh) * d.s1.W + wo * d.s1.sw) * d.s1.ld) * 4u;
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
      // reflect padding (conv_buf_loader_ok: H = 1, kh = 1, no ragged rows): every tap reads
      // a pixel of the row's image, the out-of-range ones mirrored at load time
      if (d.s0.reflect) mk = (1u << d.s0.kw) - 1u;
      wbr[r] = wb;
      rmask[r] = valid ? (mk | 0x80000000u) : 0u;
    }
    const int taps = d.s0.kh * d.s0.kw;
    const int K0 = taps * d.s0.cin;
    const int k = kt0 * BK + kq * 4;
    if (d.kcb) {   // channel-block-major K (common.h ConvDesc::kcb): t is the same in every lane
      c = (kt0 / taps) * BK + kq * 4;
      t = c < d.s0.cin ? kt0 % taps : taps;
    } else if (k < K0) {
      t = k / d.s0.cin;
      c = k - t * d.s0.cin;
    } else {
      t = taps;
      c = k - K0;
    }
    const int ky = t / d.s0.kw;
    kx = t - ky * d.s0.kw;
    tdp = ky * d.s0.dh * d.s0.W + kx * d.s0.dw;
  }

  // issue the loads of the current K-tile into `s`, then advance (tap, c) by BK
  __device__ __forceinline__ void load(const ConvDesc& d, Slot& s) {
    const int taps = d.s0.kh * d.s0.kw;
    const uint32_t toff = (uint32_t)(tdp * d.s0.ld + c) * 4u;
    const uint32_t toff2 = ADD ? (uint32_t)(tdp * d.s0.ld2 + c) * 4u : 0u;
    const bool in1 = S1 && t == taps && c < d.s1.cin;
    if (PRE) {
      const int cc = t < taps ? c : 0;
      s.pre = t < taps;
      s.psc = *reinterpret_cast<const f32x4*>(d.s0.pre_scale + cc);
      s.psh = *reinterpret_cast<const f32x4*>(d.s0.pre_shift + cc);
    }
    unsigned ok = 0;
#pragma unroll
    for (int r = 0; r < AROWS; ++r) {
      const bool b = (rmask[r] >> t) & 1u;   // t <= taps <= 30: never the row bit
      uint32_t o0 = roff[r] + toff, o2 = ADD ? roff2[r] + toff2 : 0u;
      if (d.s0.reflect) {                    // mirrored column (selects, no branch around a load)
        int wi = wbr[r] + kx * d.s0.dw;
        wi = wi < 0 ? -wi : (wi >= d.s0.W ? 2 * d.s0.W - 2 - wi : wi);
        const int dpx = wi - wbr[r];
        o0 = roff[r] + (uint32_t)(dpx * d.s0.ld + c) * 4u;
        if (ADD) o2 = roff2[r] + (uint32_t)(dpx * d.s0.ld2 + c) * 4u;
      }
      s.v[r] = buf_load4(r0, b ? o0 : BUF_OOB);
      if (ADD) s.v2[r] = buf_load4(r2, b ? o2 : BUF_OOB);
      if (S1) s.v2[r] = buf_load4(r1, (in1 && (rmask[r] >> 31)) ? roff1[r] + (uint32_t)c * 4u : BUF_OOB);
      if (PRE) ok |= (unsigned)b << r;
    }
    s.ok = ok;
    advance(d);
  }

  // (tap, c) of the next K-tile
  __device__ __forceinline__ void advance(const ConvDesc& d) {
    const int taps = d.s0.kh * d.s0.kw;
    if (d.kcb) {   // next tap of the channel block (uniform); after its last tap the next block
      if (t < taps) {
        ++t;
        ++kx;
        tdp += d.s0.dw;
        if (kx == d.s0.kw) {
          kx = 0;
          tdp += d.s0.dh * d.s0.W - d.s0.kw * d.s0.dw;
        }
        if (t == taps) {
          c += BK;
          if (c < d.s0.cin) { t = 0; kx = 0; tdp = 0; }   // past the last block t stays at taps: zeros
        }
      }
      return;
    }
    c += BK;
    if (t < taps && c >= d.s0.cin) {   // cin >= BK: at most one tap boundary per K-tile
      c -= d.s0.cin;
      ++t;
      ++kx;
      tdp += d.s0.dw;
      if (kx == d.s0.kw) {
        kx = 0;
        tdp += d.s0.dh * d.s0.W - d.s0.kw * d.s0.dw;
      }
    }
  }

  __device__ __forceinline__ f32x4 value(const Slot& s, int r) const {
    f32x4 v = s.v[r];
    if (ADD || S1) v += s.v2[r];
    if (PRE) {
      if (s.pre) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = fmaxf(fmaf(v[q], s.psc[q], s.psh[q]), 0.f);
      }
      v = ((s.ok >> r) & 1) ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    return v;
  }
};

}  // namespace spk
