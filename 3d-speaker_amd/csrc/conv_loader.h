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
    if (k < K0) {
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
    if (in0) {
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

}  // namespace spk
