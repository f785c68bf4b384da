// Kaldi log-mel filterbank (torchaudio.compliance.kaldi.fbank defaults as called by
// speakerlab/process/processor.py:133-158), gfx950, computed in fp64 end to end.
//
// Why fp64: the features feed a ~60x input-sensitive network; an
// fp32 FFT leaves ~1e-6 relative noise on every bin, i.e. up to ~1e-3 in the log of the
// quiet bands, and that alone would use most of the 1e-4 embedding budget.  In fp64 the
// only fp32 roundings left are the input samples (exact) and the stored output.
//
// Grid: G four-wave workgroups per utterance (ragged batches via sample/frame offsets),
// then one mean-normalisation workgroup per utterance.  Each wave transforms TWO frames per FFT: z = a + i*b (a, b real windowed frames), one
// 512-point complex FFT, then A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i
// -- half the FFT work per frame.  The 512-point FFT is 8 x 8 x 8: three radix-8 DFTs in
// registers (each lane holds 8 complex doubles) with two LDS transposes between them, so
// the load layout (lane + 64 j, j = 0..7) is already the first pass's input layout and no
// bit reversal is needed.  Then |A|^2, |B|^2 -> sparse 80-band mel projection -> log(max(E,
// FLT_EPSILON)), all in double; the per-utterance mean over frames (processor.py:156-157)
// is a second kernel over the (L2-resident) fp32 rows, summed in double.
#include "common.h"
#include "fbank.h"

#include <algorithm>
#include <type_traits>

#ifndef SPK_FB_PROF
#define SPK_FB_PROF 0
#endif

namespace spk {

#if SPK_FB_PROF
// diagnostic build only (tools/fb_prof.py): per-wave cycle counts of the frames kernel's
// phases, lane 0 of every wave stores its own slot (vector stores)
constexpr int FBP_PH = 6, FBP_BLK = 8192;
__device__ long long fb_prof_buf[FBP_BLK * 4 * FBP_PH];
#define FB_STAMP(i) do { const long long now_ = __builtin_amdgcn_s_memtime(); tp[i] += now_ - tl; tl = now_; } while (0)
#else
#define FB_STAMP(i) do {} while (0)
#endif

namespace {

constexpr int NFFT = 512;
constexpr int FLEN = 400;
constexpr int FSHIFT = 160;
constexpr int WAVES = 4;

__device__ __forceinline__ int PADX(int e) { return e + (e >> 3); }

// DPP move of a double (two 32-bit moves); lanes without a source lane keep `old`
template <int CTRL, bool ZERO_OOB>
__device__ __forceinline__ double dpp_d(double old, double v) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, 0xf, 0xf, ZERO_OOB);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, 0xf, 0xf, ZERO_OOB);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}

// Wave sum in a fixed order: DPP butterflies inside each 16-lane row (xor 1, xor 2, half-row
// mirror, row mirror), then the four row sums
__device__ __forceinline__ double wave_sum_d(double v) {
  v += dpp_d<0xB1, true>(0.0, v);    // quad_perm [1,0,3,2]
  v += dpp_d<0x4E, true>(0.0, v);    // quad_perm [2,3,0,1]
  v += dpp_d<0x141, true>(0.0, v);   // row_half_mirror
  v += dpp_d<0x140, true>(0.0, v);   // row_mirror
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}

// x[lane - 1] (wave_shr:1); lane 0 gets `first`
__device__ __forceinline__ float prev_lane(float x, float first) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(first), __float_as_int(x), 0x138, 0xf, 0xf, false));
}

// log of a positive double, rounded to fp32: e = m 2^k with m in [1, 2) taken from the bits,
// log e = k ln 2 (double) + logf(m) (fp32: |error| < 1e-7 absolute on [0, ln 2)).  The result
// is stored as fp32, whose rounding (half an ulp, ~1e-6 at |log e| ~ 16) dominates; a double
// log costs about ten times the instructions and was the largest share of the kernel
__device__ __forceinline__ float log_d2f(double e) {
  const int hi = __double2hiint(e), lo = __double2loint(e);
  const int k = ((hi >> 20) & 0x7FF) - 1023;
  const double m = __hiloint2double((hi & 0x000FFFFF) | 0x3FF00000, lo);
  return (float)((double)k * 0.69314718055994530942 + (double)logf((float)m));
}

// LDS hand-off between lanes of one wave: order the memory ops, no cross-wave sync
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// (x + iy) * (c + is)
__device__ __forceinline__ void cmul(double& x, double& y, double c, double s) {
  const double r = x * c - y * s;
  y = x * s + y * c;
  x = r;
}

// In-place 8-point DFT X[k] = sum_n x[n] exp(-2 pi i n k / 8), natural order in and out.
__device__ __forceinline__ void dft8(double* re, double* im) {
  constexpr double C = 0.70710678118654752440;
  // even / odd 4-point DFTs
  double er[4], ei[4], orr[4], oi[4];
  {
    const double s0r = re[0] + re[4], s0i = im[0] + im[4], d0r = re[0] - re[4], d0i = im[0] - im[4];
    const double s1r = re[2] + re[6], s1i = im[2] + im[6], d1r = re[2] - re[6], d1i = im[2] - im[6];
    er[0] = s0r + s1r; ei[0] = s0i + s1i;
    er[2] = s0r - s1r; ei[2] = s0i - s1i;
    er[1] = d0r + d1i; ei[1] = d0i - d1r;     // d0 + (-i) d1
    er[3] = d0r - d1i; ei[3] = d0i + d1r;     // d0 - (-i) d1
  }
  {
    const double s0r = re[1] + re[5], s0i = im[1] + im[5], d0r = re[1] - re[5], d0i = im[1] - im[5];
    const double s1r = re[3] + re[7], s1i = im[3] + im[7], d1r = re[3] - re[7], d1i = im[3] - im[7];
    orr[0] = s0r + s1r; oi[0] = s0i + s1i;
    orr[2] = s0r - s1r; oi[2] = s0i - s1i;
    orr[1] = d0r + d1i; oi[1] = d0i - d1r;
    orr[3] = d0r - d1i; oi[3] = d0i + d1r;
  }
  // W8^k * O[k]: k=1 (C, -C), k=2 (0, -1), k=3 (-C, -C)
  double tr[4], ti[4];
  tr[0] = orr[0];                  ti[0] = oi[0];
  tr[1] = C * (orr[1] + oi[1]);    ti[1] = C * (oi[1] - orr[1]);
  tr[2] = oi[2];                   ti[2] = -orr[2];
  tr[3] = C * (oi[3] - orr[3]);    ti[3] = -C * (orr[3] + oi[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    re[k] = er[k] + tr[k];     im[k] = ei[k] + ti[k];
    re[k + 4] = er[k] - tr[k]; im[k + 4] = ei[k] - ti[k];
  }
}

// Frames kernel: WAVES-wave workgroups, G of them per utterance, each wave one pair of
// frames at a time.  Workgroup id -> (utterance, slice) is XCD-aware: all slices of
// utterance u run on XCD u % 8 (dispatch is round-robin over the 8 XCDs), which is also
// where fbank_cmn_kernel's workgroup u runs, so the rows it re-reads are in that XCD's L2.
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(4)))
fbank_frames_kernel(const float* __restrict__ wav, const int64_t* __restrict__ wav_off,
                    float* __restrict__ feats, const int64_t* __restrict__ frame_off,
                    const FbankTables* __restrict__ tab, int n_mels, int mel_nb, int t_max, int n_utt, int G) {
  // per-wave FFT transposes / power spectra, one pad entry after every 8 (PADX): the
  // stride-8 and stride-64 transposes then hit distinct banks in every 16-lane phase
  __shared__ double2 buf[WAVES][NFFT + NFFT / 8];

  const int id = blockIdx.x, slot = id >> 3;
  const int utt = (id & 7) + 8 * (slot / G), g = slot % G;
  if (utt >= n_utt) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* x = wav + wav_off[utt];
  const int nfr = (int)(frame_off[utt + 1] - frame_off[utt]);
  // packed (t_max == 0): rows at frame_off[utt]; padded: rows at utt * t_max, rows
  // [nfr, t_max) of the utterance zeroed
  const int64_t f0 = t_max > 0 ? (int64_t)utt * t_max : frame_off[utt];
  float* out = feats + f0 * n_mels;
  if (t_max > 0)
    for (int e = nfr * n_mels + g * blockDim.x + threadIdx.x; e < t_max * n_mels; e += G * blockDim.x) out[e] = 0.f;

  double2* wb = buf[wave];
  double* pw = reinterpret_cast<double*>(wb);     // aliases wb after the FFT: [2][256]
  const int hi = lane >> 3, lo = lane & 7;
  const int npairs = (nfr + 1) >> 1;
  const double2 tw1 = tab->twiddle[lane], tw2 = tab->twiddle[8 * lo];
  double win[8];   // this lane's window samples, pair-invariant
#pragma unroll
  for (int j = 0; j < 8; ++j) win[j] = lane + 64 * j < FLEN ? tab->window[lane + 64 * j] : 0.0;
#if SPK_FB_PROF
  long long tp[FBP_PH] = {0, 0, 0, 0, 0, 0};
  long long tl = __builtin_amdgcn_s_memtime();
#endif
  for (int p = g * WAVES + wave; p < npairs; p += G * WAVES) {
    const int fa = 2 * p;
    const bool hasb = fa + 1 < nfr;
    const float* sa = x + (int64_t)fa * FSHIFT;
    const float* sb = sa + FSHIFT;
    // 1) both windows (lane + 64 j, zero past 400) and their means
    float xa[8], xb[8];
    double re[8], im[8];
    double suma = 0.0, sumb = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      xa[j] = i < FLEN ? sa[i] : 0.f;
      xb[j] = (hasb && i < FLEN) ? sb[i] : 0.f;
      suma += (double)xa[j];
      sumb += (double)xb[j];
    }
    const double ma = wave_sum_d(suma) * (1.0 / FLEN), mb = wave_sum_d(sumb) * (1.0 / FLEN);
    FB_STAMP(0);
    // 2) DC removal, pre-emphasis (previous sample from the neighbouring lane by a DPP
    // wave shift, lane 0 from lane 63 of the previous slice; the first sample is
    // replicated), Povey window
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      const float fa_ = j > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(xa[j > 0 ? j - 1 : 0]), 63)) : xa[0];
      const float fb_ = j > 0 ? __builtin_bit_cast(float, __builtin_amdgcn_readlane(__float_as_int(xb[j > 0 ? j - 1 : 0]), 63)) : xb[0];
      const float pa_ = prev_lane(xa[j], fa_), pb_ = prev_lane(xb[j], fb_);
      re[j] = 0.0;
      im[j] = 0.0;
      if (i < FLEN) {
        const double w = win[j];
        re[j] = (((double)xa[j] - ma) - 0.97 * ((double)pa_ - ma)) * w;
        im[j] = hasb ? (((double)xb[j] - mb) - 0.97 * ((double)pb_ - mb)) * w : 0.0;
      }
    }
    FB_STAMP(1);
    // 3) FFT.  Pass 1: lane L = n mod 64 holds n1 = 0..7 (n = 64 n1 + L) -> k1, times W512^(L k1)
    dft8(re, im);
    {   // W512^(L k) as powers of W512^L (loaded once): k ulp of drift.  Recomputed every pair
        // (opaque base) rather than hoisted: 28 VGPRs of powers would cost a wave per SIMD
      double wr = tw1.x, wi = tw1.y;
      asm volatile("" : "+v"(wr), "+v"(wi));
      const double b1r = wr, b1i = wi;
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        cmul(re[k], im[k], wr, wi);
        if (k < 7) cmul(wr, wi, b1r, b1i);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[PADX(k * 64 + lane)] = make_double2(re[k], im[k]);
    wave_sync();
    // pass 2: lane = (k1 = hi, n3 = lo) holds n2 = 0..7 (L = 8 n2 + n3) -> k2, times W64^(n3 k2)
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const double2 v = wb[PADX(hi * 64 + 8 * n + lo)];
      re[n] = v.x;
      im[n] = v.y;
    }
    dft8(re, im);
    {
      double wr = tw2.x, wi = tw2.y;
      asm volatile("" : "+v"(wr), "+v"(wi));
      const double b2r = wr, b2i = wi;
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        cmul(re[k], im[k], wr, wi);
        if (k < 7) cmul(wr, wi, b2r, b2i);
      }
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[PADX(hi * 64 + 8 * k + lo)] = make_double2(re[k], im[k]);
    wave_sync();
    // pass 3: lane = (k1 = hi, k2 = lo) holds n3 = 0..7 -> k3; Z[k1 + 8 k2 + 64 k3]
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const double2 v = wb[PADX(hi * 64 + 8 * lo + n)];
      re[n] = v.x;
      im[n] = v.y;
    }
    dft8(re, im);
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[PADX(hi + 8 * lo + 64 * k)] = make_double2(re[k], im[k]);
    wave_sync();
    FB_STAMP(2);
    // 4) split the two real spectra and take the power of bins 0..255 (the Nyquist column
    // of the mel bank is zero)
    double pa[4], pb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = lane + 64 * j;
      const double2 z = wb[PADX(k)], zc = wb[PADX((NFFT - k) & (NFFT - 1))];
      const double ar = z.x + zc.x, ai = z.y - zc.y;     // 2 A[k]
      const double br = z.y + zc.y, bi = zc.x - z.x;     // 2 B[k]
      pa[j] = 0.25 * (ar * ar + ai * ai);
      pb[j] = 0.25 * (br * br + bi * bi);
    }
    wave_sync();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pw[lane + 64 * j] = pa[j];
      pw[256 + lane + 64 * j] = pb[j];
    }
    wave_sync();
    FB_STAMP(3);
    // 5) mel projection + log (double), store fp32.  Bands in blocks of 32: lanes 0-31 take
    // frame a, lanes 32-63 frame b of the same 32 bands, so each pass runs only as many
    // bins as the block's widest filter (narrow low bands first).
    float* oa = out + (int64_t)fa * n_mels;
    const int f = lane >> 5;
    const double* ps = pw + 256 * f;
    for (int blk = 0; 32 * blk < n_mels; ++blk) {
      const int m = 32 * blk + (lane & 31);
      const int nbk = tab->mel_blk_nb[blk];
      if (m < n_mels && (f == 0 || hasb)) {
        const double* wm = tab->mel_wt + m;
        const int b0 = tab->mel_start[m];
        // up to 16 independent loads in flight (nbk is wave-uniform); the zero-padded tail
        // adds +0.0 to the same running sum (bins clamped to 255: finite powers, 0 * p = 0)
        double e = 0.0;
        for (int t = 0; t < nbk; t += 16) {
          double w[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) w[u] = t + u < nbk ? wm[(t + u) * n_mels] : 0.0;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (t + u < nbk) e += ps[min(b0 + t + u, 255)] * w[u];
        }
        oa[f * n_mels + m] = log_d2f(fmax(e, 1.1920928955078125e-07));
      }
    }
    wave_sync();
    FB_STAMP(4);
  }
#if SPK_FB_PROF
  tp[5] = (npairs - (g * WAVES + wave) + G * WAVES - 1) / (G * WAVES);   // pairs this wave did
  if (lane == 0 && blockIdx.x < FBP_BLK)
    for (int i = 0; i < FBP_PH; ++i) fb_prof_buf[((size_t)blockIdx.x * WAVES + wave) * FBP_PH + i] = tp[i];
#endif
}

// Per-utterance mean normalisation (processor.py:156-157: feature - feature.mean(0)) over
// the fp32 rows fbank_frames_kernel wrote: column sums in double in a fixed order (row
// lanes, then a fixed-order LDS reduction), then x - mean rounded once.  One workgroup per
// utterance on XCD u % 8, where the rows still sit in L2.  Columns as float4 when n_mels %
// 4 == 0 (V = 4), else scalar.
template <int V>
__global__ void __launch_bounds__(1024)
fbank_cmn_kernel(float* __restrict__ feats, const int64_t* __restrict__ frame_off, int n_mels, int t_max) {
  __shared__ double red[1024 * V];
  __shared__ double mean[128];
  const int utt = blockIdx.x;
  const int nfr = (int)(frame_off[utt + 1] - frame_off[utt]);
  if (nfr <= 0) return;
  const int64_t f0 = t_max > 0 ? (int64_t)utt * t_max : frame_off[utt];
  float* out = feats + f0 * n_mels;
  const int nc = n_mels / V, rl_n = blockDim.x / nc;          // column groups, row lanes
  const int c = threadIdx.x % nc, rl = threadIdx.x / nc;
  const bool act = rl < rl_n;
  using VT = typename std::conditional<V == 4, float4, float>::type;
  auto ld = [&](int r, double* s) {
    const VT q = *reinterpret_cast<const VT*>(out + (int64_t)r * n_mels + c * V);
    if constexpr (V == 4) { s[0] += q.x; s[1] += q.y; s[2] += q.z; s[3] += q.w; } else { s[0] += q; }
  };
  double s[V];
#pragma unroll
  for (int v = 0; v < V; ++v) s[v] = 0.0;
  if (act) {
    int r = rl;
    for (; r + 3 * rl_n < nfr; r += 4 * rl_n) {   // four independent row loads in flight
      ld(r, s); ld(r + rl_n, s); ld(r + 2 * rl_n, s); ld(r + 3 * rl_n, s);
    }
    for (; r < nfr; r += rl_n) ld(r, s);
#pragma unroll
    for (int v = 0; v < V; ++v) red[rl * n_mels + c * V + v] = s[v];
  }
  __syncthreads();
  for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
    double t = 0.0;
    for (int r = 0; r < rl_n; ++r) t += red[r * n_mels + m];
    mean[m] = t / (double)nfr;
  }
  __syncthreads();
  if (!act) return;
  double mu[V];
#pragma unroll
  for (int v = 0; v < V; ++v) mu[v] = mean[c * V + v];
#pragma unroll 4
  for (int r = rl; r < nfr; r += rl_n) {
    VT* dst = reinterpret_cast<VT*>(out + (int64_t)r * n_mels + c * V);
    VT q = *dst;
    if constexpr (V == 4) {
      q.x = (float)((double)q.x - mu[0]);
      q.y = (float)((double)q.y - mu[1]);
      q.z = (float)((double)q.z - mu[2]);
      q.w = (float)((double)q.w - mu[3]);
    } else {
      q = (float)((double)q - mu[0]);
    }
    *dst = q;
  }
}

}  // namespace

hipError_t launch_fbank(const float* wav, const int64_t* wav_off, int n_utt, float* feats,
                        const int64_t* frame_off, int n_mels, int mean_nor, const FbankTables* tab,
                        int mel_nb, hipStream_t s, int t_max) {
  if (n_mels <= 0 || n_mels > 128 || n_utt < 0 || t_max < 0 || mel_nb <= 0 || mel_nb % 16) return hipErrorInvalidValue;
  if (n_utt == 0) return hipSuccess;
  // slices per utterance: about 16k waves in the grid (4 per SIMD of 4 x 256), at least one
  // workgroup per utterance, at most 64 (a 5 s utterance has 249 frame pairs)
  const int G = std::max(1, std::min(64, 16384 / (WAVES * n_utt)));
  const int groups = (n_utt + 7) / 8;
  hipLaunchKernelGGL(fbank_frames_kernel, dim3(8 * G * groups), dim3(64 * WAVES), 0, s, wav, wav_off, feats,
                     frame_off, tab, n_mels, mel_nb, t_max, n_utt, G);
  if (hipError_t e = hipGetLastError(); e != hipSuccess || !mean_nor) return e;
  if (n_mels % 4 == 0)
    hipLaunchKernelGGL(fbank_cmn_kernel<4>, dim3(n_utt), dim3(1024), 0, s, feats, frame_off, n_mels, t_max);
  else
    hipLaunchKernelGGL(fbank_cmn_kernel<1>, dim3(n_utt), dim3(1024), 0, s, feats, frame_off, n_mels, t_max);
  return hipGetLastError();
}

#if SPK_FB_PROF
extern "C" int spk_exp_fb_prof(long long* host, size_t n) {
  const size_t all = sizeof(spk::fb_prof_buf) / sizeof(long long);
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(spk::fb_prof_buf), std::min(n, all) * sizeof(long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

}  // namespace spk
