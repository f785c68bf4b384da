// Kaldi log-mel filterbank (torchaudio.compliance.kaldi.fbank defaults as called by
// speakerlab/process/processor.py:133-158), gfx950, computed in fp64 end to end.
//
// Why fp64: the features feed a ~60x input-sensitive network; an
// fp32 FFT leaves ~1e-6 relative noise on every bin, i.e. up to ~1e-3 in the log of the
// quiet bands, and that alone would use most of the 1e-4 embedding budget.  In fp64 the
// only fp32 roundings left are the input samples (exact) and the stored output.
//
// Grid: one workgroup of 8 waves per utterance (ragged batches via sample/frame offsets).
// Each wave transforms TWO frames per FFT: z = a + i*b (a, b real windowed frames), one
// 512-point complex FFT, then A[k] = (Z[k] + conj Z[-k]) / 2, B[k] = (Z[k] - conj Z[-k]) / 2i
// -- half the FFT work per frame.  The 512-point FFT is 8 x 8 x 8: three radix-8 DFTs in
// registers (each lane holds 8 complex doubles) with two LDS transposes between them, so
// the load layout (lane + 64 j, j = 0..7) is already the first pass's input layout and no
// bit reversal is needed.  Then |A|^2, |B|^2 -> sparse 80-band mel projection -> log(max(E,
// FLT_EPSILON)), all in double; the per-utterance mean over frames (processor.py:156-157)
// is accumulated in double and subtracted in a second sweep over the (L2-resident) rows.
#include "common.h"
#include "fbank.h"

namespace spk {

namespace {

constexpr int NFFT = 512;
constexpr int FLEN = 400;
constexpr int FSHIFT = 160;
constexpr int WAVES = 8;

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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

__global__ void __launch_bounds__(64 * WAVES, 2)
fbank_kernel(const float* __restrict__ wav, const int64_t* __restrict__ wav_off,
             float* __restrict__ feats, const int64_t* __restrict__ frame_off,
             const FbankTables* __restrict__ tab, int n_mels, int mean_nor, int t_max) {
  __shared__ double2 buf[WAVES][NFFT];   // per-wave FFT transposes / power spectra (64 KB)

  const int utt = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* x = wav + wav_off[utt];
  const int nfr = (int)(frame_off[utt + 1] - frame_off[utt]);
  // packed (t_max == 0): rows at frame_off[utt]; padded: rows at utt * t_max, rows
  // [nfr, t_max) of the utterance zeroed
  const int64_t f0 = t_max > 0 ? (int64_t)utt * t_max : frame_off[utt];
  float* out = feats + f0 * n_mels;
  if (t_max > 0)
    for (int e = nfr * n_mels + threadIdx.x; e < t_max * n_mels; e += blockDim.x) out[e] = 0.f;

  double2* wb = buf[wave];
  double* pw = reinterpret_cast<double*>(wb);     // aliases wb after the FFT: [2][256]
  const int hi = lane >> 3, lo = lane & 7;
  double cs0 = 0.0, cs1 = 0.0;   // column sums of mel bins lane, lane + 64
  const int npairs = (nfr + 1) >> 1;
  for (int p = wave; p < npairs; p += WAVES) {
    const int fa = 2 * p;
    const bool hasb = fa + 1 < nfr;
    const float* sa = x + (int64_t)fa * FSHIFT;
    const float* sb = sa + FSHIFT;
    // 1) both windows (lane + 64 j, zero past 400) and their means
    double re[8], im[8];
    double suma = 0.0, sumb = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      re[j] = i < FLEN ? (double)sa[i] : 0.0;
      im[j] = (hasb && i < FLEN) ? (double)sb[i] : 0.0;
      suma += re[j];
      sumb += im[j];
    }
    const double ma = wave_sum_d(suma) * (1.0 / FLEN), mb = wave_sum_d(sumb) * (1.0 / FLEN);
    // 2) DC removal, pre-emphasis (replicate first sample), Povey window
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      if (i < FLEN) {
        const int ip = i == 0 ? 0 : i - 1;
        const double w = tab->window[i];
        re[j] = ((re[j] - ma) - 0.97 * ((double)sa[ip] - ma)) * w;
        im[j] = hasb ? ((im[j] - mb) - 0.97 * ((double)sb[ip] - mb)) * w : 0.0;
      }
    }
    // 3) FFT.  Pass 1: lane L = n mod 64 holds n1 = 0..7 (n = 64 n1 + L) -> k1, times W512^(L k1)
    dft8(re, im);
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const double2 w = tab->twiddle[lane * k];
      cmul(re[k], im[k], w.x, w.y);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[k * 64 + lane] = make_double2(re[k], im[k]);
    wave_sync();
    // pass 2: lane = (k1 = hi, n3 = lo) holds n2 = 0..7 (L = 8 n2 + n3) -> k2, times W64^(n3 k2)
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const double2 v = wb[hi * 64 + 8 * n + lo];
      re[n] = v.x;
      im[n] = v.y;
    }
    dft8(re, im);
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const double2 w = tab->twiddle[8 * lo * k];
      cmul(re[k], im[k], w.x, w.y);
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[hi * 64 + 8 * k + lo] = make_double2(re[k], im[k]);
    wave_sync();
    // pass 3: lane = (k1 = hi, k2 = lo) holds n3 = 0..7 -> k3; Z[k1 + 8 k2 + 64 k3]
#pragma unroll
    for (int n = 0; n < 8; ++n) {
      const double2 v = wb[hi * 64 + 8 * lo + n];
      re[n] = v.x;
      im[n] = v.y;
    }
    dft8(re, im);
    wave_sync();
#pragma unroll
    for (int k = 0; k < 8; ++k) wb[hi + 8 * lo + 64 * k] = make_double2(re[k], im[k]);
    wave_sync();
    // 4) split the two real spectra and take the power of bins 0..255 (the Nyquist column
    // of the mel bank is zero)
    double pa[4], pb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = lane + 64 * j;
      const double2 z = wb[k], zc = wb[(NFFT - k) & (NFFT - 1)];
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
    // 5) mel projection + log (double), store fp32
    float* oa = out + (int64_t)fa * n_mels;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = lane + 64 * j;
      if (m < n_mels) {
        const int b0 = tab->mel_start[m], nb = tab->mel_len[m], wo = tab->mel_off[m];
        double ea = 0.0, eb = 0.0;
        for (int t = 0; t < nb; ++t) {
          const double w = tab->mel_w[wo + t];
          ea += pw[b0 + t] * w;
          eb += pw[256 + b0 + t] * w;
        }
        const double la = log(fmax(ea, 1.1920928955078125e-07));
        const double lb = log(fmax(eb, 1.1920928955078125e-07));
        oa[m] = (float)la;
        double c = la;
        if (hasb) {
          oa[n_mels + m] = (float)lb;
          c += lb;
        }
        if (j == 0) cs0 += c; else cs1 += c;
      }
    }
    wave_sync();
  }
  if (!mean_nor) return;
  __syncthreads();
  double* colsum = reinterpret_cast<double*>(&buf[0][0]);   // [WAVES][128], FFT buffers are free
  colsum[wave * 128 + lane] = cs0;
  colsum[wave * 128 + lane + 64] = cs1;
  __syncthreads();
  if (nfr <= 0) return;
  double* mean = colsum + WAVES * 128;
  for (int idx = threadIdx.x; idx < n_mels; idx += blockDim.x) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) t += colsum[w * 128 + idx];
    mean[idx] = t / (double)nfr;
  }
  __syncthreads();
  const int total = nfr * n_mels;
  for (int e = threadIdx.x; e < total; e += blockDim.x) out[e] = (float)((double)out[e] - mean[e % n_mels]);
}

}  // namespace

hipError_t launch_fbank(const float* wav, const int64_t* wav_off, int n_utt, float* feats,
                        const int64_t* frame_off, int n_mels, int mean_nor, const FbankTables* tab,
                        hipStream_t s, int t_max) {
  if (n_mels <= 0 || n_mels > 128 || n_utt < 0 || t_max < 0) return hipErrorInvalidValue;
  if (n_utt == 0) return hipSuccess;
  hipLaunchKernelGGL(fbank_kernel, dim3(n_utt), dim3(64 * WAVES), 0, s, wav, wav_off, feats, frame_off, tab, n_mels,
                     mean_nor, t_max);
  return hipGetLastError();
}

}  // namespace spk
