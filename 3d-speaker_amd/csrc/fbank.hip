// Kaldi log-mel filterbank (torchaudio.compliance.kaldi.fbank defaults as called by
// speakerlab/process/processor.py:133-158), gfx950.
//
// One workgroup per utterance (ragged batches via sample/frame offsets), one wave per
// frame at a time: coalesced loads of the 400-sample window, DC removal + pre-emphasis +
// Povey window in registers, 512-point radix-2 FFT in LDS (fp32, host-computed twiddles),
// |X|^2, sparse 80-band mel projection, log(max(E, FLT_EPSILON)).  The per-utterance
// mean normalisation (processor.py:156-157) is a second sweep by the same workgroup after
// a wave-sum + LDS reduction of the column sums — the frames it re-reads are L2-resident.
#include "common.h"
#include "fbank.h"

namespace spk {

namespace {

constexpr int NFFT = 512;
constexpr int HALF = NFFT / 2;
constexpr int FLEN = 400;
constexpr int FSHIFT = 160;
constexpr int WAVES = 4;

__device__ __forceinline__ float wave_sum(float v) {
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

__device__ __forceinline__ int bitrev9(int x) { return __builtin_bitreverse32((unsigned)x) >> 23; }

__global__ void __launch_bounds__(256)
fbank_kernel(const float* __restrict__ wav, const int64_t* __restrict__ wav_off,
             float* __restrict__ feats, const int64_t* __restrict__ frame_off,
             const FbankTables* __restrict__ tab, int n_mels, int mean_nor, int t_max) {
  __shared__ float2 buf[WAVES][NFFT];
  __shared__ float pw[WAVES][HALF + 1];
  __shared__ float colsum[WAVES][128];

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

  float cs0 = 0.f, cs1 = 0.f;   // column sums for mel bins lane, lane+64
  for (int fr = wave; fr < nfr; fr += WAVES) {
    const float* s = x + (int64_t)fr * FSHIFT;
    // 1) load window (7 per lane; 400 = 6*64 + 16) and its mean
    float v[7];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      const int i = lane + 64 * j;
      v[j] = i < FLEN ? s[i] : 0.f;
      sum += v[j];
    }
    const float mean = wave_sum(sum) * (1.0f / FLEN);
    // 2) DC removal, pre-emphasis (replicate first sample), Povey window -> bit-reversed LDS
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = lane + 64 * j;
      float y = 0.f;
      if (i < FLEN) {
        const float cur = v[j < 7 ? j : 6] - mean;
        const float prev = (i == 0 ? s[0] : s[i - 1]) - mean;
        y = (cur - 0.97f * prev) * tab->window[i];
      }
      buf[wave][bitrev9(i)] = make_float2(y, 0.f);
    }
    wave_sync();
    // 3) radix-2 DIT FFT, 9 stages, 4 butterflies per lane per stage
#pragma unroll
    for (int lg = 0; lg < 9; ++lg) {
      const int hs = 1 << lg;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int b = lane + 64 * q;               // butterfly 0..255
        const int grp = b >> lg, pos = b & (hs - 1);
        const int i0 = grp * 2 * hs + pos, i1 = i0 + hs;
        const float2 w = tab->twiddle[pos << (8 - lg)];   // exp(-2 pi i k / 512)
        const float2 a = buf[wave][i0], c = buf[wave][i1];
        const float tr = c.x * w.x - c.y * w.y;
        const float ti = c.x * w.y + c.y * w.x;
        buf[wave][i0] = make_float2(a.x + tr, a.y + ti);
        buf[wave][i1] = make_float2(a.x - tr, a.y - ti);
      }
      wave_sync();
    }
    // 4) power spectrum bins 0..256
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int k = lane + 64 * j;
      if (k <= HALF) {
        const float2 c = buf[wave][k];
        pw[wave][k] = c.x * c.x + c.y * c.y;
      }
    }
    wave_sync();
    // 5) mel projection + log
    float* o = out + (int64_t)fr * n_mels;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = lane + 64 * j;
      if (m < n_mels) {
        const int b0 = tab->mel_start[m], nb = tab->mel_len[m], wo = tab->mel_off[m];
        float e = 0.f;
        for (int t = 0; t < nb; ++t) e += pw[wave][b0 + t] * tab->mel_w[wo + t];
        const float lv = __logf(fmaxf(e, 1.1920928955078125e-07f));
        o[m] = lv;
        if (j == 0) cs0 += lv; else cs1 += lv;
      }
    }
    wave_sync();
  }
  if (!mean_nor) return;
  colsum[wave][lane] = cs0;
  colsum[wave][lane + 64] = cs1;
  __syncthreads();
  if (nfr <= 0) return;
  const float inv = 1.0f / (float)nfr;
  for (int idx = threadIdx.x; idx < n_mels; idx += blockDim.x) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) t += colsum[w][idx];
    colsum[0][idx] = t * inv;   // idx-owned slot; only read after the barrier below
  }
  __syncthreads();
  const int total = nfr * n_mels;
  for (int e = threadIdx.x; e < total; e += blockDim.x) out[e] -= colsum[0][e % n_mels];
}

}  // namespace

hipError_t launch_fbank(const float* wav, const int64_t* wav_off, int n_utt, float* feats,
                        const int64_t* frame_off, int n_mels, int mean_nor, const FbankTables* tab,
                        hipStream_t s, int t_max) {
  if (n_mels <= 0 || n_mels > 128 || n_utt < 0 || t_max < 0) return hipErrorInvalidValue;
  if (n_utt == 0) return hipSuccess;
  hipLaunchKernelGGL(fbank_kernel, dim3(n_utt), dim3(256), 0, s, wav, wav_off, feats, frame_off, tab, n_mels,
                     mean_nor, t_max);
  return hipGetLastError();
}

}  // namespace spk
