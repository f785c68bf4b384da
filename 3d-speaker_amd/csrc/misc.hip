#include <algorithm>
// Small bandwidth-bound kernels around the implicit-GEMM convs, gfx950:
//  * stem conv 3x3, 1 -> Cout channels, reading Fbank features [B, T, F] directly (the
//    reference's permute(0,2,1).unsqueeze(1) is folded into the index math), folded BN
//    and ReLU in the epilogue, channels-last output (ERes2NetV2.py:236-238, DTDNN.py:40-41);
//  * TSTP statistics pooling (pooling_layers.py:47-55): mean and sqrt(unbiased var+1e-8)
//    over time per (freq, channel), one lane per channel so loads are coalesced;
//  * CAM++ StatsPool (layers.py:26-37: mean and unbiased std, no eps).
#include "common.h"
#include "misc.h"

namespace spk {

namespace {

// Tile of the stem: SF frequency rows x ST frames of one utterance per 256-thread block.  Thread
// t owns channel quad q = t % (cout / 4) for every pixel it visits, so its 36 weights and 4
// biases live in registers; the tile's (SF + 2) x (ST + 2) input window is staged in LDS once
// (zero outside the image / past a ragged utterance's end).  Consecutive lanes store
// consecutive 16-B quads of consecutive frames, i.e. every store instruction writes 1 KB of
// contiguous output (channels-last rows): the kernel moves 4 * cout B per pixel out against
// 4 B in, so the stores are what it is bound by.
#ifndef SPK_STEM_SF
#define SPK_STEM_SF 8   // frequency rows per block (2 / 4 / 8 measured 0.33 / 0.26 / 0.22 ms on ERes2NetV2)
#endif
constexpr int STEM_SF = SPK_STEM_SF, STEM_ST = 64;
typedef float stem_f32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256)
stem_conv3x3_kernel(const float* __restrict__ feats, int B, int T, int F, const float* __restrict__ w,
                    const float* __restrict__ bias, int cout, int act, int wstride, float* __restrict__ out,
                    int ldo, const int* __restrict__ vlen, int* range_flag, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  constexpr int WF = STEM_SF + 2, WT = STEM_ST + 2;
  __shared__ float win[WF * WT];
  const int ntt = (T + STEM_ST - 1) / STEM_ST, nft = (F + STEM_SF - 1) / STEM_SF;
  const int b = blockIdx.x / (nft * ntt), r = blockIdx.x % (nft * ntt);
  const int f0 = (r / ntt) * STEM_SF, t0 = (r % ntt) * STEM_ST;
  const int Tb = vlen ? vlen[b] : T;                 // ragged batches: frames past Tb are padding
  for (int i = threadIdx.x; i < WF * WT; i += blockDim.x) {
    const int ff = f0 - 1 + i % WF, tt = t0 - 1 + i / WF;   // f fastest: the rows are [t][F]
    win[(i % WF) * WT + i / WF] = (ff >= 0 && ff < F && tt >= 0 && tt < Tb) ? feats[((size_t)b * T + tt) * F + ff] : 0.f;
  }
  const int nq = cout / 4, q = threadIdx.x % nq, ppp = blockDim.x / nq;   // pixels per pass
  float wr[9][4], br[4];
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[k][j] = w[(4 * q + j) * wstride + k];
#pragma unroll
  for (int j = 0; j < 4; ++j) br[j] = bias[4 * q + j];
  __syncthreads();
  float amax = 0.f;                                  // range guard (common.h)
  for (int p = threadIdx.x / nq; p < STEM_SF * STEM_ST; p += ppp) {
    const int fl = p / STEM_ST, tl = p % STEM_ST;   // frame fastest: contiguous output rows
    const int f = f0 + fl, t = t0 + tl;
    if (f >= F || t >= T) continue;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const float x = win[(fl + dy) * WT + tl + dx];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = fmaf(x, wr[dy * 3 + dx][j], o[j]);
      }
    stem_f32x4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = o[j] + br[j];
      if (act == ACT_RELU) a = fmaxf(a, 0.f);
      v[j] = t >= Tb ? 0.f : a;
      amax = fmaxf(amax, fabsf(v[j]));
    }
    *reinterpret_cast<stem_f32x4*>(out + (((size_t)b * F + f) * T + t) * ldo + 4 * q) = v;
  }
  range_note(range_flag, amax);
}

// range guard on a model input (common.h): grid-stride max |x| of n floats
__global__ void __launch_bounds__(256) range_check_kernel(const float* __restrict__ x, size_t n, int* flag) {
  float amax = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    amax = fmaxf(amax, fabsf(x[i]));
  range_note(flag, amax);
}

// x: [B, H, W, C] (pixel stride ld).  out: [B, 2*H*C]: mean at [h*C + c], std at [H*C + h*C + c].
__global__ void __launch_bounds__(256)
tstp_kernel(const float* __restrict__ x, int B, int H, int W, int C, int ld, float eps, int unbiased,
            int parts, float* __restrict__ out, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  const long long total = (long long)B * H * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const int h = (int)((e / C) % H);
    const int b = (int)(e / ((long long)C * H));
    const float* p = x + ((size_t)(b * H + h) * W) * ld + c;
    // one Welford pass (mean, M2): the activation is read once, not twice
    float mean = 0.f, q = 0.f;
    scan_frames<16>(p, ld, W, [&](float v, int t) {
      const float dlt = v - mean;
      mean += dlt / (float)(t + 1);
      q = fmaf(dlt, v - mean, q);
    });
    const float var = q / (float)(unbiased ? W - 1 : W);
    // parts: bit 0 = mean (TAP), bit 1 = std (TSDP); TSTP = both, mean first
    const int np = (parts & 1) + ((parts >> 1) & 1);
    float* o = out + (size_t)b * np * H * C;
    if (parts & 1) o[h * C + c] = mean;
    if (parts & 2) o[(parts & 1) * H * C + h * C + c] = sqrtf(var + eps);
  }
}

// ASTP pooling (pooling_layers.py:93-104) over x [B, F, T, C] (pixel stride ldx) with the
// attention logits [B, T, F*C] (row stride ldl, column f*C + c): per (b, f, c) an online
// softmax over time fused with a weighted Welford pass (x and the logits read once);
// var = M2 / sum w (= sum alpha x^2 - mean^2), std = sqrt(max(var, 1e-10)).  out [B, 2*F*C]:
// mean at f*C + c, std at F*C + f*C + c (the TSTP order seg_1 is packed for).
__global__ void __launch_bounds__(256)
astp_pool_kernel(const float* __restrict__ logit, int ldl, const float* __restrict__ x, int ldx, int B, int F, int T,
                 int C, float* __restrict__ out, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  const long long total = (long long)B * F * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const int f = (int)((e / C) % F);
    const int b = (int)(e / ((long long)C * F));
    const float* l = logit + (size_t)b * T * ldl + (size_t)f * C + c;
    const float* p = x + ((size_t)(b * F + f) * T) * ldx + c;
    float mx = -INFINITY, sw = 0.f, mean = 0.f, m2 = 0.f;
    for (int t = 0; t < T; ++t) {
      const float lv = l[(size_t)t * ldl], xv = p[(size_t)t * ldx];
      if (lv > mx) {
        const float sc = __expf(mx - lv);   // 0 on the first sample
        sw *= sc;
        m2 *= sc;
        mx = lv;
      }
      const float w = __expf(lv - mx);
      sw += w;
      const float d = xv - mean;
      mean += d * (w / sw);
      m2 += w * d * (xv - mean);
    }
    float* o = out + (size_t)b * 2 * F * C;
    o[f * C + c] = mean;
    o[F * C + f * C + c] = sqrtf(fmaxf(m2 / sw, 1e-10f));
  }
}

}  // namespace

hipError_t launch_astp_pool(const float* logit, int ldl, const float* x, int ldx, int B, int F, int T, int C,
                            float* out, hipStream_t s) {
  const long long total = (long long)B * F * C;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(astp_pool_kernel, dim3(blocks), dim3(256), 0, s, logit, ldl, x, ldx, B, F, T, C, out, launch_gate());
  return hipGetLastError();
}

hipError_t launch_stem_conv3x3(const float* feats, int B, int T, int F, const float* w, const float* bias, int cout,
                               int act, int wstride, float* out, int ldo, hipStream_t s, const int* vlen,
                               int* range_flag) {
  // cout / 4 channel quads must divide the 256 threads (one quad per thread for every pixel)
  if (cout % 4 || cout > 128 || 256 % (cout / 4) || ldo % 4 || (long long)B * F * T * ldo >= (1LL << 40))
    return hipErrorInvalidValue;
  const long long blocks = (long long)B * ((F + STEM_SF - 1) / STEM_SF) * ((T + STEM_ST - 1) / STEM_ST);
  if (blocks >= (1LL << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_conv3x3_kernel, dim3((unsigned)blocks), dim3(256), 0, s, feats, B, T, F, w, bias, cout, act, wstride, out,
                     ldo, vlen, range_flag, launch_gate());
  return hipGetLastError();
}

hipError_t launch_range_check(const float* x, size_t n, int* flag, hipStream_t s) {
  if (!flag || n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(range_check_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, n, flag);
  return hipGetLastError();
}

hipError_t launch_tstp(const float* x, int B, int H, int W, int C, int ld, float eps, int unbiased, float* out,
                       hipStream_t s, int parts) {
  if (parts < 1 || parts > 3) return hipErrorInvalidValue;
  const long long total = (long long)B * H * C;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(tstp_kernel, dim3(blocks), dim3(256), 0, s, x, B, H, W, C, ld, eps, unbiased, parts, out, launch_gate());
  return hipGetLastError();
}

__global__ void word_reset_kernel(int* w) {
  if (threadIdx.x == 0) *w = 0;
}

hipError_t launch_word_reset(int* w, hipStream_t s) {
  hipLaunchKernelGGL(word_reset_kernel, dim3(1), dim3(64), 0, s, w);
  return hipGetLastError();
}

__global__ void split_f16_kernel(const float* w, _Float16* hi, _Float16* lo, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = w[i];
    const _Float16 h = (_Float16)v;
    hi[i] = h;
    lo[i] = (_Float16)((v - (float)h) * 2048.0f);
  }
}

hipError_t launch_split_f16(const float* w, uint16_t* hi, uint16_t* lo, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const int blocks = (int)std::min<size_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(split_f16_kernel, dim3(blocks), dim3(256), 0, s, w, reinterpret_cast<_Float16*>(hi),
                     reinterpret_cast<_Float16*>(lo), n);
  return hipGetLastError();
}

}  // namespace spk
