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

__global__ void __launch_bounds__(256)
stem_conv3x3_kernel(const float* __restrict__ feats, int B, int T, int F, const float* __restrict__ w,
                    const float* __restrict__ bias, int cout, int act, int wstride, float* __restrict__ out,
                    int ldo, const int* __restrict__ vlen, int* range_flag, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  // thread -> (pixel, 16 output channels); pixel = (b, f, t) of the (F, T) image.  Weights and
  // bias are staged in LDS once per block; 32-bit index math only.
  __shared__ float ws[128 * 9];
  __shared__ float bs[128];
  for (int i = threadIdx.x; i < cout * 9; i += blockDim.x) ws[i] = w[(i / 9) * wstride + (i % 9)];
  for (int i = threadIdx.x; i < cout; i += blockDim.x) bs[i] = bias[i];
  __syncthreads();
  const int groups = cout / 16;
  const int total = B * F * T * groups;
  float amax = 0.f;                                  // range guard (common.h)
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int g = e % groups;
    const int pix = e / groups;
    const int t = pix % T;
    const int bf = pix / T;
    const int f = bf % F;
    const int b = bf / F;
    const int Tb = vlen ? vlen[b] : T;               // ragged batches: frames past Tb are padding
    float in[9];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int ff = f + dy - 1, tt = t + dx - 1;
        in[dy * 3 + dx] = (ff >= 0 && ff < F && tt >= 0 && tt < Tb) ? feats[(b * T + tt) * F + ff] : 0.f;
      }
    const bool dead = t >= Tb;
    float* op = out + (size_t)pix * ldo + g * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 o;
      float* ov = &o.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = g * 16 + q * 4 + j;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) acc = fmaf(in[k], ws[c * 9 + k], acc);
        acc += bs[c];
        ov[j] = dead ? 0.f : (act == ACT_RELU ? fmaxf(acc, 0.f) : acc);
        amax = fmaxf(amax, fabsf(ov[j]));
      }
      *reinterpret_cast<float4*>(op + q * 4) = o;
    }
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
    for (int t = 0; t < W; ++t) {
      const float v = p[(size_t)t * ld];
      const float dlt = v - mean;
      mean += dlt / (float)(t + 1);
      q = fmaf(dlt, v - mean, q);
    }
    const float var = q / (float)(unbiased ? W - 1 : W);
    // parts: bit 0 = mean (TAP), bit 1 = std (TSDP); TSTP = both, mean first
    const int np = (parts & 1) + ((parts >> 1) & 1);
    float* o = out + (size_t)b * np * H * C;
    if (parts & 1) o[h * C + c] = mean;
    if (parts & 2) o[(parts & 1) * H * C + h * C + c] = sqrtf(var + eps);
  }
}

}  // namespace

hipError_t launch_stem_conv3x3(const float* feats, int B, int T, int F, const float* w, const float* bias, int cout,
                               int act, int wstride, float* out, int ldo, hipStream_t s, const int* vlen,
                               int* range_flag) {
  if (cout % 16 || cout > 128 || ldo % 4 || (long long)B * F * T * (cout / 16) >= (1LL << 31))
    return hipErrorInvalidValue;
  const long long total = (long long)B * F * T * (cout / 16);
  const int blocks = (int)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(stem_conv3x3_kernel, dim3(blocks), dim3(256), 0, s, feats, B, T, F, w, bias, cout, act, wstride, out,
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
