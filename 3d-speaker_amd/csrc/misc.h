#pragma once
#include <algorithm>
#include "common.h"

namespace spk {

// vlen (optional, ragged batches): valid frames per utterance; outputs past them are 0
hipError_t launch_stem_conv3x3(const float* feats, int B, int T, int F, const float* w, const float* bias, int cout,
                               int act, int wstride, float* out, int ldo, hipStream_t s, const int* vlen = nullptr,
                               int* range_flag = nullptr);
// range word of a forward := 0 (a kernel node, not a memset node, in the captured forward)
hipError_t launch_word_reset(int* w, hipStream_t s);
// range guard on a model input (common.h kRangeLimit): flag |= 1 if any |x[i]| >= 2^15
hipError_t launch_range_check(const float* x, size_t n, int* flag, hipStream_t s);
// fp32 -> (hi, lo) fp16 planes for the split-fp16 MFMA GEMM: hi = fp16(w),
// lo = fp16((w - hi) * 2^11) (conv_gemm.hip, "fp16x3").
hipError_t launch_split_f16(const float* w, uint16_t* hi, uint16_t* lo, size_t n, hipStream_t s);
// TSTP / TAP / TSDP (pooling_layers.py:10-55): parts bit 0 = mean, bit 1 = std (TSTP = 3)
hipError_t launch_tstp(const float* x, int B, int H, int W, int C, int ld, float eps, int unbiased, float* out,
                       hipStream_t s, int parts = 3);

// ASTP attentive statistics (pooling_layers.py:93-104): x [B, F, T, C] (pixel stride ldx),
// logits [B, T, F*C] (column f*C + c, row stride ldl) -> out [B, 2*F*C] (mean, std; f*C + c order)
hipError_t launch_astp_pool(const float* logit, int ldl, const float* x, int ldx, int B, int F, int T, int C,
                            float* out, hipStream_t s);

}  // namespace spk
