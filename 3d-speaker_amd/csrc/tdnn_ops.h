#pragma once
#include <algorithm>
#include "common.h"

namespace spk {

// vlen (optional): per-utterance valid frames; the statistics cover frames [0, vlen[b])
hipError_t launch_time_mean(const float* x, int B, int T, int C, int ld, float* out, int ldo, hipStream_t s,
                            const int* vlen = nullptr);
hipError_t launch_asp_stats(const float* x, int B, int T, int C, int ld, float eps, float* out, hipStream_t s,
                            const int* vlen = nullptr);
hipError_t launch_attn_pool(const float* logit, int ldl, const float* x, int ldx, int B, int T, int C, float eps,
                            float* out, hipStream_t s, const int* vlen = nullptr);
// range_flag (fp16x3 range guard, common.h): set when an output reaches kRangeLimit -- the SE
// block outputs accumulate into the next blocks' inputs and the MFA conv's K-concatenated input
hipError_t launch_se_apply(const float* x, int ldx, const float* gate, int ldg, const float* res, int ldr, float* out,
                           int ldo, int B, int T, int C, hipStream_t s, int* range_flag = nullptr);
// vlen (optional, ragged batches): valid frames per utterance
hipError_t launch_cam_context(const float* x, int B, int T, int C, int ld, int seg, int nseg, float* out, int ldo,
                              hipStream_t s, const int* vlen = nullptr);
// CAMLayer context -> linear1 -> ReLU -> linear2 -> sigmoid, once per (utterance, segment):
// gate[(b * nseg + s) * ldg + i]; w1 [red][k1p], w2 [growth][k2p] fp32 (packed GEMM weights);
// segsum: [B][nseg][C] floats of scratch
hipError_t launch_cam_gate(const float* x, int B, int T, int C, int ld, int seg, int nseg, const float* w1, int k1p,
                          const float* b1, int red, const float* w2, int k2p, const float* b2, int growth, float* gate,
                          int ldg, float* segsum, hipStream_t s, const int* vlen = nullptr);
hipError_t launch_stats_pool(const float* x, int B, int T, int C, int ld, float* out, hipStream_t s,
                             const int* vlen = nullptr);
// out[b] = (in[b] + 2 pad - k) / stride + 1 (valid frames after a strided conv)
hipError_t launch_derive_len(const int* in, int* out, int B, int pad, int k, int stride, hipStream_t s);

}  // namespace spk
