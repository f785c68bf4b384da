// Reductions and elementwise ops of the TDNN models (ECAPA-TDNN, CAM++), gfx950.
// All tensors are channels-last [B, T, C] with pixel stride `ld`; every kernel puts one
// lane on one channel so the time loops read coalesced 256-B rows.
//
//  * time_mean        SEBlock squeeze, s = mean_T(x)                       ECAPA_TDNN.py:209-216
//  * asp_stats        global-context mean / std, weights 1/T, clamp 1e-12  ECAPA_TDNN.py:256-270
//  * attn_pool        softmax_T(logits) weighted mean / std               ECAPA_TDNN.py:276-287
//  * se_apply         out = x * gate[b, c] + residual                       ECAPA_TDNN.py:222, 347
//  * cam_context      mean_T + 100-frame segment mean (ceil_mode)          campplus/layers.py:93-110
//  * stats_pool       mean + unbiased std (no eps)                          campplus/layers.py:26-37
#include "common.h"
#include <cstdlib>

#include "tdnn_ops.h"

namespace spk {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int CAM_SEGS = 4;   // segments whose 1x1 layers run together (weights read once)
constexpr int CAM_WQ = 8;
#ifndef SPK_SEGSUM_U
#define SPK_SEGSUM_U 4   // cam_segsum: row loads in flight per thread
#endif
#ifndef SPK_ATTN_U
#define SPK_ATTN_U 8     // attn_pool: frames per load batch
#endif     // lean gate: float4 quads of a thread's weight slice per layer

inline int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 65536); }

// vlen (optional): utterance b's statistics cover frames [0, valid(b)) only -- ECAPA's
// masked SE / ASP (ECAPA_TDNN.py:211-214, 259-270, 281-282); the host guarantees
// 1 <= vlen[b] <= T and the kernels clamp to that range anyway
__device__ __forceinline__ int valid_frames(const int* vlen, int b, int T) {
  return vlen ? min(max(vlen[b], 1), T) : T;
}

__global__ void time_mean_kernel(const float* __restrict__ x, int B, int T, int C, int ld, float* __restrict__ out,
                                 int ldo, const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * C;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C), b = (int)(e / C);
    const int Tb = valid_frames(vlen, b, T);
    const float* p = x + (size_t)b * T * ld + c;
    float s = 0.f;
    scan_frames<16>(p, ld, Tb, [&](float v, int) { s += v; });
    out[(size_t)b * ldo + c] = s / (float)Tb;
  }
}

__global__ void asp_stats_kernel(const float* __restrict__ x, int B, int T, int C, int ld, float eps,
                                 float* __restrict__ out, const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * C;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C), b = (int)(e / C);
    const int Tb = valid_frames(vlen, b, T);
    const float* p = x + (size_t)b * T * ld + c;
    // one Welford pass (mean, M2) instead of two passes over x; var = M2 / T
    float mean = 0.f, m2 = 0.f;
    scan_frames<16>(p, ld, Tb, [&](float xv, int t) {
      const float d = xv - mean;
      mean += d / (float)(t + 1);
      m2 += d * (xv - mean);
    });
    out[(size_t)b * 2 * C + c] = mean;
    out[(size_t)b * 2 * C + C + c] = sqrtf(fmaxf(m2 / (float)Tb, eps));
  }
}

__global__ void attn_pool_kernel(const float* __restrict__ logit, int ldl, const float* __restrict__ x, int ldx, int B,
                                 int T, int C, float eps, float* __restrict__ out, const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * C;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C), b = (int)(e / C);
    const int Tb = valid_frames(vlen, b, T);   // masked_fill(-inf) past it: weight 0
    const float* l = logit + (size_t)b * T * ldl + c;
    const float* p = x + (size_t)b * T * ldx + c;
    // one pass: online softmax (running max, weights rescaled when it moves) fused with a
    // weighted Welford update of mean and M2 = sum w (x - mean)^2, so logits and x are read
    // once instead of four and two times; var = M2 / sum w (ECAPA_TDNN.py:276-287)
    float mx = -INFINITY, sw = 0.f, mean = 0.f, m2 = 0.f;
    scan_frames2<SPK_ATTN_U>(l, ldl, p, ldx, Tb, [&](float lv, float xv) {
      if (lv > mx) {
        const float sc = __expf(mx - lv);           // 0 on the first sample
        sw *= sc;
        m2 *= sc;
        mx = lv;
      }
      const float w = __expf(lv - mx);
      sw += w;
      const float d = xv - mean;
      mean += d * (w / sw);
      m2 += w * d * (xv - mean);
    });
    out[(size_t)b * 2 * C + c] = mean;
    out[(size_t)b * 2 * C + C + c] = sqrtf(fmaxf(m2 / sw, eps));
  }
}

__global__ void se_apply_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ gate, int ldg,
                                const float* __restrict__ res, int ldr, float* __restrict__ out, int ldo, int B, int T,
                                int C, int* range_flag, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  const int C4 = C / 4;
  float amax = 0.f;   // range guard (common.h): block outputs feed the next block's split GEMM
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * T * C4;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C4) * 4;
    const long long row = e / C4;
    const int b = (int)(row / T);
    const float4 v = *reinterpret_cast<const float4*>(x + row * ldx + c);
    const float4 g = *reinterpret_cast<const float4*>(gate + (size_t)b * ldg + c);
    const float4 r = *reinterpret_cast<const float4*>(res + row * ldr + c);
    float4 o;
    o.x = v.x * g.x + r.x; o.y = v.y * g.y + r.y; o.z = v.z * g.z + r.z; o.w = v.w * g.w + r.w;
    amax = fmaxf(amax, fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fmaxf(fabsf(o.z), fabsf(o.w))));
    *reinterpret_cast<float4*>(out + row * ldo + c) = o;
  }
  range_note(range_flag, amax);
}

// ctx[b, s, c] = mean_T(x)[b, c] + mean over frames [100 s, min(100 s + 100, T)) of x[b, :, c]
// (ragged batches: utterance b has vlen[b] valid frames; segments past them are written as 0)
__global__ void cam_context_kernel(const float* __restrict__ x, int B, int T, int C, int ld, int seg, int nseg,
                                   float* __restrict__ out, int ldo, const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * C;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C), b = (int)(e / C);
    const int Tb = valid_frames(vlen, b, T);
    const float* p = x + (size_t)b * T * ld + c;
    float tot = 0.f;
    for (int t = 0; t < Tb; ++t) tot += p[(size_t)t * ld];
    const float mean = tot / (float)Tb;
    for (int s = 0; s < nseg; ++s) {
      const int t0 = s * seg, t1 = min(Tb, t0 + seg);
      float a = 0.f;
      for (int t = t0; t < t1; ++t) a += p[(size_t)t * ld];
      out[((size_t)b * nseg + s) * ldo + c] = t1 > t0 ? mean + a / (float)(t1 - t0) : 0.f;
    }
  }
}

// CAMLayer's context branch (campplus/layers.py:93-110: context = mean_T(x) +
// seg_pooling(x, 100) -> linear1 -> ReLU -> linear2 -> sigmoid).  The context is constant
// inside a 100-frame segment, so both 1x1 layers run once per segment, in fp32 on the
// VALU (K = 128 / 64: far too small for MFMA tiles); the gate [B][nseg][growth] then
// scales linear_local's output rows in its epilogue.  Two kernels:
//  * cam_segsum: one workgroup per (segment, utterance) sums the segment's valid rows
//    (float4 column quads x row lanes, four row loads in flight, fixed-order reduction);
//  * cam_gate: one workgroup per utterance: mean = (sum of its segment sums) / T, the
//    contexts, and both layers with the weights staged transposed in LDS.
// segment sg's sum of utterance b's valid rows: quad tid % nq of row lanes tid / nq, combined
// through `part` in a fixed order; written by threads tid < nq to out[4 tid ..]
__device__ __forceinline__ void cam_segsum_body(const float* __restrict__ x, int T, int C, int ld, int seg, int sg,
                                                int b, int Tb, f32x4* part, float* out) {
  const int tid = threadIdx.x;
  const int nq = C / 4, RL = 256 / nq;
  const int cq = tid % nq, rl = tid / nq;
  const int t0 = sg * seg, t1 = min(Tb, t0 + seg);
  f32x4 a = {0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    const float* xb = x + (size_t)b * T * ld + cq * 4;
    int t = t0 + rl;
    for (; t + (SPK_SEGSUM_U - 1) * RL < t1; t += SPK_SEGSUM_U * RL) {
      f32x4 q[SPK_SEGSUM_U];
#pragma unroll
      for (int j = 0; j < SPK_SEGSUM_U; ++j) q[j] = *reinterpret_cast<const f32x4*>(xb + (size_t)(t + j * RL) * ld);
#pragma unroll
      for (int j = 0; j < SPK_SEGSUM_U; ++j) a += q[j];
    }
    for (; t < t1; t += RL) a += *reinterpret_cast<const f32x4*>(xb + (size_t)t * ld);
  }
  part[tid] = a;
  __syncthreads();
  if (tid < nq) {
    f32x4 v = part[tid];
    for (int r = 1; r < RL; ++r) v += part[r * nq + tid];
    *reinterpret_cast<f32x4*>(out + tid * 4) = v;
  }
}

__global__ void __launch_bounds__(256)
cam_segsum_kernel(const float* __restrict__ x, int T, int C, int ld, int seg, int nseg, float* __restrict__ segsum,
                  const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  __shared__ f32x4 part[256];
  const int sg = blockIdx.x, b = blockIdx.y;
  cam_segsum_body(x, T, C, ld, seg, sg, b, valid_frames(vlen, b, T), part, segsum + ((size_t)b * nseg + sg) * C);
}

__global__ void __launch_bounds__(1024)
cam_gate_kernel(const float* __restrict__ segsum, int T, int C, int seg, int nseg, const float* __restrict__ w1,
                int k1p, const float* __restrict__ b1, int red, const float* __restrict__ w2, int k2p,
                const float* __restrict__ b2, int growth, float* __restrict__ gate, int ldg,
                const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  extern __shared__ float sm[];
  float* w1t = sm;                          // [C][red + 1]  (transposed, padded: conflict-free)
  float* w2t = w1t + C * (red + 1);         // [red][growth + 1]
  float* mean = w2t + red * (growth + 1);   // [C]
  float* ctx = mean + C;                    // [CAM_SEGS][C]
  float* h = ctx + CAM_SEGS * C;            // [CAM_SEGS][red]
  float* part = h + CAM_SEGS * red;         // [CAM_SEGS][1024] dot partials
  const int b = blockIdx.x, tid = threadIdx.x;
  const int Tb = valid_frames(vlen, b, T);
#pragma unroll 4
  for (int e = tid; e < red * C; e += blockDim.x) {       // coalesced rows, transposed into LDS
    const int n = e / C, k = e - n * C;
    w1t[k * (red + 1) + n] = w1[(size_t)n * k1p + k];
  }
#pragma unroll 2
  for (int e = tid; e < growth * red; e += blockDim.x) {
    const int n = e / red, k = e - n * red;
    w2t[k * (growth + 1) + n] = w2[(size_t)n * k2p + k];
  }
  const float* ss = segsum + (size_t)b * nseg * C;
  for (int c = tid; c < C; c += blockDim.x) {
    float v = 0.f;
    for (int sg = 0; sg < nseg; ++sg) v += ss[(size_t)sg * C + c];
    mean[c] = v / (float)Tb;
  }
  __syncthreads();
  // out[s][n] = act(bias[n] + sum_k wt[k][n] in[s][k]): P = blockDim / N partial dots per
  // output over contiguous K slices (all segments of the chunk at once), then in slice order
  auto dense = [&](const float* in, int K, const float* wt, int N, const float* bias, bool relu, int ns, float* out,
                   int ldout) {
    const int P = blockDim.x / N, n = tid % N, pi = tid / N, kk = (K + P - 1) / P;
    if (pi < P) {
      float acc[CAM_SEGS];
#pragma unroll
      for (int j = 0; j < CAM_SEGS; ++j) acc[j] = 0.f;
      const int k0 = pi * kk, k1 = min(K, k0 + kk);
      for (int k = k0; k < k1; ++k) {
        const float wv = wt[k * (N + 1) + n];
#pragma unroll
        for (int j = 0; j < CAM_SEGS; ++j)
          if (j < ns) acc[j] += wv * in[j * K + k];
      }
#pragma unroll
      for (int j = 0; j < CAM_SEGS; ++j)
        if (j < ns) part[j * 1024 + pi * N + n] = acc[j];
    }
    __syncthreads();
    for (int e = tid; e < ns * N; e += blockDim.x) {
      const int j = e / N, o = e - j * N;
      float v = bias ? bias[o] : 0.f;
      for (int q = 0; q < P; ++q) v += part[j * 1024 + q * N + o];
      out[(size_t)j * ldout + o] = relu ? fmaxf(v, 0.f) : 1.0f / (1.0f + __expf(-v));
    }
    __syncthreads();
  };
  for (int s0 = 0; s0 < nseg; s0 += CAM_SEGS) {
    const int ns = min(CAM_SEGS, nseg - s0);
    for (int e = tid; e < ns * C; e += blockDim.x) {
      const int j = e / C, c = e - j * C;
      const int t0 = (s0 + j) * seg, t1 = min(Tb, t0 + seg);
      ctx[e] = t1 > t0 ? mean[c] + ss[(size_t)(s0 + j) * C + c] / (float)(t1 - t0) : 0.f;
    }
    __syncthreads();
    dense(ctx, C, w1t, red, b1, true, ns, h, red);
    dense(h, red, w2t, growth, b2, false, ns, gate + ((size_t)b * nseg + s0) * ldg, ldg);
  }
}

// Lean form of cam_gate_kernel (CAMLayer context MLP, layers.py:40-67) for the shapes every
// CAM++ layer has: 256 threads per utterance, the weights read straight from global memory
// (row slices of 16 B quads, L2-resident: every utterance reads the same few KB) instead of
// transposed into LDS per block, partial dots over Q = 256 / N contiguous K-slices combined by
// a butterfly over the Q neighbouring lanes (fixed order).  Requires 256 % red == 0,
// 256 % growth == 0, C % (4 * (256 / red)) == 0, red % (4 * (256 / growth)) == 0 (host).
// `ss`: utterance b's segment sums [nseg][C] (global memory, or LDS in the fused kernel);
// `sm`: C + CAM_SEGS (C + red) floats of LDS
__device__ __forceinline__ void cam_gate_lean_body(const float* ss, int C, int seg, int nseg, const float* __restrict__ w1,
                                                   int k1p, const float* __restrict__ b1, int red,
                                                   const float* __restrict__ w2, int k2p, const float* __restrict__ b2,
                                                   int growth, float* __restrict__ gate, int ldg, int b, int Tb, float* sm) {
  float* mean = sm;                         // [C]
  float* ctx = mean + C;                    // [CAM_SEGS][C]
  float* h = ctx + CAM_SEGS * C;            // [CAM_SEGS][red]
  const int tid = threadIdx.x;
  // this thread's weight slices and biases of both layers, requested first: the phases below
  // are a chain of dependent steps, and a weight load at its use was one more L2 round trip
  // in it (host: K / Q <= 4 * CAM_WQ for both layers)
  f32x4 wq1[CAM_WQ], wq2[CAM_WQ];
  float bq1 = 0.f, bq2 = 0.f;
  auto load_w = [&](const float* w, int kp, int K, int N, const float* bias, f32x4 (&wq)[CAM_WQ], float& bq) {
    const int Q = 256 / N, n = tid / Q, q = tid % Q, kk = K / Q;
    const float* wr = w + (size_t)n * kp + q * kk;
#pragma unroll
    for (int i = 0; i < CAM_WQ; ++i)
      wq[i] = 4 * i < kk ? *reinterpret_cast<const f32x4*>(wr + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
    bq = bias ? bias[n] : 0.f;
  };
  load_w(w1, k1p, C, red, b1, wq1, bq1);
  load_w(w2, k2p, red, growth, b2, wq2, bq2);
  for (int c = tid; c < C; c += 256) {
    float v = 0.f;
    for (int sg = 0; sg < nseg; ++sg) v += ss[(size_t)sg * C + c];
    mean[c] = v / (float)Tb;
  }
  // out[j][n] = act(bias[n] + sum_k w[n][k] in[j][k]): thread = (n, slice q of K / Q)
  auto dense = [&](const float* in, int K, const f32x4 (&wq)[CAM_WQ], float bq, int N, bool relu, int ns,
                   float* out, int ldout) {
    const int Q = 256 / N, n = tid / Q, q = tid % Q, kk = K / Q;
    float acc[CAM_SEGS];
#pragma unroll
    for (int j = 0; j < CAM_SEGS; ++j) acc[j] = 0.f;
#pragma unroll
    for (int i = 0; i < CAM_WQ; ++i) {
      if (4 * i >= kk) break;
      const f32x4 wv = wq[i];
#pragma unroll
      for (int j = 0; j < CAM_SEGS; ++j) {
        if (j < ns) {
          const f32x4 iv = *reinterpret_cast<const f32x4*>(in + j * K + q * kk + 4 * i);
          acc[j] += wv[0] * iv[0] + wv[1] * iv[1] + wv[2] * iv[2] + wv[3] * iv[3];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < CAM_SEGS; ++j)
      for (int m = 1; m < Q; m <<= 1) acc[j] += __shfl_xor(acc[j], m);   // the Q lanes of n are adjacent
    if (q == 0) {
#pragma unroll
      for (int j = 0; j < CAM_SEGS; ++j) {
        if (j < ns) {
          const float v = acc[j] + bq;
          out[(size_t)j * ldout + n] = relu ? fmaxf(v, 0.f) : __builtin_amdgcn_rcpf(1.0f + __expf(-v));
        }
      }
    }
  };
  for (int s0 = 0; s0 < nseg; s0 += CAM_SEGS) {
    const int ns = min(CAM_SEGS, nseg - s0);
    __syncthreads();                                       // mean ready / previous chunk's h read
    for (int e = tid; e < ns * C; e += 256) {
      const int j = e / C, c = e - j * C;
      const int t0 = (s0 + j) * seg, t1 = min(Tb, t0 + seg);
      ctx[e] = t1 > t0 ? mean[c] + ss[(size_t)(s0 + j) * C + c] / (float)(t1 - t0) : 0.f;
    }
    __syncthreads();
    dense(ctx, C, wq1, bq1, red, true, ns, h, red);
    __syncthreads();
    dense(h, red, wq2, bq2, growth, false, ns, gate + ((size_t)b * nseg + s0) * ldg, ldg);
  }
}

__global__ void __launch_bounds__(256)
cam_gate_lean_kernel(const float* __restrict__ segsum, int T, int C, int seg, int nseg, const float* __restrict__ w1,
                     int k1p, const float* __restrict__ b1, int red, const float* __restrict__ w2, int k2p,
                     const float* __restrict__ b2, int growth, float* __restrict__ gate, int ldg,
                     const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  extern __shared__ float sm[];
  const int b = blockIdx.x;
  cam_gate_lean_body(segsum + (size_t)b * nseg * C, C, seg, nseg, w1, k1p, b1, red, w2, k2p, b2, growth, gate, ldg, b,
                     valid_frames(vlen, b, T), sm);
}

// The segment sums and the lean gate in one launch (one workgroup per utterance; the sums stay
// in LDS): CAM++ runs this pair once per dense layer, 52 times a forward, and the two launches
// of ~7 us each were dominated by their fixed cost.  Same arithmetic and order as the pair.
__global__ void __launch_bounds__(256)
cam_gate_fused_kernel(const float* __restrict__ x, int T, int C, int ld, int seg, int nseg, const float* __restrict__ w1,
                      int k1p, const float* __restrict__ b1, int red, const float* __restrict__ w2, int k2p,
                      const float* __restrict__ b2, int growth, float* __restrict__ gate, int ldg,
                      const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  extern __shared__ float sm[];
  f32x4* part = reinterpret_cast<f32x4*>(sm);            // [256] segment-sum partials
  float* ssl = sm + 4 * 256;                             // [nseg][C]
  const int b = blockIdx.x;
  const int Tb = valid_frames(vlen, b, T);
  for (int sg = 0; sg < nseg; ++sg) {
    cam_segsum_body(x, T, C, ld, seg, sg, b, Tb, part, ssl + (size_t)sg * C);
    __syncthreads();                                     // sums written, partials free again
  }
  cam_gate_lean_body(ssl, C, seg, nseg, w1, k1p, b1, red, w2, k2p, b2, growth, gate, ldg, b, Tb, ssl + (size_t)nseg * C);
}

__global__ void stats_pool_kernel(const float* __restrict__ x, int B, int T, int C, int ld, float* __restrict__ out,
                                  const int* __restrict__ vlen, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < (long long)B * C;
       e += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(e % C), b = (int)(e / C);
    const int Tb = valid_frames(vlen, b, T);
    const float* p = x + (size_t)b * T * ld + c;
    float mean = 0.f, q = 0.f;                       // one Welford pass (mean, M2)
    scan_frames<16>(p, ld, Tb, [&](float v, int t) {
      const float d = v - mean;
      mean += d / (float)(t + 1);
      q += d * (v - mean);
    });
    out[(size_t)b * 2 * C + c] = mean;
    out[(size_t)b * 2 * C + C + c] = sqrtf(q / (float)(Tb - 1));
  }
}

// out[b] = (in[b] + 2 pad - k) / stride + 1: valid output frames of a strided conv
__global__ void derive_len_kernel(const int* __restrict__ in, int* __restrict__ out, int B, int pad, int k, int stride, const int* __restrict__ run_if) {
  SPK_GATE(run_if);
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) out[b] = (in[b] + 2 * pad - k) / stride + 1;
}

}  // namespace

hipError_t launch_time_mean(const float* x, int B, int T, int C, int ld, float* out, int ldo, hipStream_t s,
                            const int* vlen) {
  hipLaunchKernelGGL(time_mean_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, s, x, B, T, C, ld, out, ldo,
                     vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_asp_stats(const float* x, int B, int T, int C, int ld, float eps, float* out, hipStream_t s,
                            const int* vlen) {
  hipLaunchKernelGGL(asp_stats_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, s, x, B, T, C, ld, eps, out,
                     vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_attn_pool(const float* logit, int ldl, const float* x, int ldx, int B, int T, int C, float eps,
                            float* out, hipStream_t s, const int* vlen) {
  hipLaunchKernelGGL(attn_pool_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, s, logit, ldl, x, ldx, B, T, C,
                     eps, out, vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_se_apply(const float* x, int ldx, const float* gate, int ldg, const float* res, int ldr, float* out,
                           int ldo, int B, int T, int C, hipStream_t s, int* range_flag) {
  if (C % 4 || ldx % 4 || ldg % 4 || ldr % 4 || ldo % 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(se_apply_kernel, dim3(grid_for((long long)B * T * C / 4)), dim3(256), 0, s, x, ldx, gate, ldg,
                     res, ldr, out, ldo, B, T, C, range_flag, launch_gate());
  return hipGetLastError();
}

hipError_t launch_cam_context(const float* x, int B, int T, int C, int ld, int seg, int nseg, float* out, int ldo,
                              hipStream_t s, const int* vlen) {
  hipLaunchKernelGGL(cam_context_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, s, x, B, T, C, ld, seg, nseg,
                     out, ldo, vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_cam_gate(const float* x, int B, int T, int C, int ld, int seg, int nseg, const float* w1, int k1p,
                          const float* b1, int red, const float* w2, int k2p, const float* b2, int growth, float* gate,
                          int ldg, float* segsum, hipStream_t s, const int* vlen) {
  if (C % 4 || C / 4 > 256 || ld % 4 || red <= 0 || red > 1024 || growth <= 0 || growth > 1024 || B <= 0 || nseg <= 0)
    return hipErrorInvalidValue;
  static const bool lean_off = std::getenv("SPK_CAM_GATE_LDS") != nullptr;   // A/B: the transposing kernel
  static const bool fuse_off = std::getenv("SPK_CAM_GATE_PAIR") != nullptr;  // A/B: segment sums as their own launch
  // the lean kernel's butterfly sums Q = 256 / red (or 256 / growth) adjacent lanes with
  // __shfl_xor, i.e. within one wave only when Q <= 64
  const bool lean = !lean_off && red >= 4 && growth >= 4 && 256 % red == 0 && 256 % growth == 0 && C % (4 * (256 / red)) == 0 &&
                    red % (4 * (256 / growth)) == 0 && C / (256 / red) <= 4 * CAM_WQ &&
                    red / (256 / growth) <= 4 * CAM_WQ && k1p % 4 == 0 && k2p % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(w1) & 15) == 0 && (reinterpret_cast<uintptr_t>(w2) & 15) == 0;
  const size_t lds_f = sizeof(float) * (4 * 256 + (size_t)nseg * C + C + CAM_SEGS * ((size_t)C + red));
  if (lean && !fuse_off && lds_f <= 64 * 1024) {
    hipLaunchKernelGGL(cam_gate_fused_kernel, dim3(B), dim3(256), lds_f, s, x, T, C, ld, seg, nseg, w1, k1p, b1, red,
                       w2, k2p, b2, growth, gate, ldg, vlen, launch_gate());
    return hipGetLastError();
  }
  hipLaunchKernelGGL(cam_segsum_kernel, dim3(nseg, B), dim3(256), 0, s, x, T, C, ld, seg, nseg, segsum, vlen, launch_gate());
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  if (lean) {
    const size_t lds_l = sizeof(float) * ((size_t)C + CAM_SEGS * ((size_t)C + red));
    hipLaunchKernelGGL(cam_gate_lean_kernel, dim3(B), dim3(256), lds_l, s, segsum, T, C, seg, nseg, w1, k1p, b1, red,
                       w2, k2p, b2, growth, gate, ldg, vlen, launch_gate());
    return hipGetLastError();
  }
  const size_t lds = sizeof(float) * ((size_t)C * (red + 1) + (size_t)red * (growth + 1) + C +
                                      CAM_SEGS * (C + red + 1024));
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cam_gate_kernel, dim3(B), dim3(1024), lds, s, segsum, T, C, seg, nseg, w1, k1p, b1, red, w2, k2p,
                     b2, growth, gate, ldg, vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_stats_pool(const float* x, int B, int T, int C, int ld, float* out, hipStream_t s, const int* vlen) {
  hipLaunchKernelGGL(stats_pool_kernel, dim3(grid_for((long long)B * C)), dim3(256), 0, s, x, B, T, C, ld, out, vlen, launch_gate());
  return hipGetLastError();
}

hipError_t launch_derive_len(const int* in, int* out, int B, int pad, int k, int stride, hipStream_t s) {
  hipLaunchKernelGGL(derive_len_kernel, dim3((B + 255) / 256), dim3(256), 0, s, in, out, B, pad, k, stride, launch_gate());
  return hipGetLastError();
}

}  // namespace spk
