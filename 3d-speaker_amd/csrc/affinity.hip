// Pairwise cosine affinity on fp32 MFMA, gfx950 (used by
// speakerlab/process/cluster.py:59-62,150,218,232 and compute_score_metrics.py:110-114).
//
// out[i, j] = <a_i, b_j> / (|a_i| |b_j|), zero-norm rows divide by 1 like sklearn's
// normalize().  One 128x128 output tile per 256-thread block (4 waves, 64x64 each, as
// v_mfma_f32_32x32x2_f32 tiles), K = embedding dim streamed in 16-deep LDS tiles.  The
// row norms are accumulated by the loaders from the same registers that feed LDS, so the
// embeddings are read once per tile and the N x N matrix is written exactly once.
// 2*E FLOPs per 4-byte output => MFMA-bound for E >= 32.
#include "common.h"

namespace spk {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TB = 128, BK = 16, LROW = BK + 4;

__global__ void __launch_bounds__(256)
cosine_affinity_kernel(const float* __restrict__ A, long long Na, const float* __restrict__ Bm, long long Nb, int E,
                       float* __restrict__ out, long long ldo) {
  __shared__ __attribute__((aligned(16))) float As[2][TB * LROW];
  __shared__ __attribute__((aligned(16))) float Bs[2][TB * LROW];
  __shared__ float nA[TB], nB[TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.y * TB, n0 = (long long)blockIdx.x * TB;
  const int kq = tid & 3;
  const int nkt = (E + BK - 1) / BK;
  f32x4 ra[2], rb[2];
  float ssa[2] = {0.f, 0.f}, ssb[2] = {0.f, 0.f};
  auto load = [&](int kt) {
    const int k = kt * BK + kq * 4;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const long long ia = m0 + (tid >> 2) + 64 * r, ib = n0 + (tid >> 2) + 64 * r;
      f32x4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
      if (ia < Na && k < E) va = *reinterpret_cast<const f32x4*>(A + ia * E + k);
      if (ib < Nb && k < E) vb = *reinterpret_cast<const f32x4*>(Bm + ib * E + k);
      ra[r] = va; rb[r] = vb;
      ssa[r] += va[0] * va[0] + va[1] * va[1] + va[2] * va[2] + va[3] * va[3];
      ssb[r] += vb[0] * vb[0] + vb[1] * vb[1] + vb[2] * vb[2] + vb[3] * vb[3];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      *reinterpret_cast<f32x4*>(&As[buf][((tid >> 2) + 64 * r) * LROW + kq * 4]) = ra[r];
      *reinterpret_cast<f32x4*>(&Bs[buf][((tid >> 2) + 64 * r) * LROW + kq * 4]) = rb[r];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int li = lane & 31, lh = lane >> 5;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) load(kt + 1);
    f32x4 af[2][2], bf[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* p = &As[buf][(wm * 64 + i * 32 + li) * LROW + lh * 8];
      af[i][0] = *reinterpret_cast<const f32x4*>(p);
      af[i][1] = *reinterpret_cast<const f32x4*>(p + 4);
      const float* q = &Bs[buf][(wn * 64 + i * 32 + li) * LROW + lh * 8];
      bf[i][0] = *reinterpret_cast<const f32x4*>(q);
      bf[i][1] = *reinterpret_cast<const f32x4*>(q + 4);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s >> 2][s & 3], bf[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
    if (kt + 1 < nkt) store(buf ^ 1);
    __syncthreads();
  }
  // row norms: the 4 threads of a row (kq = 0..3) are adjacent lanes
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float a = ssa[r], b = ssb[r];
    a += __shfl_xor(a, 1, 64); a += __shfl_xor(a, 2, 64);
    b += __shfl_xor(b, 1, 64); b += __shfl_xor(b, 2, 64);
    if (kq == 0) {
      const float na = sqrtf(a), nb = sqrtf(b);
      nA[(tid >> 2) + 64 * r] = na == 0.f ? 1.f : na;
      nB[(tid >> 2) + 64 * r] = nb == 0.f ? 1.f : nb;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wn * 64 + j * 32 + li;
    const long long n = n0 + cl;
    if (n >= Nb) continue;
    const float inb = nB[cl];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const long long m = m0 + rl;
        if (m < Na) out[m * ldo + n] = acc[i][j][r] / (nA[rl] * inb);
      }
  }
}

}  // namespace

hipError_t launch_cosine_affinity(const float* A, long long Na, const float* B, long long Nb, int E, float* out,
                                  long long ldo, hipStream_t s) {
  if (E <= 0 || E % 4 || Na < 0 || Nb < 0 || ldo < Nb) return hipErrorInvalidValue;
  if (Na == 0 || Nb == 0) return hipSuccess;
  if ((Na + TB - 1) / TB > 65535) return hipErrorInvalidValue;
  dim3 grid((unsigned)((Nb + TB - 1) / TB), (unsigned)((Na + TB - 1) / TB));
  hipLaunchKernelGGL(cosine_affinity_kernel, grid, dim3(256), 0, s, A, Na, B, Nb, E, out, ldo);
  return hipGetLastError();
}

}  // namespace spk
