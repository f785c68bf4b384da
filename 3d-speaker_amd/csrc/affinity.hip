// Pairwise cosine affinity on fp32 MFMA, gfx950 (used by
// speakerlab/process/cluster.py:59-62,150,218,232 and compute_score_metrics.py:110-114).
//
// out[i, j] = <a_i, b_j> / (|a_i| |b_j|), zero-norm rows divide by 1 like sklearn's
// normalize().  One 128x128 output tile per 256-thread block (4 waves, 64x64 each, as
// v_mfma_f32_32x32x2_f32 tiles), K = embedding dim streamed in 16-deep LDS tiles.  The
// row norms are accumulated by the loaders from the same registers that feed LDS, so the
// embeddings are read once per tile and the N x N matrix is written exactly once.
// 2*E FLOPs per 4-byte output => MFMA-bound for E >= 32.
#include <algorithm>
#include <climits>
#include <cmath>

#include "common.h"

namespace spk {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TB = 128, BK = 16, LROW = BK + 4;

// One 128 x 128 tile of A.B^T: accumulators in the MFMA C layout plus the row norms of the
// tile's A and B rows in nA / nB (zero norms -> 1, sklearn normalize()).
__device__ __forceinline__ void affinity_tile(const float* __restrict__ A, long long Na, const float* __restrict__ Bm,
                                              long long Nb, int E, long long m0, long long n0, float (*As)[TB * LROW],
                                              float (*Bs)[TB * LROW], float* nA, float* nB, f32x16 (&acc)[2][2]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
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
}

__global__ void __launch_bounds__(256)
cosine_affinity_kernel(const float* __restrict__ A, long long Na, const float* __restrict__ Bm, long long Nb, int E,
                       float* __restrict__ out, long long ldo) {
  __shared__ __attribute__((aligned(16))) float As[2][TB * LROW];
  __shared__ __attribute__((aligned(16))) float Bs[2][TB * LROW];
  __shared__ float nA[TB], nB[TB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const long long m0 = (long long)blockIdx.y * TB, n0 = (long long)blockIdx.x * TB;
  f32x16 acc[2][2];
  affinity_tile(A, Na, Bm, Nb, E, m0, n0, As, Bs, nA, nB, acc);
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


// ---- consumers: the affinity is reduced where it is produced, never materialised -----------
//
// Row-block top-k (each rank consumes its row block of the N x N cosine
// matrix locally).  Block (seg, rowtile) walks the column tiles of its segment: every tile
// is computed by affinity_tile, scaled by the norms and parked in LDS; thread (row, half)
// keeps a sorted top-K of the 64 columns of its half, ordered by (score desc, index asc) so
// the result is deterministic, and counts scores >= thr.  Per-(row, segment) partials are
// merged by cosine_topk_merge_kernel.
constexpr int KMAX = 8;
constexpr int SROW = TB + 1;   // score tile row stride (floats): rows on distinct banks

struct TopkArgs {
  int k;                 // 1..KMAX
  long long self_off;    // column n is row m's own entry when n == m + self_off (excluded)
  int has_self;
  float thr;             // counted: scores >= thr
  int nseg, tiles_per_seg;
  float* part_s;         // [nseg][Na][KMAX]
  long long* part_i;     // [nseg][Na][KMAX]
  long long* part_c;     // [nseg][Na]
};

__device__ __forceinline__ bool topk_better(float s, long long i, float t, long long j) {
  return s > t || (s == t && i < j);
}

// insert (s, i) into the sorted list ts/ti (best first) of length k; registers only
// (static indices: the list lives in VGPRs)
__device__ __forceinline__ void topk_insert(float (&ts)[KMAX], long long (&ti)[KMAX], int k, float s, long long i) {
  if (!topk_better(s, i, ts[k - 1], ti[k - 1])) return;
  bool placed = false;
#pragma unroll
  for (int q = KMAX - 1; q >= 0; --q) {
    if (q < k && !placed) {
      constexpr int dummy = 0;
      const int up = q > 0 ? q - 1 : dummy;
      if (q > 0 && topk_better(s, i, ts[up], ti[up])) {
        ts[q] = ts[up];
        ti[q] = ti[up];
      } else {
        ts[q] = s;
        ti[q] = i;
        placed = true;
      }
    }
  }
}

__global__ void __launch_bounds__(256)
cosine_topk_kernel(const float* __restrict__ A, long long Na, const float* __restrict__ Bm, long long Nb, int E,
                   TopkArgs t) {
  __shared__ __attribute__((aligned(16))) float As[2][TB * LROW];
  __shared__ __attribute__((aligned(16))) float Bs[2][TB * LROW];
  __shared__ float nA[TB], nB[TB];
  __shared__ float sc[TB * SROW];
  __shared__ float ms[TB][KMAX];
  __shared__ long long mi[TB][KMAX];
  __shared__ long long mc[TB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  const long long m0 = (long long)blockIdx.y * TB;
  const int seg = blockIdx.x;
  const long long ntn = (Nb + TB - 1) / TB;
  const long long c0 = (long long)seg * t.tiles_per_seg, c1 = min(ntn, c0 + t.tiles_per_seg);
  const int row = tid & (TB - 1), half = tid >> 7;
  const long long m = m0 + row;
  float ts[KMAX];
  long long ti[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) { ts[q] = -INFINITY; ti[q] = LLONG_MAX; }
  long long cnt = 0;
  for (long long ct = c0; ct < c1; ++ct) {
    const long long n0 = ct * TB;
    f32x16 acc[2][2];
    affinity_tile(A, Na, Bm, Nb, E, m0, n0, As, Bs, nA, nB, acc);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cl = wn * 64 + j * 32 + li;
      const float inb = nB[cl];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          sc[rl * SROW + cl] = acc[i][j][r] / (nA[rl] * inb);
        }
    }
    __syncthreads();
    if (m < Na) {
      const float* srow = sc + row * SROW + half * 64;
      for (int c = 0; c < 64; ++c) {
        const long long n = n0 + half * 64 + c;
        if (n >= Nb || (t.has_self && n == m + t.self_off)) continue;
        const float v = srow[c];
        cnt += v >= t.thr;
        topk_insert(ts, ti, t.k, v, n);
      }
    }
    __syncthreads();
  }
  // merge the two halves of each row
  if (half == 1) {
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { ms[row][q] = ts[q]; mi[row][q] = ti[q]; }
    mc[row] = cnt;
  }
  __syncthreads();
  if (half == 0 && m < Na) {
    for (int q = 0; q < t.k; ++q) topk_insert(ts, ti, t.k, ms[row][q], mi[row][q]);
    cnt += mc[row];
    const size_t o = ((size_t)seg * Na + m) * KMAX;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { t.part_s[o + q] = ts[q]; t.part_i[o + q] = ti[q]; }
    t.part_c[(size_t)seg * Na + m] = cnt;
  }
}

__global__ void cosine_topk_merge_kernel(long long Na, TopkArgs t, float* __restrict__ top_s,
                                         long long* __restrict__ top_i, long long* __restrict__ count) {
  const long long m = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Na) return;
  float ts[KMAX];
  long long ti[KMAX];
#pragma unroll
  for (int q = 0; q < KMAX; ++q) { ts[q] = -INFINITY; ti[q] = LLONG_MAX; }
  long long cnt = 0;
  for (int seg = 0; seg < t.nseg; ++seg) {
    const size_t o = ((size_t)seg * Na + m) * KMAX;
    for (int q = 0; q < t.k; ++q) topk_insert(ts, ti, t.k, t.part_s[o + q], t.part_i[o + q]);
    cnt += t.part_c[(size_t)seg * Na + m];
  }
  for (int q = 0; q < t.k; ++q) {
    if (top_s) top_s[m * t.k + q] = ts[q];
    if (top_i) top_i[m * t.k + q] = ti[q] == LLONG_MAX ? -1 : ti[q];
  }
  if (count) count[m] = cnt;
}

// Trial gather (compute_score_metrics.py:102-118): score[t] = cos(Ea[ia[t]], Eb[ib[t]]), one
// wave per trial, float4 per lane, the three sums reduced across the wave.  O(T * E) instead of
// the Ne x Nt affinity the reference's per-trial sklearn calls amount to.
__global__ void __launch_bounds__(256)
cosine_trials_kernel(const float* __restrict__ A, const float* __restrict__ Bm, int E, const long long* __restrict__ ia,
                     const long long* __restrict__ ib, long long T, float* __restrict__ out) {
  const long long tr = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (tr >= T) return;
  const float* a = A + ia[tr] * E;
  const float* b = Bm + ib[tr] * E;
  float d = 0.f, na = 0.f, nb = 0.f;
  for (int k = lane * 4; k < E; k += 256) {
    const f32x4 x = *reinterpret_cast<const f32x4*>(a + k);
    const f32x4 y = *reinterpret_cast<const f32x4*>(b + k);
    d += x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
    na += x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
    nb += y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    d += __shfl_xor(d, o, 64);
    na += __shfl_xor(na, o, 64);
    nb += __shfl_xor(nb, o, 64);
  }
  if (lane == 0) {
    const float sa = na == 0.f ? 1.f : sqrtf(na), sb = nb == 0.f ? 1.f : sqrtf(nb);
    out[tr] = d / (sa * sb);
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

int cosine_topk_nseg(long long Na, long long Nb) {
  const long long rt = (Na + TB - 1) / TB, ct = (Nb + TB - 1) / TB;
  long long nseg = (512 + rt - 1) / rt;                      // >= 2 blocks per CU
  nseg = std::max(1LL, std::min(nseg, ct));
  return (int)nseg;
}

size_t cosine_topk_workspace(long long Na, long long Nb) {
  const size_t nseg = cosine_topk_nseg(Na, Nb);
  return nseg * Na * (KMAX * (sizeof(float) + sizeof(long long)) + sizeof(long long));
}

hipError_t launch_cosine_topk(const float* A, long long Na, const float* B, long long Nb, int E, int k,
                              long long self_off, int has_self, float thr, void* ws, size_t ws_bytes, float* top_s,
                              long long* top_i, long long* count, hipStream_t s) {
  if (E <= 0 || E % 4 || Na < 0 || Nb <= 0 || k < 1 || k > KMAX) return hipErrorInvalidValue;
  if (Na == 0) return hipSuccess;
  if ((Na + TB - 1) / TB > 65535 || ws_bytes < cosine_topk_workspace(Na, Nb) || !ws) return hipErrorInvalidValue;
  TopkArgs t;
  t.k = k; t.self_off = self_off; t.has_self = has_self; t.thr = thr;
  t.nseg = cosine_topk_nseg(Na, Nb);
  const long long ct = (Nb + TB - 1) / TB;
  t.tiles_per_seg = (int)((ct + t.nseg - 1) / t.nseg);
  t.nseg = (int)((ct + t.tiles_per_seg - 1) / t.tiles_per_seg);
  char* p = static_cast<char*>(ws);
  t.part_s = reinterpret_cast<float*>(p);
  p += (size_t)t.nseg * Na * KMAX * sizeof(float);
  t.part_i = reinterpret_cast<long long*>(p);
  p += (size_t)t.nseg * Na * KMAX * sizeof(long long);
  t.part_c = reinterpret_cast<long long*>(p);
  hipLaunchKernelGGL(cosine_topk_kernel, dim3((unsigned)t.nseg, (unsigned)((Na + TB - 1) / TB)), dim3(256), 0, s, A, Na,
                     B, Nb, E, t);
  hipLaunchKernelGGL(cosine_topk_merge_kernel, dim3((unsigned)((Na + 255) / 256)), dim3(256), 0, s, Na, t, top_s, top_i,
                     count);
  return hipGetLastError();
}

hipError_t launch_cosine_trials(const float* A, const float* B, int E, const long long* ia, const long long* ib,
                                long long T, float* out, hipStream_t s) {
  if (E <= 0 || E % 4 || T < 0) return hipErrorInvalidValue;
  if (T == 0) return hipSuccess;
  if ((T + 3) / 4 > 0x7FFFFFFF) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cosine_trials_kernel, dim3((unsigned)((T + 3) / 4)), dim3(256), 0, s, A, B, E, ia, ib, T, out);
  return hipGetLastError();
}

}  // namespace spk
