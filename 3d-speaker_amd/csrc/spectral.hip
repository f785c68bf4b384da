// Spectral-clustering preparation on the GPU (reference
// speakerlab/process/cluster.py SpectralCluster.p_pruning :64-77, get_laplacian :79-84,
// get_spec_embs :86-100).
//
//   p-pruning: in every row of the cosine affinity, the n_elems smallest entries become 0.
//     One workgroup per row: a 4-pass, 8-bit radix select over order-preserving uint32 keys
//     finds the n_elems-th smallest value; entries below it are zeroed and ties at it are
//     zeroed lowest index first (numpy's argsort leaves the order of ties unspecified).
//   Laplacian: M = (P + P^T) / 2 with a zero diagonal (32x32 tiles transposed through LDS),
//     L = diag(sum_j |M_ij|) - M; the row sums are a fixed-order block reduction, so the
//     result is deterministic.
//   Eigen-decomposition of the symmetric Laplacian: rocSOLVER ssyevd (all eigenpairs,
//     ascending) in place of ARPACK eigsh(which='SM').
#include <algorithm>
#include <map>
#include <mutex>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "../../include/spk_hip.h"
#include "common.h"
#include "runtime.h"

namespace spk {

namespace {

__device__ __forceinline__ unsigned sort_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int PT = 1024;   // threads per row-workgroup

__global__ void __launch_bounds__(PT) p_prune_kernel(const float* __restrict__ S, long long N, long long lds,
                                                     int n_elems, float* __restrict__ P, long long ldp) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_rank;
  __shared__ unsigned scan[PT];
  const long long row = blockIdx.x;
  const float* s = S + row * lds;
  float* p = P + row * ldp;
  const int tid = threadIdx.x;
  if (n_elems <= 0) {
    for (long long j = tid; j < N; j += PT) p[j] = s[j];
    return;
  }
  // ---- radix select of the n_elems-th smallest key (rank r = n_elems - 1)
  if (tid == 0) { s_prefix = 0; s_rank = (unsigned)(n_elems - 1); }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    const unsigned mask_hi = pass == 0 ? 0u : (0xFFFFFFFFu << (shift + 8));
    for (int i = tid; i < 256; i += PT) hist[i] = 0;
    __syncthreads();
    const unsigned prefix = s_prefix;
    for (long long j = tid; j < N; j += PT) {
      const unsigned k = sort_key(s[j]);
      if ((k & mask_hi) == (prefix & mask_hi)) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned r = s_rank, acc = 0;
      int b = 0;
      for (; b < 256; ++b) {
        if (acc + hist[b] > r) break;
        acc += hist[b];
      }
      s_rank = r - acc;         // rank within the chosen bin
      s_prefix = prefix | ((unsigned)b << shift);
    }
    __syncthreads();
  }
  const unsigned thr = s_prefix;
  // count keys strictly below thr (the radix passes only counted within the prefix path)
  unsigned less = 0;
  for (long long j = tid; j < N; j += PT) less += sort_key(s[j]) < thr ? 1u : 0u;
  scan[tid] = less;
  __syncthreads();
  for (int off = PT / 2; off > 0; off >>= 1) {
    if (tid < off) scan[tid] += scan[tid + off];
    __syncthreads();
  }
  const unsigned need = (unsigned)n_elems - scan[0];   // ties at thr to zero, lowest index first
  __syncthreads();
  // ---- write the pruned row, in index order chunk by chunk (ties need a running count)
  unsigned seen = 0;
  for (long long base = 0; base < N; base += PT) {
    const long long j = base + tid;
    const float v = j < N ? s[j] : 0.f;
    const unsigned k = sort_key(v);
    const unsigned eq = (j < N && k == thr) ? 1u : 0u;
    scan[tid] = eq;
    __syncthreads();
    // inclusive Hillis-Steele scan of the tie flags of this chunk
    for (int off = 1; off < PT; off <<= 1) {
      const unsigned add = tid >= off ? scan[tid - off] : 0u;
      __syncthreads();
      scan[tid] += add;
      __syncthreads();
    }
    const unsigned before = seen + scan[tid] - eq;       // ties at lower indices
    if (j < N) p[j] = (k < thr || (eq && before < need)) ? 0.f : v;
    seen += scan[PT - 1];
    __syncthreads();
  }
}

// L_ij = -(P_ij + P_ji) / 2 (i != j), L_ii = 0 for now
__global__ void sym_offdiag_kernel(const float* __restrict__ P, long long N, long long ldp, float* __restrict__ L,
                                   long long ldl) {
  __shared__ float t[32][33];
  const long long bi = blockIdx.y * 32LL, bj = blockIdx.x * 32LL;
  const int tx = threadIdx.x, ty = threadIdx.y;   // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const long long i = bj + r, j = bi + tx;        // the transposed tile P[bj.., bi..]
    t[r][tx] = (i < N && j < N) ? P[i * ldp + j] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const long long i = bi + r, j = bj + tx;
    if (i < N && j < N) L[i * ldl + j] = i == j ? 0.f : -(0.5f * (P[i * ldp + j] + t[tx][r]));
  }
}

// L_ii = sum_j |L_ij| (fixed-order block reduction: deterministic)
__global__ void __launch_bounds__(256) degree_kernel(float* __restrict__ L, long long N, long long ldl) {
  __shared__ float red[256];
  const long long i = blockIdx.x;
  float acc = 0.f;
  for (long long j = threadIdx.x; j < N; j += 256) acc += fabsf(L[i * ldl + j]);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) L[i * ldl + i] = red[0];
}

std::mutex g_blas_mu;
std::map<int, rocblas_handle> g_blas;

}  // namespace

}  // namespace spk

using namespace spk;

extern "C" {

int spk_spectral_laplacian(const float* S, int64_t N, int64_t lds, int32_t n_elems, float* L, int64_t ldl,
                           void* workspace, size_t workspace_bytes, void* stream) {
  if (!S || !L || N <= 0 || lds < N || ldl < N || n_elems < 0 || n_elems > N ||
      workspace_bytes < (size_t)N * N * sizeof(float) || !workspace) {
    set_error("spk_spectral_laplacian: invalid argument (workspace needs N*N floats)");
    return SPK_E_INVALID;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* P = reinterpret_cast<float*>(workspace);
  hipLaunchKernelGGL(p_prune_kernel, dim3((unsigned)N), dim3(PT), 0, s, S, (long long)N, (long long)lds, n_elems, P,
                     (long long)N);
  const unsigned nb = (unsigned)((N + 31) / 32);
  hipLaunchKernelGGL(sym_offdiag_kernel, dim3(nb, nb), dim3(32, 8), 0, s, P, (long long)N, (long long)N, L,
                     (long long)ldl);
  hipLaunchKernelGGL(degree_kernel, dim3((unsigned)N), dim3(256), 0, s, L, (long long)N, (long long)ldl);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("spk_spectral_laplacian: ") + hipGetErrorString(e));
    return SPK_E_HIP;
  }
  return SPK_OK;
}

int spk_symmetric_eig(float* A, int64_t N, int64_t lda, float* w, void* stream) {
  if (!A || !w || N <= 0 || lda < N || N > (1LL << 30)) {
    set_error("spk_symmetric_eig: invalid argument");
    return SPK_E_INVALID;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SPK_E_HIP;
  rocblas_handle h = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_blas_mu);
    auto it = g_blas.find(dev);
    if (it == g_blas.end()) {
      if (rocblas_create_handle(&h) != rocblas_status_success) {
        set_error("spk_symmetric_eig: rocblas_create_handle failed");
        return SPK_E_HIP;
      }
      g_blas[dev] = h;
    } else {
      h = it->second;
    }
    rocblas_set_stream(h, reinterpret_cast<hipStream_t>(stream));
    float* E = nullptr;
    rocblas_int* info = nullptr;
    if (hipMalloc(&E, sizeof(float) * N) != hipSuccess || hipMalloc(&info, sizeof(rocblas_int)) != hipSuccess) {
      if (E) (void)hipFree(E);
      set_error("spk_symmetric_eig: hipMalloc failed");
      return SPK_E_HIP;
    }
    // row-major A is its own column-major transpose (symmetric); eigenvector k comes back
    // as column k of the column-major matrix = row k of the caller's row-major buffer
    const rocblas_status st = rocsolver_ssyevd(h, rocblas_evect_original, rocblas_fill_upper, (rocblas_int)N, A,
                                               (rocblas_int)lda, w, E, info);
    rocblas_int hinfo = 0;
    const hipError_t ce = hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost,
                                         reinterpret_cast<hipStream_t>(stream));
    const hipError_t se = hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream));
    (void)hipFree(E);
    (void)hipFree(info);
    if (st != rocblas_status_success || ce != hipSuccess || se != hipSuccess) {
      set_error("spk_symmetric_eig: rocsolver_ssyevd failed");
      return SPK_E_HIP;
    }
    if (hinfo != 0) {
      set_error("spk_symmetric_eig: ssyevd did not converge (info " + std::to_string(hinfo) + ")");
      return SPK_E_HIP;
    }
  }
  return SPK_OK;
}

}  // extern "C"
