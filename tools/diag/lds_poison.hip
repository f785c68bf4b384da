// Diagnostic only (never linked into libspk_hip): fill every CU's LDS with a poison value,
// again and again, from many short blocks, so that a kernel of the library that reads LDS
// it has not written sees the poison instead of the previous kernel's leftovers.
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(256) lds_poison_kernel(float value) {
  extern __shared__ float lds[];
  const int n = 160 * 1024 / 4;
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = value;
  __syncthreads();
}

extern "C" int lds_poison(void* stream, float value, int blocks, int reps) {
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), 160 * 1024, (hipStream_t)stream, value);
  return (int)hipGetLastError();
}
