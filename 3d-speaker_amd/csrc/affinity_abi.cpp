// C ABI entry for the cosine-affinity kernel (affinity.hip).
#include "runtime.h"

namespace spk {

hipError_t launch_cosine_affinity(const float* A, long long Na, const float* B, long long Nb, int E, float* out,
                                  long long ldo, hipStream_t s);




}  // namespace spk

extern "C" int spk_cosine_affinity(const float* Ea, int64_t Na, const float* Eb, int64_t Nb, int32_t E, float* out,
                                   int64_t ldo, void* stream) {
  hipError_t e = spk::launch_cosine_affinity(Ea, Na, Eb, Nb, E, out, ldo, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) {
    spk::set_error(std::string("spk_cosine_affinity: ") + hipGetErrorString(e));
    return e == hipErrorInvalidValue ? SPK_E_INVALID : SPK_E_HIP;
  }
  return SPK_OK;
}
