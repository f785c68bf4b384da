// C ABI entry for the cosine-affinity kernel (affinity.hip).
#include "runtime.h"

namespace spk {

hipError_t launch_cosine_affinity(const float* A, long long Na, const float* B, long long Nb, int E, float* out,
                                  long long ldo, hipStream_t s);
size_t cosine_topk_workspace(long long Na, long long Nb);
hipError_t launch_cosine_topk(const float* A, long long Na, const float* B, long long Nb, int E, int k,
                              long long self_off, int has_self, float thr, void* ws, size_t ws_bytes, float* top_s,
                              long long* top_i, long long* count, hipStream_t s);
hipError_t launch_cosine_trials(const float* A, const float* B, int E, const long long* ia, const long long* ib,
                                long long T, float* out, hipStream_t s);

static int fail(const char* fn, hipError_t e) {
  set_error(std::string(fn) + ": " + hipGetErrorString(e));
  return e == hipErrorInvalidValue ? SPK_E_INVALID : SPK_E_HIP;
}

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

extern "C" int spk_cosine_topk_workspace_bytes(int64_t Na, int64_t Nb, size_t* bytes) {
  if (!bytes || Na < 0 || Nb < 0) {
    spk::set_error("spk_cosine_topk_workspace_bytes: bad arguments");
    return SPK_E_INVALID;
  }
  *bytes = Na == 0 || Nb == 0 ? 0 : spk::cosine_topk_workspace(Na, Nb);
  return SPK_OK;
}

extern "C" int spk_cosine_topk(const float* Ea, int64_t Na, const float* Eb, int64_t Nb, int32_t E,
                               const spk_affinity_consumer_t* c, void* stream) {
  if (!c || c->kind != SPK_CONSUME_TOPK) {
    spk::set_error("spk_cosine_topk: consumer kind must be SPK_CONSUME_TOPK");
    return SPK_E_INVALID;
  }
  hipError_t e = spk::launch_cosine_topk(Ea, Na, Eb, Nb, E, c->k, c->self_offset, c->exclude_self, c->threshold,
                                         c->workspace, c->workspace_bytes, c->top_scores,
                                         reinterpret_cast<long long*>(c->top_index),
                                         reinterpret_cast<long long*>(c->count_ge), reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? SPK_OK : spk::fail("spk_cosine_topk", e);
}

extern "C" int spk_cosine_trials(const float* Ea, const float* Eb, int32_t E, const int64_t* ia, const int64_t* ib,
                                 int64_t n_trials, float* scores, void* stream) {
  hipError_t e = spk::launch_cosine_trials(Ea, Eb, E, reinterpret_cast<const long long*>(ia),
                                           reinterpret_cast<const long long*>(ib), n_trials, scores,
                                           reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? SPK_OK : spk::fail("spk_cosine_trials", e);
}
