// TEST INFRASTRUCTURE ONLY — host emulation of libspk_hip's kernel *contracts*.
//
// Built by tests/emu/Makefile into tests/emu/libspk_emu.so together with the unmodified
// executor sources (runtime.cpp, eres2net.cpp, ...), so the launch plans, weight folding
// and packing, channel layouts and workspace aliasing of the real library can be checked
// against the oracle on a machine without a GPU.  "Device" pointers are host pointers.
// It is never loaded by the product package; the GPU tests exercise the real kernels.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#include "../../3d-speaker_amd/csrc/tdnn_ops.h"

#include "../../3d-speaker_amd/csrc/common.h"
#include "../../include/spk_hip.h"
#include "../../3d-speaker_amd/csrc/fbank.h"
#include "../../3d-speaker_amd/csrc/misc.h"
#include "../../3d-speaker_amd/csrc/aff.h"
#include "../../3d-speaker_amd/csrc/res2block.h"

namespace spk {

// launches of the gated exact plan do nothing unless the forward's range word is set
// (common.h SPK_GATE; the gate pointer is host memory here)
#define EMU_GATE() do { if (const int* g_ = spk::launch_gate()) { if (*g_ == 0) return hipSuccess; } } while (0)

static float act_f(float v, int act) {
  switch (act) {
    case ACT_RELU: return v > 0.f ? v : 0.f;
    case ACT_HTANH: return std::fmin(std::fmax(v, 0.f), 20.f);
    case ACT_SILU: return v / (1.f + std::exp(-v));
    case ACT_SIGMOID: return 1.f / (1.f + std::exp(-v));
    case ACT_TANH: return std::tanh(v);
    default: return v;
  }
}

static float epilogue(const ConvDesc& d, int m, int n, float v) {
  if (d.bias) v += d.bias[n];
  if (d.rowbias) v += d.rowbias[(size_t)(m / (d.Ho * d.Wo)) * d.rowbias_ld + n];
  if (d.res) v += d.res[(size_t)m * d.ldr + n];
  if (d.affx) {
    const float t = 1.0f + std::tanh(v);
    return d.affx[(size_t)m * d.ldx + n] * t + d.affy[(size_t)m * d.ldy + n] * (2.0f - t);
  }
  v = act_f(v, d.act);
  if (d.post_scale) v = v * d.post_scale[n] + d.post_shift[n];
  v = act_f(v, d.act2);
  if (d.gate) {
    const int wo = m % d.Wo, img = m / (d.Wo * d.Ho);
    v *= d.gate[((size_t)img * d.gate_nseg + wo / d.gate_seg) * d.gate_ld + n];
  }
  return row_masked(d, m) ? 0.f : v;
}

static void emu_range_note(int* flag, float v) {   // common.h range guard: max of the float bits
  const float a = std::fabs(v);
  if (flag && a >= kRangeLimit) {
    int bits;
    std::memcpy(&bits, &a, sizeof(bits));
    if (bits > *flag) *flag = bits;
  }
}

hipError_t launch_conv(const ConvDesc& d, hipStream_t) {
  EMU_GATE();
  if (d.s0.cin % 4 || d.s0.ld % 4 || d.Kp % 16 || (d.osplit ? (d.osplit % 4 || d.ldo < d.osplit) : d.ldo < d.N) || d.K > d.Kp) return hipErrorInvalidValue;
  const int M = d.nimg * d.Ho * d.Wo;
  const int K0 = d.s0.kh * d.s0.kw * d.s0.cin;
  std::vector<float> a(d.Kp);
  for (int m = 0; m < M; ++m) {
    const int wo = m % d.Wo, ho = (m / d.Wo) % d.Ho, img = m / (d.Wo * d.Ho);
    for (int k = 0; k < d.Kp; ++k) {
      float v = 0.f;
      if (k < K0) {
        // K order (common.h ConvDesc::kcb): (tap, c) or 32-channel blocks outer, taps inner
        const int taps = d.s0.kh * d.s0.kw;
        const int tap = d.kcb ? (k / 32) % taps : k / d.s0.cin;
        const int c = d.kcb ? (k / 32 / taps) * 32 + k % 32 : k % d.s0.cin;
        const int ky = tap / d.s0.kw, kx = tap % d.s0.kw;
        int hi = ho * d.s0.sh - d.s0.ph + ky * d.s0.dh;
        int wi = wo * d.s0.sw - d.s0.pw + kx * d.s0.dw;
        if (d.s0.reflect) {
          hi = hi < 0 ? -hi : (hi >= d.s0.H ? 2 * d.s0.H - 2 - hi : hi);
          wi = wi < 0 ? -wi : (wi >= d.s0.W ? 2 * d.s0.W - 2 - wi : wi);
        }
        if (hi >= 0 && hi < d.s0.H && wi >= 0 && wi < d.s0.W && (!d.s0.vlen || wi < d.s0.vlen[img])) {
          const size_t pix = (size_t)(img * d.s0.H + hi) * d.s0.W + wi;
          v = d.s0.p[pix * d.s0.ld + c];
          if (d.s0.p2) v += d.s0.p2[pix * d.s0.ld2 + c];
          if (d.s0.pre_scale) v = std::fmax(v * d.s0.pre_scale[c] + d.s0.pre_shift[c], 0.f);
        }
      } else if (d.s1.p && k - K0 < d.s1.cin) {
        const int c = k - K0;
        const size_t pix = (size_t)(img * d.s1.H + ho * d.s1.sh) * d.s1.W + wo * d.s1.sw;
        v = d.s1.p[pix * d.s1.ld + c];
      }
      a[k] = v;
    }
    for (int n = 0; n < d.N; ++n) {
      const float* w = d.w + (size_t)n * d.Kp;
      double acc = 0.0;
      for (int k = 0; k < d.Kp; ++k) acc += (double)a[k] * w[k];
      {
        const float o = epilogue(d, m, n, (float)acc);
        emu_range_note(d.range_flag, o);
        *out_at(d, m, n) = o;
      }
    }
  }
  return hipSuccess;
}

std::string conv_kernel_name(const ConvDesc&) { return "emu_conv"; }

// fused AFF (aff.hip contract): h = SiLU(W1 [x|y] + b1), z = W2 h + b2,
// out = x (1 + tanh z) + y (1 - tanh z); fp32 weights, double accumulation
bool aff_x3_supported(int cp, int nmid) { return (nmid == 32 || nmid == 64) && cp % 8 == 0 && cp >= 8 && cp <= 208; }
std::string aff_x3_kernel_name(int, int nmid) { return "emu_aff<" + std::to_string(nmid / 32) + ">"; }
hipError_t launch_aff_x3(const AffDesc& a, hipStream_t) {
  EMU_GATE();
  if (!aff_x3_supported(a.cp, a.nmid) || a.kp1 < 2 * a.cp || a.kp2 < a.nmid) return hipErrorInvalidValue;
  std::vector<double> h(a.nmid);
  for (int m = 0; m < a.M; ++m) {
    const float* x = a.x + (size_t)m * a.ldx;
    const float* y = a.y + (size_t)m * a.ldy;
    for (int j = 0; j < a.nmid; ++j) {
      double acc = a.b1[j];
      const float* w = a.w1 + (size_t)j * a.kp1;
      for (int k = 0; k < a.cp; ++k) acc += (double)w[k] * x[k] + (double)w[a.cp + k] * y[k];
      const float v = (float)acc;
      h[j] = v / (1.0f + std::exp(-v));
    }
    for (int n = 0; n < a.cp; ++n) {
      double acc = a.b2[n];
      const float* w = a.w2 + (size_t)n * a.kp2;
      for (int j = 0; j < a.nmid; ++j) acc += (double)w[j] * h[j];
      const float t = 1.0f + std::tanh((float)acc);
      a.out[(size_t)m * a.ldo + n] = x[n] * t + y[n] * (2.0f - t);
    }
  }
  return hipSuccess;
}

// the emulated GEMM reads the fp32 weights; the split planes are not needed on the host
hipError_t launch_split_f16(const float*, uint16_t*, uint16_t*, size_t, hipStream_t) {
  EMU_GATE(); return hipSuccess; }
// nor the fragment-order copy of the LDS-DMA GEMM (conv_gemm_f.hip)
size_t frag_halves(int N, int Kp) { return (size_t)Kp * (size_t)((N + 255) / 256 * 256) * 2; }
hipError_t launch_pack_frag(const uint16_t*, const uint16_t*, int, int, uint16_t*, hipStream_t) { return hipSuccess; }


hipError_t launch_word_reset(int* w, hipStream_t) {
  *w = 0;
  return hipSuccess;
}

hipError_t launch_range_check(const float* x, size_t n, int* flag, hipStream_t) {
  EMU_GATE();
  for (size_t i = 0; i < n; ++i) emu_range_note(flag, x[i]);
  return hipSuccess;
}

hipError_t launch_stem_conv3x3(const float* feats, int B, int T, int F, const float* w, const float* bias, int cout,
                               int act, int wstride, float* out, int ldo, hipStream_t, const int* vlen, int* range_flag) {
  EMU_GATE();
  for (int b = 0; b < B; ++b) {
    const int Tb = vlen ? vlen[b] : T;
    for (int f = 0; f < F; ++f)
      for (int t = 0; t < T; ++t)
        for (int c = 0; c < cout; ++c) {
          double acc = 0.0;
          for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) {
              const int ff = f + dy - 1, tt = t + dx - 1;
              if (ff >= 0 && ff < F && tt >= 0 && tt < Tb) acc += (double)feats[((size_t)b * T + tt) * F + ff] * w[c * wstride + dy * 3 + dx];
            }
          float v = (float)acc + bias[c];
          const float o = t >= Tb ? 0.f : (act == ACT_RELU ? std::fmax(v, 0.f) : v);
          emu_range_note(range_flag, o);
          out[(((size_t)b * F + f) * T + t) * ldo + c] = o;
        }
  }
  return hipSuccess;
}

hipError_t launch_tstp(const float* x, int B, int H, int W, int C, int ld, float eps, int unbiased, float* out,
                       hipStream_t, int parts) {
  EMU_GATE();
  const int np = (parts & 1) + ((parts >> 1) & 1);
  for (int b = 0; b < B; ++b)
    for (int h = 0; h < H; ++h)
      for (int c = 0; c < C; ++c) {
        double s = 0, q = 0;
        for (int t = 0; t < W; ++t) s += x[((size_t)(b * H + h) * W + t) * ld + c];
        const double mean = s / W;
        for (int t = 0; t < W; ++t) {
          const double dl = x[((size_t)(b * H + h) * W + t) * ld + c] - mean;
          q += dl * dl;
        }
        const double var = q / (unbiased ? W - 1 : W);
        if (parts & 1) out[(size_t)b * np * H * C + h * C + c] = (float)mean;
        if (parts & 2) out[(size_t)b * np * H * C + (parts & 1) * H * C + h * C + c] = (float)std::sqrt(var + eps);
      }
  return hipSuccess;
}

hipError_t launch_astp_pool(const float* logit, int ldl, const float* x, int ldx, int B, int F, int T, int C, float* out,
                            hipStream_t) {
  EMU_GATE();
  for (int b = 0; b < B; ++b)
    for (int f = 0; f < F; ++f)
      for (int c = 0; c < C; ++c) {
        double mx = -1e300;
        for (int t = 0; t < T; ++t) mx = std::max(mx, (double)logit[((size_t)b * T + t) * ldl + f * C + c]);
        double sw = 0, s1 = 0, s2 = 0;
        for (int t = 0; t < T; ++t) {
          const double w = std::exp((double)logit[((size_t)b * T + t) * ldl + f * C + c] - mx);
          const double v = x[((size_t)(b * F + f) * T + t) * ldx + c];
          sw += w; s1 += w * v; s2 += w * v * v;
        }
        const double mean = s1 / sw, var = s2 / sw - mean * mean;
        out[(size_t)b * 2 * F * C + f * C + c] = (float)mean;
        out[(size_t)b * 2 * F * C + F * C + f * C + c] = (float)std::sqrt(std::max(var, 1e-10));
      }
  return hipSuccess;
}

hipError_t launch_fbank(const float*, const int64_t*, int, float*, const int64_t*, int, int, const FbankTables*, int,
                        hipStream_t, int) {
  EMU_GATE();
  return hipErrorNotSupported;
}

bool conv_use_x3() {
  const char* e = std::getenv("SPK_CONV_MFMA");
  return !(e && std::string(e) == "f32");
}

// fused Res2Net block (res2block.hip), the kernels' contract in double
// precision: conv1 + bn1 + Hardtanh -> s0 | s1 (slices padded to SW = 32 or 64 channels),
// y0 = Ht(conv3x3(s0)), y1 = Ht(conv3x3(y0 + s1)), out = Ht(conv3(cat(y0, y1)) + x) -- or,
// with the projection shortcut, Ht(conv3(cat(y0, y1, x))) -- zero padding at the edges; conv1
// and the shortcut read input pixel (s y, s x) for output pixel (y, x) (stride s)
bool res2_block_supported(const Res2Desc& d) {
  const int co = d.Cout ? d.Cout : d.C;
  const int hin = d.Hin ? d.Hin : d.H, win = d.Win ? d.Win : d.W;
  const bool st1 = d.stride == 1 && hin == d.H && win == d.W;
  const bool st2 = d.stride == 2 && (hin - 1) / 2 + 1 == d.H && (win - 1) / 2 + 1 == d.W;
  const bool s1 = st1 && (d.proj ? (d.C == 64 && co == 128) : (d.C == 128 && co == 128)) && d.width >= 1 && d.width <= 32;
  const bool s2 = (d.proj ? (st2 && d.C == 128) : (st1 && d.C == 256)) && co == 256 && d.width > 32 && d.width <= 64;
  return (s1 || s2) && d.w1 && d.wa && d.wb && d.w3 && d.b1 && d.ba && d.bb && d.b3;
}
std::string res2_block_kernel_name(const Res2Desc& d) { return "emu_res2_block<" + std::to_string(d.C) + ">"; }
hipError_t launch_res2_block(const Res2Desc& d, hipStream_t) {
  EMU_GATE();
  if (!res2_block_supported(d) || d.x == d.out) return hipErrorInvalidValue;
  const int SW = d.width <= 32 ? 32 : 64;
  const int H = d.H, W = d.W, C = d.C, CO = d.Cout ? d.Cout : d.C, K3 = d.proj ? 2 * SW + C : 2 * SW;
  const int S = d.stride, Hin = d.Hin ? d.Hin : H, Win = d.Win ? d.Win : W;
  auto ht = [](double v) { return std::min(std::max(v, 0.0), 20.0); };
  std::vector<double> t1((size_t)H * W * 2 * SW), y0((size_t)H * W * SW), sp((size_t)H * W * SW), y1((size_t)H * W * SW);
  auto conv3 = [&](const std::vector<double>& in, const float* w, const float* b, std::vector<double>& out) {
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        for (int n = 0; n < SW; ++n) {
          double acc = b[n];
          for (int tap = 0; tap < 9; ++tap) {
            const int yy = y + tap / 3 - 1, xx = x + tap % 3 - 1;
            if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
            const double* iv = &in[((size_t)yy * W + xx) * SW];
            for (int c = 0; c < SW; ++c) acc += (double)w[(size_t)n * 9 * SW + tap * SW + c] * iv[c];
          }
          out[((size_t)y * W + x) * SW + n] = ht(acc);
        }
  };
  for (int img = 0; img < d.nimg; ++img) {
    const float* xin = d.x + (size_t)img * Hin * Win * C;
    float* oi = d.out + (size_t)img * H * W * CO;
    auto xi_at = [&](size_t p) { return xin + ((size_t)(p / W) * S * Win + (p % W) * S) * C; };
    for (size_t p = 0; p < (size_t)H * W; ++p)
      for (int n = 0; n < 2 * SW; ++n) {
        double acc = d.b1[n];
        for (int k = 0; k < C; ++k) acc += (double)d.w1[(size_t)n * C + k] * xi_at(p)[k];
        t1[p * 2 * SW + n] = ht(acc);
      }
    std::vector<double> s0((size_t)H * W * SW);
    for (size_t p = 0; p < (size_t)H * W; ++p)
      for (int c = 0; c < SW; ++c) s0[p * SW + c] = t1[p * 2 * SW + c];
    conv3(s0, d.wa, d.ba, y0);
    for (size_t p = 0; p < (size_t)H * W; ++p)
      for (int c = 0; c < SW; ++c) sp[p * SW + c] = y0[p * SW + c] + t1[p * 2 * SW + SW + c];
    conv3(sp, d.wb, d.bb, y1);
    for (size_t p = 0; p < (size_t)H * W; ++p)
      for (int n = 0; n < CO; ++n) {
        double acc = d.b3[n] + (d.proj ? 0.0 : xi_at(p)[n]);
        for (int c = 0; c < SW; ++c)
          acc += (double)d.w3[(size_t)n * K3 + c] * y0[p * SW + c] + (double)d.w3[(size_t)n * K3 + SW + c] * y1[p * SW + c];
        if (d.proj)
          for (int c = 0; c < C; ++c) acc += (double)d.w3[(size_t)n * K3 + 2 * SW + c] * xi_at(p)[c];
        oi[p * CO + n] = (float)ht(acc);
      }
  }
  return hipSuccess;
}

// affinity consumers (affinity.hip): GPU-only, not part of any launch plan
size_t cosine_topk_workspace(long long, long long) { return 0; }
hipError_t launch_cosine_topk(const float*, long long, const float*, long long, int, int, long long, int, float, void*,
                              size_t, float*, long long*, long long*, hipStream_t) {
  EMU_GATE();
  return hipErrorNotSupported;
}
hipError_t launch_cosine_trials(const float*, const float*, int, const long long*, const long long*, long long, float*,
                                hipStream_t) {
  EMU_GATE();
  return hipErrorNotSupported;
}

hipError_t launch_cosine_affinity(const float* A, long long Na, const float* B, long long Nb, int E, float* out,
                                  long long ldo, hipStream_t) {
  EMU_GATE();
  for (long long i = 0; i < Na; ++i)
    for (long long j = 0; j < Nb; ++j) {
      double d = 0, na = 0, nb = 0;
      for (int e = 0; e < E; ++e) {
        d += (double)A[i * E + e] * B[j * E + e];
        na += (double)A[i * E + e] * A[i * E + e];
        nb += (double)B[j * E + e] * B[j * E + e];
      }
      na = na == 0 ? 1 : std::sqrt(na);
      nb = nb == 0 ? 1 : std::sqrt(nb);
      out[i * ldo + j] = (float)(d / (na * nb));
    }
  return hipSuccess;
}

}  // namespace spk

// ---- HIP runtime API stubs (host memory stands in for device memory)
extern "C" {
hipError_t hipMalloc(void** p, size_t n) { *p = std::malloc(n ? n : 1); return *p ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipFree(void* p) { std::free(p); return hipSuccess; }
hipError_t hipDeviceSynchronize(void) { return hipSuccess; }
// graph replay is not emulated (emu_runner sets SPK_GRAPH=0); these only satisfy the linker
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t) {
  std::memcpy(d, s, n);
  return hipSuccess;
}
hipError_t hipStreamCreateWithFlags(hipStream_t*, unsigned int) { return hipErrorNotSupported; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
hipError_t hipStreamBeginCapture(hipStream_t, hipStreamCaptureMode) { return hipErrorNotSupported; }
hipError_t hipStreamEndCapture(hipStream_t, hipGraph_t*) { return hipErrorNotSupported; }
hipError_t hipGraphDebugDotPrint(hipGraph_t, const char*, unsigned int) { return hipErrorNotSupported; }
hipError_t hipGraphInstantiate(hipGraphExec_t*, hipGraph_t, hipGraphNode_t*, char*, size_t) {
  return hipErrorNotSupported;
}
hipError_t hipGraphDestroy(hipGraph_t) { return hipSuccess; }
hipError_t hipGraphExecDestroy(hipGraphExec_t) { return hipSuccess; }
hipError_t hipGraphLaunch(hipGraphExec_t, hipStream_t) { return hipErrorNotSupported; }
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) { std::memcpy(d, s, n); return hipSuccess; }
hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "hipSuccess" : "emulated hip error"; }
hipError_t hipEventCreate(hipEvent_t* e) { *e = nullptr; return hipSuccess; }
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { *e = nullptr; return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) { return hipSuccess; }
hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) { *ms = 0.f; return hipSuccess; }
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t) { std::memset(p, v, n); return hipSuccess; }
hipError_t hipMemset(void* p, int v, size_t n) { std::memset(p, v, n); return hipSuccess; }
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
// the spectral entry points (csrc/spectral.hip) are not emulated: their parity is a -m gpu test
int spk_spectral_laplacian(const float*, int64_t, int64_t, int32_t, float*, int64_t, void*, size_t, void*) {
  return SPK_E_UNSUPPORTED;
}
int spk_symmetric_eig(float*, int64_t, int64_t, float*, void*) { return SPK_E_UNSUPPORTED; }
}

// ---- TDNN reductions (contracts of csrc/tdnn_ops.h)
namespace spk {
static int vframes(const int* vlen, int b, int T) { return vlen ? std::min(std::max(vlen[b], 1), T) : T; }
hipError_t launch_time_mean(const float* x, int B, int T, int C, int ld, float* out, int ldo, hipStream_t,
                            const int* vlen) {
  EMU_GATE();
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c) {
      const int Tb = vframes(vlen, b, T);
      double s = 0;
      for (int t = 0; t < Tb; ++t) s += x[((size_t)b * T + t) * ld + c];
      out[(size_t)b * ldo + c] = (float)(s / Tb);
    }
  return hipSuccess;
}
hipError_t launch_asp_stats(const float* x, int B, int T, int C, int ld, float eps, float* out, hipStream_t,
                            const int* vlen) {
  EMU_GATE();
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c) {
      const int Tb = vframes(vlen, b, T);
      double s = 0, q = 0;
      for (int t = 0; t < Tb; ++t) s += x[((size_t)b * T + t) * ld + c];
      const double mean = s / Tb;
      for (int t = 0; t < Tb; ++t) { const double d = x[((size_t)b * T + t) * ld + c] - mean; q += d * d / Tb; }
      out[(size_t)b * 2 * C + c] = (float)mean;
      out[(size_t)b * 2 * C + C + c] = (float)std::sqrt(std::fmax(q, (double)eps));
    }
  return hipSuccess;
}
hipError_t launch_attn_pool(const float* l, int ldl, const float* x, int ldx, int B, int T, int C, float eps,
                            float* out, hipStream_t, const int* vlen) {
  EMU_GATE();
  std::vector<double> p(T);
  for (int b = 0; b < B; ++b)
    for (int c = 0; c < C; ++c) {
      const int Tb = vframes(vlen, b, T);
      double mx = -1e300, den = 0, mean = 0, q = 0;
      for (int t = 0; t < Tb; ++t) mx = std::fmax(mx, l[((size_t)b * T + t) * ldl + c]);
      for (int t = 0; t < Tb; ++t) { p[t] = std::exp(l[((size_t)b * T + t) * ldl + c] - mx); den += p[t]; }
      for (int t = 0; t < Tb; ++t) mean += p[t] / den * x[((size_t)b * T + t) * ldx + c];
      for (int t = 0; t < Tb; ++t) { const double d = x[((size_t)b * T + t) * ldx + c] - mean; q += p[t] / den * d * d; }
      out[(size_t)b * 2 * C + c] = (float)mean;
      out[(size_t)b * 2 * C + C + c] = (float)std::sqrt(std::fmax(q, (double)eps));
    }
  return hipSuccess;
}
hipError_t launch_se_apply(const float* x, int ldx, const float* g, int ldg, const float* r, int ldr, float* out,
                           int ldo, int B, int T, int C, hipStream_t, int* range_flag) {
  EMU_GATE();
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < T; ++t)
      for (int c = 0; c < C; ++c) {
        const size_t row = (size_t)b * T + t;
        out[row * ldo + c] = x[row * ldx + c] * g[(size_t)b * ldg + c] + r[row * ldr + c];
        emu_range_note(range_flag, out[row * ldo + c]);
      }
  return hipSuccess;
}
hipError_t launch_cam_gate(const float* x, int B, int T, int C, int ld, int seg, int nseg, const float* w1, int k1p,
                          const float* b1, int red, const float* w2, int k2p, const float* b2, int growth, float* gate,
                          int ldg, float*, hipStream_t, const int* vlen) {
  EMU_GATE();
  std::vector<double> ctx(C), h(red);
  for (int b = 0; b < B; ++b) {
    const int Tb = vlen ? std::min(std::max(vlen[b], 1), T) : T;
    for (int s = 0; s < nseg; ++s) {
      const int t0 = s * seg, t1 = std::min(Tb, t0 + seg);
      for (int c = 0; c < C; ++c) {
        double tot = 0, a = 0;
        for (int t = 0; t < Tb; ++t) tot += x[((size_t)b * T + t) * ld + c];
        for (int t = t0; t < t1; ++t) a += x[((size_t)b * T + t) * ld + c];
        ctx[c] = t1 > t0 ? tot / Tb + a / (t1 - t0) : 0.0;
      }
      for (int j = 0; j < red; ++j) {
        double v = b1 ? b1[j] : 0.0;
        for (int c = 0; c < C; ++c) v += (double)w1[(size_t)j * k1p + c] * ctx[c];
        h[j] = std::max(v, 0.0);
      }
      for (int i = 0; i < growth; ++i) {
        double v = b2 ? b2[i] : 0.0;
        for (int j = 0; j < red; ++j) v += (double)w2[(size_t)i * k2p + j] * h[j];
        gate[((size_t)b * nseg + s) * ldg + i] = (float)(1.0 / (1.0 + std::exp(-v)));
      }
    }
  }
  return hipSuccess;
}
hipError_t launch_cam_context(const float* x, int B, int T, int C, int ld, int seg, int nseg, float* out, int ldo,
                              hipStream_t, const int* vlen) {
  EMU_GATE();
  for (int b = 0; b < B; ++b) {
    const int Tb = vlen ? vlen[b] : T;
    for (int c = 0; c < C; ++c) {
      double tot = 0;
      for (int t = 0; t < Tb; ++t) tot += x[((size_t)b * T + t) * ld + c];
      for (int s = 0; s < nseg; ++s) {
        const int t0 = s * seg, t1 = std::min(Tb, t0 + seg);
        double a = 0;
        for (int t = t0; t < t1; ++t) a += x[((size_t)b * T + t) * ld + c];
        out[((size_t)b * nseg + s) * ldo + c] = t1 > t0 ? (float)(tot / Tb + a / (t1 - t0)) : 0.f;
      }
    }
  }
  return hipSuccess;
}
hipError_t launch_stats_pool(const float* x, int B, int T, int C, int ld, float* out, hipStream_t, const int* vlen) {
  EMU_GATE();
  for (int b = 0; b < B; ++b) {
    const int Tb = vlen ? vlen[b] : T;
    for (int c = 0; c < C; ++c) {
      double s = 0, q = 0;
      for (int t = 0; t < Tb; ++t) s += x[((size_t)b * T + t) * ld + c];
      const double mean = s / Tb;
      for (int t = 0; t < Tb; ++t) { const double d = x[((size_t)b * T + t) * ld + c] - mean; q += d * d; }
      out[(size_t)b * 2 * C + c] = (float)mean;
      out[(size_t)b * 2 * C + C + c] = (float)std::sqrt(q / (Tb - 1));
    }
  }
  return hipSuccess;
}
hipError_t launch_derive_len(const int* in, int* out, int B, int pad, int k, int stride, hipStream_t) {
  EMU_GATE();
  for (int b = 0; b < B; ++b) out[b] = (in[b] + 2 * pad - k) / stride + 1;
  return hipSuccess;
}
}  // namespace spk
namespace spk { int conv_tile_blocks(const ConvDesc& d) { return (d.nimg * d.Ho * d.Wo + 127) / 128 * ((d.N + 127) / 128); } }
