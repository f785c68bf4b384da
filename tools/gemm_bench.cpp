// Conv-GEMM micro-benchmark (dev tool): times spk::launch_conv of one or more builds of
// libspk_hip.so (dlopen'ed, so variant builds A/B in one process) on the ERes2NetV2 B = 256
// layer shapes that carry most of the forward, and checks sampled outputs against an fp64
// host reference.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -I3d-speaker_amd/csrc tools/gemm_bench.cpp -ldl -o tools/gemm_bench
//   tools/gemm_bench [--reps N] [--shapes a,b,..] lib1.so [lib2.so ...]
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "common.h"

using namespace spk;

typedef hipError_t (*launch_fn)(const ConvDesc&, hipStream_t);
typedef hipError_t (*split_fn)(const float*, uint16_t*, uint16_t*, size_t, hipStream_t);
typedef size_t (*fh_fn)(int, int);
typedef hipError_t (*pack_fn)(const uint16_t*, const uint16_t*, int, int, uint16_t*, hipStream_t);

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

struct Shape {
  const char* name;
  int nimg, H, W, cin, N, k, s, act;
  bool res;
  int addend;   // Res2Net addend operand (s0.p2)
  int s1cin = 0, s1H = 0, s1W = 0, s1s = 1;   // K-concatenated 1x1 operand (projection shortcut)
  int oned = 0, dil = 1, reflect = 0, pre = 0;   // 1-D (TDNN) conv over W, dilation, reflect pad, BN-ReLU pre-activation
};

// ERes2NetV2 (m_channels 64, baseWidth 26, scale 2, expansion 2) at B = 256, T = 198
static const Shape kShapes[] = {
    {"l3.conv1", 256, 20, 50, 512, 208, 1, 1, ACT_HTANH, false, 0},
    {"l3.conv3", 256, 20, 50, 208, 512, 1, 1, ACT_HTANH, true, 0},
    {"l3.convs0", 256, 20, 50, 104, 104, 3, 1, ACT_HTANH, false, 0},
    {"l3.convs1", 256, 20, 50, 104, 104, 3, 1, ACT_HTANH, false, 1},
    {"l4.conv1", 256, 10, 25, 1024, 416, 1, 1, ACT_HTANH, false, 0},
    {"l4.conv3", 256, 10, 25, 416, 1024, 1, 1, ACT_HTANH, true, 0},
    {"l4.convs0", 256, 10, 25, 208, 208, 3, 1, ACT_HTANH, false, 0},
    {"l3_ds", 256, 20, 50, 512, 1024, 3, 2, ACT_NONE, false, 0},
    {"l2.conv1", 256, 40, 99, 256, 104, 1, 1, ACT_HTANH, false, 0},
    {"l2.0.conv3", 256, 40, 99, 104, 256, 1, 1, ACT_HTANH, false, 0, 128, 80, 198, 2},
    {"l3.0.conv3", 256, 20, 50, 208, 512, 1, 1, ACT_HTANH, false, 0, 256, 40, 99, 2},
    {"fuse34.att0", 256, 10, 25, 1024, 256, 1, 1, ACT_SILU, false, 0, 1024, 10, 25, 1},
    // ECAPA-TDNN (C=1024) and CAM++ layers at B = 256, T = 198 on the tiled fp16x3 GEMM
    {"ec.b0", 256, 1, 198, 80, 1024, 5, 1, ACT_RELU, false, 0, 0, 0, 0, 1, 1, 1, 1, 0},
    {"ec.r2n", 256, 1, 198, 128, 128, 3, 1, ACT_RELU, false, 1, 0, 0, 0, 1, 1, 2, 1, 0},
    {"ec.tdnn1", 256, 1, 198, 1024, 1024, 1, 1, ACT_RELU, false, 0, 0, 0, 0, 1, 1, 1, 1, 0},
    {"cam.transit", 256, 1, 99, 512, 256, 1, 1, ACT_NONE, false, 0, 0, 0, 0, 1, 1, 1, 0, 1},
    {"cam.linear1", 256, 1, 99, 256, 128, 1, 1, ACT_NONE, false, 0, 0, 0, 0, 1, 1, 1, 0, 1},
};

struct Lib {
  std::string path;
  launch_fn launch;
  split_fn split;
  fh_fn frag_halves;   // null: a build without the LDS-DMA GEMM
  pack_fn pack;
};

int main(int argc, char** argv) {
  int reps = 20;
  std::string only;
  std::vector<Lib> libs;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--reps") && i + 1 < argc) { reps = std::atoi(argv[++i]); continue; }
    if (!std::strcmp(argv[i], "--shapes") && i + 1 < argc) { only = argv[++i]; continue; }
    void* h = dlopen(argv[i], RTLD_NOW | RTLD_LOCAL);
    if (!h) { std::fprintf(stderr, "dlopen %s: %s\n", argv[i], dlerror()); return 1; }
    Lib l{argv[i], (launch_fn)dlsym(h, "_ZN3spk11launch_convERKNS_8ConvDescEP12ihipStream_t"),
          (split_fn)dlsym(h, "_ZN3spk16launch_split_f16EPKfPtS2_mP12ihipStream_t"),
          (fh_fn)dlsym(h, "_ZN3spk11frag_halvesEii"),
          (pack_fn)dlsym(h, "_ZN3spk16launch_pack_fragEPKtS1_iiPtP12ihipStream_t")};
    if (!l.launch || !l.split) { std::fprintf(stderr, "%s: symbols missing\n", argv[i]); return 1; }
    libs.push_back(l);
  }
  if (libs.empty()) { std::fprintf(stderr, "usage: gemm_bench [--reps N] [--shapes a,b] lib.so ...\n"); return 1; }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::mt19937_64 rng(12345);

  for (const Shape& sh : kShapes) {
    if (!only.empty() && ("," + only + ",").find(std::string(",") + sh.name + ",") == std::string::npos) continue;
    const int kh = sh.oned ? 1 : sh.k, pad = sh.dil * (sh.k / 2), padh = sh.oned ? 0 : pad;
    const int Ho = sh.oned ? 1 : (sh.H + 2 * pad - sh.k) / sh.s + 1;
    const int Wo = (sh.W + 2 * pad - sh.dil * (sh.k - 1) - 1) / sh.s + 1;
    const int M = sh.nimg * Ho * Wo;
    const int taps = kh * sh.k, K0 = taps * sh.cin, K = K0 + sh.s1cin, Kp = round_up(K, 32);
    std::vector<float> ps(sh.pre ? sh.cin : 0), pt(sh.pre ? sh.cin : 0);
    const size_t nin = (size_t)sh.nimg * sh.H * sh.W * sh.cin;
    const size_t nin1 = (size_t)sh.nimg * sh.s1H * sh.s1W * sh.s1cin;
    std::vector<float> x(nin), x2(sh.addend ? nin : 0), w((size_t)sh.N * Kp, 0.f), b(sh.N), r(sh.res ? (size_t)M * sh.N : 0);
    std::uniform_real_distribution<float> ua(0.f, 2.f), uw(-1.f, 1.f);
    for (auto& v : x) v = ua(rng);
    for (auto& v : x2) v = ua(rng);
    std::vector<float> x1(nin1);
    for (auto& v : x1) v = ua(rng);
    const float ws = 1.0f / std::sqrt((float)K);
    for (int n = 0; n < sh.N; ++n)
      for (int k = 0; k < K; ++k) w[(size_t)n * Kp + k] = uw(rng) * ws;
    for (auto& v : b) v = uw(rng) * 0.1f;
    for (auto& v : r) v = ua(rng);
    for (auto& v : ps) v = 0.5f + 0.5f * ua(rng);
    for (auto& v : pt) v = uw(rng);
    float *dps = nullptr, *dpt = nullptr;
    if (sh.pre) {
      CK(hipMalloc(&dps, ps.size() * 4));
      CK(hipMalloc(&dpt, pt.size() * 4));
      CK(hipMemcpy(dps, ps.data(), ps.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(dpt, pt.data(), pt.size() * 4, hipMemcpyHostToDevice));
    }
    float *dx, *dx2 = nullptr, *dx1 = nullptr, *dw, *db, *dr = nullptr, *dout;
    if (nin1) {
      CK(hipMalloc(&dx1, nin1 * 4));
      CK(hipMemcpy(dx1, x1.data(), nin1 * 4, hipMemcpyHostToDevice));
    }
    uint16_t *dwh, *dwl;
    CK(hipMalloc(&dx, nin * 4));
    if (sh.addend) CK(hipMalloc(&dx2, nin * 4));
    CK(hipMalloc(&dw, w.size() * 4));
    CK(hipMalloc(&dwh, w.size() * 2));
    CK(hipMalloc(&dwl, w.size() * 2));
    CK(hipMalloc(&db, b.size() * 4));
    if (sh.res) CK(hipMalloc(&dr, r.size() * 4));
    CK(hipMalloc(&dout, (size_t)M * sh.N * 4));
    CK(hipMemcpy(dx, x.data(), nin * 4, hipMemcpyHostToDevice));
    if (sh.addend) CK(hipMemcpy(dx2, x2.data(), nin * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice));
    if (sh.res) CK(hipMemcpy(dr, r.data(), r.size() * 4, hipMemcpyHostToDevice));

    ConvDesc d;
    d.s0.p = dx; d.s0.p2 = dx2; d.s0.ld = sh.cin; d.s0.ld2 = sh.addend ? sh.cin : 0;
    d.s0.H = sh.H; d.s0.W = sh.W; d.s0.cin = sh.cin;
    d.s0.kh = kh; d.s0.kw = sh.k; d.s0.sh = d.s0.sw = sh.s; d.s0.ph = padh; d.s0.pw = pad;
    d.s0.dw = sh.dil; d.s0.reflect = sh.reflect; d.s0.pre_scale = dps; d.s0.pre_shift = dpt;
    d.nimg = sh.nimg; d.Ho = Ho; d.Wo = Wo; d.N = sh.N; d.K = K; d.Kp = Kp;
    d.w = dw; d.wh = dwh; d.wl = dwl; d.bias = db; d.out = dout; d.ldo = sh.N; d.act = sh.act;
    d.res = dr; d.ldr = sh.res ? sh.N : 0;
    if (nin1) {
      d.s1.p = dx1; d.s1.ld = sh.s1cin; d.s1.cin = sh.s1cin; d.s1.H = sh.s1H; d.s1.W = sh.s1W;
      d.s1.sh = d.s1.sw = sh.s1s;
    }

    // host reference of sampled outputs (fp64)
    std::vector<int> sm, sn;
    std::uniform_int_distribution<int> um(0, M - 1), un(0, sh.N - 1);
    for (int i = 0; i < 256; ++i) { sm.push_back(i < 8 ? (i < 4 ? i : M - 1 - (i - 4)) : um(rng)); sn.push_back(un(rng)); }
    std::vector<double> ref(sm.size()), mag(sm.size());
    for (size_t i = 0; i < sm.size(); ++i) {
      const int m = sm[i], n = sn[i];
      const int wo = m % Wo, ho = (m / Wo) % Ho, img = m / (Wo * Ho);
      double acc = b[n], a = std::fabs(b[n]);
      for (int ky = 0; ky < kh; ++ky)
        for (int kx = 0; kx < sh.k; ++kx) {
          const int hi = ho * sh.s - padh + ky;
          int wi = wo * sh.s - pad + kx * sh.dil;
          if (sh.reflect) wi = wi < 0 ? -wi : wi >= sh.W ? 2 * (sh.W - 1) - wi : wi;
          if (hi < 0 || hi >= sh.H || wi < 0 || wi >= sh.W) continue;
          const size_t px = ((size_t)img * sh.H + hi) * sh.W + wi;
          for (int c = 0; c < sh.cin; ++c) {
            double xv = x[px * sh.cin + c];
            if (sh.addend) xv += x2[px * sh.cin + c];
            if (sh.pre) xv = std::max((double)(float)(x[px * sh.cin + c] * ps[c] + pt[c]), 0.0);
            const double p = xv * w[(size_t)n * Kp + (ky * sh.k + kx) * sh.cin + c];
            acc += p;
            a += std::fabs(p);
          }
        }
      if (nin1) {
        const size_t px1 = ((size_t)img * sh.s1H + ho * sh.s1s) * sh.s1W + wo * sh.s1s;
        for (int c = 0; c < sh.s1cin; ++c) {
          const double p = (double)x1[px1 * sh.s1cin + c] * w[(size_t)n * Kp + K0 + c];
          acc += p;
          a += std::fabs(p);
        }
      }
      if (sh.res) { acc += r[(size_t)m * sh.N + n]; a += std::fabs(r[(size_t)m * sh.N + n]); }
      if (sh.act == ACT_HTANH) acc = std::min(std::max(acc, 0.0), 20.0);
      if (sh.act == ACT_RELU) acc = std::max(acc, 0.0);
      if (sh.act == ACT_SILU) {
        const double a0 = a;
        acc = acc / (1.0 + std::exp(-acc));
        a = a0;
      }
      ref[i] = acc;
      mag[i] = a;
    }
    const double flop = 2.0 * M * (double)K * sh.N;
    const double bytes = 4.0 * ((double)nin * (sh.addend ? 2 : 1) + (double)M * sh.s1cin + (double)M * sh.N * (sh.res ? 2 : 1));
    std::printf("%-10s M=%d K=%d N=%d  %.1f GFLOP  %.0f MB\n", sh.name, M, K, sh.N, flop * 1e-9, bytes * 1e-6);
    for (const Lib& L : libs) {
      CK(L.split(dw, dwh, dwl, w.size(), st));
      uint16_t* dwf = nullptr;
      if (L.frag_halves && L.pack) {
        CK(hipMalloc(&dwf, L.frag_halves(sh.N, Kp) * 2));
        CK(L.pack(dwh, dwl, sh.N, Kp, dwf, st));
      }
      d.wf = dwf;
      CK(hipMemsetAsync(dout, 0xff, (size_t)M * sh.N * 4, st));
      hipError_t le = L.launch(d, st);
      if (le != hipSuccess) {
        std::printf("  %-40s launch failed: %s\n", L.path.c_str(), hipGetErrorString(le));
        if (dwf) CK(hipFree(dwf));
        continue;
      }
      CK(hipStreamSynchronize(st));
      std::vector<float> o((size_t)M * sh.N);
      CK(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
      double worst = 0.0;
      for (size_t i = 0; i < sm.size(); ++i) {
        const double g = o[(size_t)sm[i] * sh.N + sn[i]];
        const double e = std::fabs(g - ref[i]) / (mag[i] + 1e-30);
        if (!(e <= worst)) worst = std::isnan(e) ? 1e30 : std::max(worst, e);
      }
      for (int i = 0; i < 3; ++i) CK(L.launch(d, st));
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) CK(L.launch(d, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / reps;
      std::printf("  %-40s %8.1f us  %6.1f TF(fp32-eq)  %5.2f TB/s  err %.2e %s\n", L.path.c_str(), us,
                  flop / us * 1e-6, bytes / us * 1e-6, worst, worst < 3e-6 ? "ok" : "BAD");
      std::fflush(stdout);
      if (dwf) CK(hipFree(dwf));
    }
    CK(hipFree(dx)); if (dx2) CK(hipFree(dx2)); if (dx1) CK(hipFree(dx1)); CK(hipFree(dw)); CK(hipFree(dwh)); CK(hipFree(dwl)); CK(hipFree(db));
    if (dr) CK(hipFree(dr)); CK(hipFree(dout));
    if (dps) CK(hipFree(dps)); if (dpt) CK(hipFree(dpt));
  }
  return 0;
}
