// Shared device/host definitions for libspk_hip (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>
#include <string>

namespace spk {

// Fused epilogue activations (applied after bias + residual).
enum Act : int {
  ACT_NONE = 0,
  ACT_RELU = 1,      // max(x, 0)                       (F.relu / nn.ReLU)
  ACT_HTANH = 2,     // clamp(x, 0, 20)                 (ERes2Net "ReLU" = nn.Hardtanh(0,20))
  ACT_SILU = 3,      // x * sigmoid(x)
  ACT_SIGMOID = 4,
  ACT_TANH = 5,
};

// One input operand of the implicit GEMM, channels-last: element (img, h, w, c) lives at
// p[((img*H + h)*W + w)*ld + c].  `cin` is the padded channel count the weights were packed
// with (multiple of 4); channels cin_real..cin-1 must hold finite values (they meet zero
// weights).  A 1-D (TDNN) tensor is H == 1.
struct ConvSrc {
  const float* p = nullptr;
  const float* p2 = nullptr;   // optional addend with the same geometry (Res2Net "sp + spx")
  int ld = 0, ld2 = 0;
  int H = 1, W = 1;
  int cin = 0;
  int kh = 1, kw = 1, sh = 1, sw = 1, ph = 0, pw = 0, dh = 1, dw = 1;
  int reflect = 0;             // speechbrain 'same' reflect padding (ECAPA Conv1d)
  // optional pre-activation applied to in-bounds operand values: relu(v*scale[c] + shift[c])
  // (CAM++ BN-ReLU in front of a conv; padding stays zero like the reference's F.pad of the
  // activated tensor)
  const float* pre_scale = nullptr;
  const float* pre_shift = nullptr;
  // optional per-image valid width (ragged batches: time axis = W): positions w >= vlen[img]
  // read as padding (zero), exactly like the end of an utterance of that length
  const int* vlen = nullptr;
};

// out[m, n] = epi( sum_k A[m, k] * Wt[n, k] ), m = (img, ho, wo), k = (tap, c) of s0 then c of s1.
struct ConvDesc {
  ConvSrc s0, s1;              // s1 used only when s1.p != nullptr (1x1, K-concatenated)
  int nimg = 0, Ho = 0, Wo = 0;
  int N = 0;                   // output channels written (incl. zero padding columns)
  int K = 0, Kp = 0;           // K = taps0*s0.cin + s1.cin ; Kp = round_up(K, 16)
  const float* w = nullptr;    // [N][Kp]
  const uint16_t* wh = nullptr;  // the same weights split for the fp16x3 MFMA path: fp16(w)
  const uint16_t* wl = nullptr;  //   and fp16((w - fp16(w)) * 2^11), both [N][Kp]
  const float* bias = nullptr; // [N] or null
  const float* rowbias = nullptr; int rowbias_ld = 0;  // per-image bias [nimg][rowbias_ld] (ECAPA ASP context)
  float* out = nullptr; int ldo = 0;
  // planar output slices (Res2Net conv1 -> T1): column n goes to plane n / osplit at
  // offset n % osplit of a [M][ldo] plane, planes oplane floats apart (0: one dense buffer)
  int osplit = 0; long long oplane = 0;
  int act = ACT_NONE;
  int act2 = ACT_NONE;         // applied after the post-affine (ECAPA ASP: BN then tanh)
  const float* res = nullptr; int ldr = 0;             // added before act
  const float* post_scale = nullptr;                   // after act: y*scale+shift (ECAPA BN after ReLU)
  const float* post_shift = nullptr;
  const float* affx = nullptr; int ldx = 0;            // AFF combine: x*(1+tanh v) + y*(1-tanh v)
  const float* affy = nullptr; int ldy = 0;
  const float* gate = nullptr; int gate_ld = 0; int gate_seg = 0;  // out *= gate[img][t/seg][n] (CAM)
  int gate_nseg = 0;
  int ksplit = 1; float* partial = nullptr;            // split-K partial slabs [ksplit][M][N]
  const int* rowlen = nullptr;  // ragged batches: outputs with wo >= rowlen[img] are written as 0
  int* range_flag = nullptr;    // fp16x3 range guard (below): set when an output reaches kRangeLimit
  int x1 = 0;                   // single-product fp16 MFMA (SPK_PRECISION_FP16): hi planes only
  int wbig = 0;                 // a packed weight >= kX3WeightLimit: the tiled fp16x3 GEMM (whose
                                // hi x hi product uses 2^11 hi_w) would overflow -> exact fp32 GEMM
  const int* run_if = nullptr;  // launch gate (below): set by launch_conv from launch_gate()
  // K order of s0 in the packed weights and the A loaders.  0: k = tap * cin + c.  1 (deep
  // multi-tap convs, cin a multiple of 32, no s1): 32-channel blocks outer, taps inner,
  // k = ((c / 32) * taps + tap) * 32 + c % 32 -- a 32-deep K-tile is one tap of one channel
  // block, and the taps of a block follow each other, so the block's input pixels are re-read
  // from L2 within a few K-tiles instead of once per sweep over the whole K (runtime.cpp pack)
  int kcb = 0;
  // the weights in MFMA fragment order for the LDS-DMA GEMM (conv_gemm_f.hip launch_pack_frag;
  // null: that kernel is not used)
  const uint16_t* wf = nullptr;
  const int* range_in = nullptr;  // scaled split (below): the forward's range word, read for the operand scale
};

// fp16x3 range guard.  The split-precision GEMMs represent an operand as two fp16 values,
// so an activation at or above fp16's largest finite value (65504) would saturate silently.
// Every producer of an unbounded activation that a split GEMM later reads (conv / linear
// epilogues, the ERes2Net stem, AFF, the model input) raises the forward's range word (a slot
// of the caller's workspace, zeroed at the start of every forward) to the bit pattern of the
// largest |output| it writes, when that reaches kRangeLimit (atomicMax on the bits of a
// non-negative float orders like the floats; the word stays 0 while everything is in range).
// The ops between two GEMMs grow a value at most 2x (AFF combine: |x t + y (2 - t)| <=
// 2 max(|x|, |y|); residual + Hardtanh; the Res2Net addend), so while the word is 0 every
// operand a split GEMM reads stays below 2 kRangeLimit = 2^15 < 65504 (a limit of 2^15 would
// let a doubled 32767.9 reach 65535.8, past fp16's largest finite value).  A set word is
// resolved one of two ways, both on the device without a host round trip:
//  - exact twin (ERes2Net*, ResNet): the exact-fp32 plan is captured behind the fp16x3 one on
//    the same stream with its launches gated on the word (launch_gate);
//  - scaled split (ECAPA, CAM++: every split GEMM of the plan takes ConvDesc::range_in): a
//    GEMM multiplies the operand it splits by range_scale(word) = 2^-s, s chosen so that
//    word * 2^-s < kRangeLimit, and its accumulator by 2^s (both exact: powers of two).  Every
//    operand is at most twice the largest value any earlier producer wrote, which the word
//    holds by the time the GEMM starts, so the scaled operand stays below 2^15; relative
//    precision is that of the unscaled split.
//    A loader that applies an affine pre-activation (CAM++ BN-ReLU, |relu(psc x + psh)| <=
//    |psc| |x| + |psh|) breaks the 2x growth bound by up to P = max_c max(|psc|, |psh| / 2^14):
//    with |x| < 2^(e+2) (e: the word's exponent, 13 when clear) the operand is below
//    1.5 P 2^(e+2), so a further 2^-b with P <= 1.3 * 2^b keeps the scaled operand below
//    1.95 * 2^15 < 65504.  That 2^-b is folded into the affine on the host (psc 2^-b,
//    psh 2^-b: relu is positively homogeneous and power-of-two scaling is exact) and 2^b into
//    the GEMM's packed weights (Model::pack wexp; the products are unchanged, bit for bit), so
//    no kernel sees it: the GEMM keeps its in-range instance while the word is clear, and the
//    exact-fp32 kernels and the twin plans read the same packed operands.  A block may read a larger word than another (producers of its own
//    launch raising it meanwhile): each block undoes its own scale, so every output is consistent.
constexpr float kRangeLimit = 16384.0f;
// the tiled fp16x3 GEMM scales the weights' hi plane by 2^11 (conv_gemm.hip): 31.5 * 2^11 < 65504
constexpr float kX3WeightLimit = 31.5f;
#ifdef __HIPCC__
__device__ __forceinline__ void range_note(int* flag, float amax) {
  if (flag && amax >= kRangeLimit) atomicMax(flag, __float_as_int(amax));
}
// operand scale of a scaled-split GEMM (above): 1 while the word is clear (or absent, or
// non-finite: the result is inf / NaN either way), else 2^-s with word * 2^-s in [2^13, 2^14)
__device__ __forceinline__ float range_scale(const int* word) {
  if (!word) return 1.f;
  const int w = *word;
  if (w < 0x46800000 || w >= 0x7F800000) return 1.f;       // below 2^14 (i.e. 0), or inf / NaN
  const int e = (w >> 23) - 127;                             // word in [2^e, 2^(e+1)), e >= 14
  return __int_as_float((127 - (e - 13)) << 23);             // 2^-(e-13)
}
// the same value without early returns: the LDS-DMA, pointwise and halo kernels measured
// 2 % faster with this form on ECAPA (its 256x256 GEMMs), while the tiled GEMM's 128-VGPR
// allocation spills inside its in-range instance with it (PRE instance 42 -> 58 spilled VGPRs,
// CAM++ dense layers +70 %): each keeps the form it was tuned with
__device__ __forceinline__ float range_scale_flat(const int* word) {
  int s = 0;
  if (word) {
    const int w = *word;
    if (w >= 0x46800000 && w < 0x7F800000) s = ((w >> 23) - 127) - 13;   // word in [2^e, 2^(e+1)), e >= 14
  }
  return __int_as_float((127 - min(s, 126)) << 23);   // 2^-s, kept normal
}
// 2^k * sc and 2^k / sc of a power-of-two scale by exponent arithmetic (scalar integer ops:
// the values stay in SGPRs instead of taking a VGPR each for a float multiply / divide)
__device__ __forceinline__ float pow2_mul(float sc, int k) { return __int_as_float(__float_as_int(sc) + k * (1 << 23)); }
__device__ __forceinline__ float pow2_div(float sc, int k) {
  return __int_as_float(0x7F000000 + k * (1 << 23) - __float_as_int(sc));
}
// Time reductions with one lane per channel (TDNN statistics, TSTP pooling) are latency-
// bound: a frame's load feeds a serial update, so a wave keeps only a load or two in flight.
// scan_frames issues U frames' loads back to back, then runs the updates in frame order
// (results bit-identical to the frame-at-a-time loop).
template <int U, class F>
__device__ __forceinline__ void scan_frames(const float* p, size_t ld, int Tb, F f) {
  int t = 0;
  for (; t + U <= Tb; t += U) {
    float v[U];
#pragma unroll
    for (int j = 0; j < U; ++j) v[j] = p[(size_t)(t + j) * ld];
#pragma unroll
    for (int j = 0; j < U; ++j) f(v[j], t + j);
  }
  for (; t < Tb; ++t) f(p[(size_t)t * ld], t);
}

// the same over two arrays read in step (logits and x of the attentive pooling)
template <int U, class F>
__device__ __forceinline__ void scan_frames2(const float* p, size_t ldp, const float* q, size_t ldq, int Tb, F f) {
  int t = 0;
  for (; t + U <= Tb; t += U) {
    float a[U], b[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      a[j] = p[(size_t)(t + j) * ldp];
      b[j] = q[(size_t)(t + j) * ldq];
    }
#pragma unroll
    for (int j = 0; j < U; ++j) f(a[j], b[j]);
  }
  for (; t < Tb; ++t) f(p[(size_t)t * ldp], q[(size_t)t * ldq]);
}

// launch gate: a kernel of the gated exact plan returns at once unless *run_if != 0 (the
// word is not written while that plan runs, so every wave of the grid sees the same value)
#define SPK_GATE(run_if) do { if ((run_if) != nullptr && *(run_if) == 0) return; } while (0)
#endif

// Host: the gate that launches issued by the calling thread carry (null: ungated).  The
// plan runner sets it around the exact plan's steps (runtime.cpp GateScope).
const int* launch_gate();

// XCD-aware bijective block remap: consecutive logical ids (same M tile, all N tiles) are
// placed on one XCD so the A tile they share stays in that XCD's L2 (the dispatcher deals
// blocks round-robin over the 8 XCDs; cdna_hip_programming.md §5.5 T1, bijective form).
__device__ __forceinline__ int xcd_remap(int orig, int nblk) {
  const int q = nblk / 8, r = nblk % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// address of output element (m, n) (4 consecutive columns never straddle a plane:
// osplit is a multiple of 4, checked on the host)
__host__ __device__ inline float* out_at(const ConvDesc& d, int m, int n) {
  if (d.osplit) return d.out + (size_t)(n / d.osplit) * d.oplane + (size_t)m * d.ldo + n % d.osplit;
  return d.out + (size_t)m * d.ldo + n;
}

// true when output row m is past its image's valid length (ragged batches)
__host__ __device__ inline bool row_masked(const ConvDesc& d, int m) {
  if (!d.rowlen) return false;
  const int wo = m % d.Wo, img = m / (d.Wo * d.Ho);
  return wo >= d.rowlen[img];
}

// The conv GEMM's buffer-resource loader (conv_loader.h BufALoader) applies: zero padding,
// s0.cin >= 32 (one tap boundary per 32-deep K-tile), at most 30 taps, and every operand
// byte a block of `bm` rows can touch within 2 GiB of its first image.  Otherwise the
// generic loader runs, which exists for the plain and the addend (ADD) forms only.
inline bool conv_buf_loader_ok(const ConvDesc& d, int bm) {
  // reflect padding: the 1-D form only (ECAPA's Conv1d, H = 1), full-length rows, pad < W
  if (d.s0.reflect && !(d.s0.H == 1 && d.s0.kh == 1 && !d.s0.vlen && d.s0.pw < d.s0.W)) return false;
  if (d.s0.cin < 32 || d.s0.kh * d.s0.kw > 30) return false;
  const double span = (double)(bm / (d.Ho * d.Wo) + 2);
  const double lim = 0x7FFFFFF0 - 64;
  if (span * d.s0.H * d.s0.W * d.s0.ld * 4.0 > lim) return false;
  if (d.s0.p2 && span * d.s0.H * d.s0.W * d.s0.ld2 * 4.0 > lim) return false;
  if (d.s1.p && span * d.s1.H * d.s1.W * d.s1.ld * 4.0 > lim) return false;
  return (double)d.N * d.Kp * 2.0 < lim;
}

hipError_t launch_conv(const ConvDesc& d, hipStream_t s);
bool conv_use_x3();   // fp16x3 split-precision MFMA path (default; SPK_CONV_MFMA=f32 selects exact fp32 MFMA)
std::string conv_kernel_name(const ConvDesc& d);
int conv_tile_blocks(const ConvDesc& d);
// halo-tiled 3x3 kernel for small channel counts (conv3x3_halo.hip); launch_conv routes to it
bool halo_conv_supported(const ConvDesc& d);
hipError_t launch_conv3x3_halo(const ConvDesc& d, hipStream_t s);
std::string halo_kernel_name(const ConvDesc& d);
hipError_t launch_splitk_reduce(const ConvDesc& d, hipStream_t s);   // conv_gemm.hip
// persistent short-K 1x1 GEMM (pw_gemm.hip); launch_conv routes to it
bool pw_supported(const ConvDesc& d);
hipError_t launch_pw(const ConvDesc& d, hipStream_t s);
std::string pw_kernel_name(const ConvDesc& d);   // blocks of one split of the tile config launch_conv picks

// fp16x3 GEMM with fragment-packed weights streamed by LDS-DMA (conv_gemm_f.hip); launch_conv
// routes the plain buffer-loader layers to it
bool gemm_f_supported(const ConvDesc& d);
hipError_t launch_gemm_f(const ConvDesc& d, hipStream_t s);
std::string gemm_f_kernel_name(const ConvDesc& d);
size_t frag_halves(int N, int Kp);   // size of one matrix in fragment order (N padded to 128)
hipError_t launch_pack_frag(const uint16_t* wh, const uint16_t* wl, int N, int Kp, uint16_t* out, hipStream_t s);

int device_cus();   // CU count of the current device, cached per device (pw_gemm.hip)

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace spk
