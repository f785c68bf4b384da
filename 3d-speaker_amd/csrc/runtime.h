// Native executor: weight folding/packing, per-shape launch plans, workspace layout.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <tuple>
#include <string>
#include <vector>

#include "../../include/spk_hip.h"
#include "common.h"

namespace spk {

struct SpkError : std::runtime_error {
  int code;
  SpkError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// A pointer resolved at launch time: into the caller's workspace, the input features, the
// output embeddings, or the model's packed weights (absolute).
struct Buf {
  enum Kind { NONE = 0, WS = 1, IN = 2, OUT = 3, ABS = 4, LEN = 5 };   // LEN: caller's per-utterance frames
  int kind = NONE;
  size_t off = 0;           // bytes (WS/IN/OUT) ; ABS uses ptr
  const float* ptr = nullptr;
  Buf at(size_t floats) const { Buf b = *this; if (kind == ABS) b.ptr += floats; else b.off += floats * 4; return b; }
  explicit operator bool() const { return kind != NONE; }
};

struct Ctx {
  char* ws;
  const float* in;
  float* out;
  hipStream_t stream;
  const int* lens = nullptr;   // ragged batches: valid frames per utterance (device int32 [B])
  int* flag = nullptr;         // this forward's fp16x3 range-guard word (workspace slot; null: exact plan)
  float* resolve(const Buf& b) const {
    switch (b.kind) {
      case Buf::WS: return reinterpret_cast<float*>(ws + b.off);
      case Buf::IN: return const_cast<float*>(reinterpret_cast<const float*>(reinterpret_cast<const char*>(in) + b.off));
      case Buf::OUT: return reinterpret_cast<float*>(reinterpret_cast<char*>(out) + b.off);
      case Buf::ABS: return const_cast<float*>(b.ptr);
      case Buf::LEN: return lens ? reinterpret_cast<float*>(const_cast<int*>(lens)) : nullptr;
      default: return nullptr;
    }
  }
  int* resolve_i(const Buf& b) const { return reinterpret_cast<int*>(resolve(b)); }
};

using Step = std::function<hipError_t(const Ctx&)>;

struct Plan {
  std::vector<Step> steps;
  std::vector<std::string> names;   // for error messages / tracing
  std::vector<std::string> kernels; // kernel instantiation each step launches
  std::vector<double> flops;        // algorithmic FLOPs of the step (whole batch)
  std::vector<double> bytes;        // algorithmic HBM bytes of the step (each operand once; 0 = not priced)
  size_t ws_bytes = 0;              // intermediates (the pair adds staging, PlanPair)
  // range-guard segments (Builder::segment): step ranges [seg_end[i-1], seg_end[i]) and whether
  // the segment's exact twin must follow it (a split-GEMM operand of the segment is not proved
  // below kRangeLimit); empty = one segment, twin always.  `allocs` logs the workspace layout,
  // so the runtime can check that both plans of a pair place every buffer alike
  std::vector<size_t> seg_end;
  std::vector<char> seg_twin;
  // scaled split (common.h): every split GEMM of the plan scales its operand by the range
  // word, so a set word needs no exact twin (ECAPA, CAM++)
  bool scaled = false;
  std::vector<std::pair<size_t, size_t>> allocs;
};

// A shape's fp16x3 plan and exact-fp32 plan over one workspace layout: intermediates in
// [0, max ws), then the staging regions and the range word both plans share.  `graphs`
// holds the captured forward (fp16x3 steps + gated exact steps) per workspace address.
struct PlanPair {
  std::unique_ptr<Plan> x3, ex;     // x3 == null: the handle runs exact only
  size_t ws_bytes = 0;
  size_t stage_in = 0, stage_out = 0, stage_len = 0, stage_flag = 0;
  size_t in_bytes = 0, out_bytes = 0, len_bytes = 0;
  std::map<const void*, hipGraphExec_t> graphs;
  // completion of the last graph replay enqueued from this pair on each stream it was
  // replayed on (recorded after the launch; a pair's graphs can be replayed from several
  // threads on several streams): an evicted pair's executable graphs are destroyed only once
  // every one of them has completed (Model::retired), never by synchronising the device.
  // Guarded by Model::mu.
  std::vector<std::pair<hipStream_t, hipEvent_t>> last;
  bool idle() const;                // no replay of this pair can still be running, on any stream
  hipError_t mark(hipStream_t s);   // record this stream's completion event behind a replay
  ~PlanPair();
};

// Logical -> physical channel map of a channels-last tensor (zero-padded slices).
struct ChanMap {
  std::vector<int> phys;
  int n_phys = 0;
  static ChanMap dense(int c, int align = 4);
  static ChanMap slices(int width, int n, int align = 4);   // n slices of `width`, each padded
  int n_log() const { return (int)phys.size(); }
};

// Packed GEMM operand: weights [N][Kp] (+ bias [N]) at offsets of the model's arena.
struct Packed {
  size_t w_off = 0, b_off = 0;
  int N = 0, K = 0, Kp = 0;
  size_t ps_off = SIZE_MAX, pt_off = SIZE_MAX;   // optional post-activation affine
  // the same affine times 2^-pre_bits, for a GEMM's pre-activation loader (common.h range
  // guard, pre_range_bits; SIZE_MAX while pre_bits = 0); that GEMM's weights are packed times
  // 2^pre_bits (wexp)
  size_t ps2_off = SIZE_MAX, pt2_off = SIZE_MAX;
  int pre_bits = 0;
  int wexp = 0;                                   // weights packed times 2^wexp (Model::pack)
  bool has_bias = false;
  float wmax = 0.f;                               // max |w| of the packed matrix
  double l1max = 0.0;                             // max over output channels of sum_k |w| (bounds)
  double bmax = 0.0;                              // max |bias|
  int kcb = 0;                                    // K order (common.h ConvDesc::kcb)
  size_t f_off = SIZE_MAX;                        // fragment-order copy in Model::dfrag (halves)
};

// One weight tensor's contribution to a packed GEMM.
struct Part {
  std::string wkey;        // conv / linear weight [Cout][Cin](...[kh][kw])
  std::string bias_key;    // optional conv bias
  std::string bn;          // optional BatchNorm prefix folded into this part
  ChanMap in;              // physical layout of the part's input source
  int ci_lo = 0;           // first logical input channel of the weight read by this part
  int kofs = 0;            // K offset of this part in the packed matrix
  std::string bn_in;       // optional BatchNorm applied to the INPUT (linear in between), folded
                           // as W*diag(s) and bias += W*t  (ECAPA asp_bn -> fc)
};

struct Model {
  spk_model_config_t cfg{};
  int device = 0;
  struct HostT { std::vector<int64_t> shape; std::vector<float> data; };
  std::map<std::string, HostT> W;                 // host copies (dropped after create)
  std::vector<float> arena;                       // packed host weights (dropped after upload)
  float* dweights = nullptr;
  size_t dweights_bytes = 0;
  uint16_t* dsplit = nullptr;                     // fp16 hi plane then lo plane of the whole arena
  uint16_t* dfrag = nullptr;                      // MFMA fragment order of the LDS-DMA GEMM's weights
  std::map<std::string, Packed> packed;
  // launch plans by (B, T, ragged): the fp16x3 plan and its exact-fp32 twin (the range
  // guard's gated re-run; the same object when the handle runs exact only), sharing one
  // workspace layout.  At most kMaxPlans are kept, least recently used evicted; callers hold
  // a shared_ptr, so an evicted pair lives until its last forward has been enqueued
  std::map<std::tuple<int, int, int>, std::shared_ptr<PlanPair>> plans;
  std::map<std::tuple<int, int, int>, uint64_t> plan_use;
  std::vector<std::shared_ptr<PlanPair>> retired;  // evicted pairs whose last replay may still run
  uint64_t plan_clock = 0;
  static constexpr size_t kMaxPlans = 24;
  bool force_exact = false;                       // a packed weight is out of fp16 range: exact path only
  bool fp16 = false;                              // SPK_PRECISION_FP16: single-product fp16 GEMMs
  float gemm_wmax = 0.f;                          // max |w| over the packed GEMM weights
  std::mutex mu;
  bool uploaded = false;

  std::map<std::string, std::vector<int64_t>> shapes;   // every state_dict key (kept for the handle's life)

  const HostT& get(const std::string& k) const;
  bool has(const std::string& k) const { return shapes.count(k) != 0; }
  int64_t dim(const std::string& k, int i) const;

  size_t put(const std::vector<float>& v);        // append 64-float aligned, return offset (floats)
  const float* dptr(size_t off) const { return dweights + off; }
  const uint16_t* dhi(size_t off) const { return dsplit ? dsplit + off : nullptr; }
  const uint16_t* dlo(size_t off) const { return dsplit ? dsplit + dweights_bytes / sizeof(float) + off : nullptr; }
  // fold BN (+conv bias) into per-output-channel (scale, shift) in double precision
  void bn_fold(const std::string& bn, int n, std::vector<double>& s, std::vector<double>& t, double eps = 1e-5) const;
  // wexp: weights (not bias) times 2^wexp, for a GEMM behind a pre-activation packed times
  // 2^-wexp (Packed::pre_bits; exact: the products are unchanged)
  const Packed& pack(const std::string& name, const ChanMap& out, const std::vector<Part>& parts, int K, int wexp = 0);
  const Packed& pack_post_affine(const std::string& name, const std::string& bn, const ChanMap& out);
};

// Per-architecture graph builders.  With plan == nullptr they only pack weights.
struct Builder {
  Model& m;
  Plan* plan;
  int B;
  size_t ws = 0;
  double macs_per_utt = 0;   // algorithmic conv/linear MACs for this (T)
  double macs_at_last_step = 0;
  bool ragged = false;       // per-utterance lengths (Buf::LEN) mask the time axis
  bool exact = false;        // exact-fp32 MFMA kernels only (no fp16x3 split anywhere)
  bool scaled = false;       // scaled split: convs read the range word for their operand scale
                             // (common.h), the plan has no exact twin
  bool x1_scope = true;      // SPK_PRECISION_FP16 handles: convs emitted while set use the
                             // single-product kernels (model builders keep the input-side
                             // layers, whose error the network amplifies most, fp16x3)
  Builder(Model& mm, Plan* p, int b, bool rg = false, bool ex = false) : m(mm), plan(p), B(b), ragged(rg), exact(ex) {}
  bool x3() const { return !exact && conv_use_x3(); }
  Buf alloc(size_t floats);
  void step(const std::string& name, Step s, const std::string& kernel = "", double bytes = 0.0);
  // Scaled-split invariant (common.h): every split-GEMM operand is at most 2x the largest value
  // an earlier producer noted in the range word.  In a scaled plan every non-conv step declares
  // the workspace buffers it writes before it is emitted (`writes(...).step(...)`): NOTED (its
  // kernel raises the word, like every conv epilogue), BOUNDED (its outputs stay within 2x of
  // its inputs' largest value: means, standard deviations, gates) or AUX (lengths, gates and
  // partial sums that no GEMM reads as an operand).  Builder::conv then refuses an operand
  // whose allocation has an AUX writer or no declared writer at all (SpkError at plan build),
  // so a future amplifying step cannot feed a split GEMM unnoticed.
  enum Grow { NOTED = 0, BOUNDED = 1, AUX = 2 };
  struct Write {
    Buf buf;
    Grow grow;
  };
  Builder& writes(std::vector<Write> w) {
    pending_writes = std::move(w);
    writes_declared = true;
    return *this;
  }
  std::vector<Write> pending_writes;
  bool writes_declared = false;
  std::map<size_t, int> alloc_writers;   // allocation offset -> OR of (1 << Grow) of its writers
  void record_write(const Buf& b, Grow g);
  void check_operand(const std::string& name, const Buf& b) const;
  // close a range-guard segment at the current step (Plan::seg_end); `twin`: the gated
  // exact twin of the segment must run behind it (models without segments: one segment, twin)
  void segment(bool twin);
  // static bound of a conv's output |W x + b| given |x| <= in (kRangeLimit analysis)
  static double bound(const Packed& p, double in) { return p.l1max * in + p.bmax; }
  // emit an implicit-GEMM conv; pointers of `d` are taken from the Bufs
  struct ConvIO {
    Buf s0, s0b, s1, out, res, affx, affy, gate, partial, rowbias;
    Buf rowlen, vlen;   // ragged batches (int32 arrays): output / s0-input valid time extents
    const Packed* pre = nullptr;   // s0's BN-ReLU pre-activation (Model::pack_post_affine)
  };
  void conv(const std::string& name, ConvDesc d, const Packed& p, const ConvIO& io, bool use_bias = true);
};

// operand scale bits for a GEMM whose loader applies the pre-activation `pre` (common.h
// range guard; Packed::pre_bits / wexp): the smallest b >= 0 with
// max_c max(|psc|, |psh| / 2^14) <= 1.3 * 2^b
int pre_range_bits(const Packed& pre);

void build_eres2net(Builder& b, int T, bool v2);
void build_ecapa(Builder& b, int T);
void build_campplus(Builder& b, int T);
void build_resnet(Builder& b, int T, bool res2);

void set_error(const std::string& msg);

}  // namespace spk
