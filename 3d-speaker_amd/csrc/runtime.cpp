// libspk_hip C ABI + executor core (weight folding/packing, plans, workspace).
#include <algorithm>
#include "runtime.h"

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "fbank.h"
#include "misc.h"

namespace spk {

thread_local std::string g_last_error;
thread_local const int* g_launch_gate = nullptr;

void set_error(const std::string& msg) { g_last_error = msg; }

const int* launch_gate() { return g_launch_gate; }

// launches issued in this scope carry `gate` (common.h SPK_GATE)
struct GateScope {
  const int* prev;
  explicit GateScope(const int* g) : prev(g_launch_gate) { g_launch_gate = g; }
  ~GateScope() { g_launch_gate = prev; }
};

ChanMap ChanMap::dense(int c, int align) {
  ChanMap m;
  m.phys.resize(c);
  for (int i = 0; i < c; ++i) m.phys[i] = i;
  m.n_phys = round_up(c, align);
  return m;
}

ChanMap ChanMap::slices(int width, int n, int align) {
  ChanMap m;
  const int wp = round_up(width, align);
  m.phys.resize((size_t)width * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < width; ++i) m.phys[(size_t)j * width + i] = j * wp + i;
  m.n_phys = wp * n;
  return m;
}

const Model::HostT& Model::get(const std::string& k) const {
  auto it = W.find(k);
  if (it == W.end()) throw SpkError(SPK_E_WEIGHTS, "missing state_dict tensor: " + k);
  return it->second;
}

int64_t Model::dim(const std::string& k, int i) const {
  auto it = shapes.find(k);
  if (it == shapes.end()) throw SpkError(SPK_E_WEIGHTS, "missing state_dict tensor: " + k);
  if (i >= (int)it->second.size()) throw SpkError(SPK_E_WEIGHTS, "rank too small: " + k);
  return it->second[i];
}

size_t Model::put(const std::vector<float>& v) {
  const size_t off = (arena.size() + 63) / 64 * 64;
  arena.resize(off + v.size());
  std::memcpy(arena.data() + off, v.data(), v.size() * sizeof(float));
  return off;
}

void Model::bn_fold(const std::string& bn, int n, std::vector<double>& s, std::vector<double>& t, double eps) const {
  s.assign(n, 1.0);
  t.assign(n, 0.0);
  if (bn.empty()) return;
  const HostT& mean = get(bn + ".running_mean");
  const HostT& var = get(bn + ".running_var");
  if ((int)mean.data.size() != n || (int)var.data.size() != n)
    throw SpkError(SPK_E_WEIGHTS, bn + ": BatchNorm size mismatch");
  const HostT* g = W.count(bn + ".weight") ? &get(bn + ".weight") : nullptr;
  const HostT* be = W.count(bn + ".bias") ? &get(bn + ".bias") : nullptr;
  for (int c = 0; c < n; ++c) {
    const double gamma = g ? g->data[c] : 1.0;
    const double beta = be ? be->data[c] : 0.0;
    s[c] = gamma / std::sqrt((double)var.data[c] + eps);
    t[c] = beta - (double)mean.data[c] * s[c];
  }
}

const Packed& Model::pack(const std::string& name, const ChanMap& out, const std::vector<Part>& parts, int K, int wexp) {
  auto it = packed.find(name);
  if (it != packed.end()) {
    if (it->second.wexp != wexp) throw SpkError(SPK_E_INVALID, "internal: " + name + " packed with two weight scales");
    return it->second;
  }
  if (uploaded) throw SpkError(SPK_E_INVALID, "internal: pack after upload: " + name);
  const int N = out.n_phys;
  const int Kp = round_up(K, 32);
  std::vector<double> wd((size_t)N * Kp, 0.0), bd(N, 0.0);
  std::map<std::string, int> seen;
  bool has_bias = false;
  int taps0 = 1, cinp0 = 0;
  for (const Part& part : parts) {
    const HostT& w = get(part.wkey);
    if (w.shape.size() < 2) throw SpkError(SPK_E_WEIGHTS, part.wkey + ": expected a conv/linear weight");
    const int cout = (int)w.shape[0], cin = (int)w.shape[1];
    int taps = 1;
    for (size_t i = 2; i < w.shape.size(); ++i) taps *= (int)w.shape[i];
    if (cout != out.n_log()) throw SpkError(SPK_E_WEIGHTS, part.wkey + ": out channels mismatch");
    const int nin = part.in.n_log(), cinp = part.in.n_phys;
    if (part.ci_lo + nin > cin) throw SpkError(SPK_E_WEIGHTS, part.wkey + ": in channels mismatch");
    if (part.kofs + taps * cinp > K) throw SpkError(SPK_E_INVALID, "internal: K overflow packing " + part.wkey);
    taps0 = taps;
    cinp0 = cinp;
    std::vector<double> s, t, si, ti;
    bn_fold(part.bn, cout, s, t);
    bn_fold(part.bn_in, cin, si, ti);
    const bool first = seen.count(part.wkey) == 0;
    seen[part.wkey] = 1;
    for (int co = 0; co < cout; ++co) {
      double* row = wd.data() + (size_t)out.phys[co] * Kp + part.kofs;
      const float* src = w.data.data() + (size_t)co * cin * taps;
      double in_shift = 0.0;
      for (int ci = 0; ci < nin; ++ci)
        for (int tap = 0; tap < taps; ++tap) {
          const double wv = src[(size_t)(part.ci_lo + ci) * taps + tap];
          row[(size_t)tap * cinp + part.in.phys[ci]] = wv * si[part.ci_lo + ci] * s[co];
          in_shift += wv * ti[part.ci_lo + ci];
        }
      if (!part.bn_in.empty()) {
        bd[out.phys[co]] += s[co] * in_shift;
        has_bias = true;
      }
    }
    if (first) {
      const HostT* cb = part.bias_key.empty() ? nullptr : &get(part.bias_key);
      if (cb || !part.bn.empty()) has_bias = true;
      for (int co = 0; co < cout; ++co) bd[out.phys[co]] += (cb ? s[co] * cb->data[co] : 0.0) + t[co];
    }
  }
  Packed p;
  p.N = N; p.K = K; p.Kp = Kp; p.has_bias = has_bias;
  // channel-block-major K order for deep multi-tap convs (common.h ConvDesc::kcb)
  static const bool kcb_on = [] {
    const char* e = std::getenv("SPK_KCB");
    return e && std::string(e) == "1";
  }();
  if (kcb_on && parts.size() == 1 && parts[0].kofs == 0 && taps0 > 1 && cinp0 >= 128 && cinp0 % 32 == 0 &&
      K == taps0 * cinp0) {
    std::vector<double> row(Kp);
    for (int n = 0; n < N; ++n) {
      double* wr = wd.data() + (size_t)n * Kp;
      for (int tap = 0; tap < taps0; ++tap)
        for (int c = 0; c < cinp0; ++c) row[((size_t)(c / 32) * taps0 + tap) * 32 + c % 32] = wr[(size_t)tap * cinp0 + c];
      std::copy(row.begin(), row.begin() + K, wr);
    }
    p.kcb = 1;
  }
  if (wexp)
    for (double& v : wd) v = std::ldexp(v, wexp);   // before the fp32 rounding: the same as scaling after it
  p.wexp = wexp;
  std::vector<float> wf(wd.begin(), wd.end()), bf(bd.begin(), bd.end());
  for (float v : wf) p.wmax = std::max(p.wmax, std::fabs(v));
  for (int n = 0; n < N; ++n) {
    double l1 = 0.0;
    for (int k = 0; k < Kp; ++k) l1 += std::fabs((double)wf[(size_t)n * Kp + k]);
    p.l1max = std::max(p.l1max, l1);
    p.bmax = std::max(p.bmax, std::fabs((double)bf[n]));
  }
  gemm_wmax = std::max(gemm_wmax, p.wmax);   // range guard (common.h)
  p.w_off = put(wf);
  p.b_off = put(bf);
  return packed.emplace(name, p).first->second;
}

const Packed& Model::pack_post_affine(const std::string& name, const std::string& bn, const ChanMap& out) {
  const std::string key = name + "#post";
  auto it = packed.find(key);
  if (it != packed.end()) return it->second;
  if (uploaded) throw SpkError(SPK_E_INVALID, "internal: pack after upload: " + key);
  std::vector<double> s, t;
  bn_fold(bn, out.n_log(), s, t);
  std::vector<float> ps(out.n_phys, 0.f), pt(out.n_phys, 0.f);
  for (int c = 0; c < out.n_log(); ++c) { ps[out.phys[c]] = (float)s[c]; pt[out.phys[c]] = (float)t[c]; }
  Packed p;
  p.N = out.n_phys;
  for (int c = 0; c < out.n_phys; ++c) {   // |s x + t| <= l1max |x| + bmax (Builder::bound)
    p.l1max = std::max(p.l1max, std::fabs((double)ps[c]));
    p.bmax = std::max(p.bmax, std::fabs((double)pt[c]));
  }
  p.ps_off = put(ps);
  p.pt_off = put(pt);
  p.pre_bits = pre_range_bits(p);
  if (p.pre_bits) {   // powers of two: exact (the fp32 values stay normal for any sane affine)
    std::vector<float> ps2(ps), pt2(pt);
    for (int c = 0; c < out.n_phys; ++c) {
      ps2[c] = std::ldexp(ps[c], -p.pre_bits);
      pt2[c] = std::ldexp(pt[c], -p.pre_bits);
    }
    p.ps2_off = put(ps2);
    p.pt2_off = put(pt2);
  }
  return packed.emplace(key, p).first->second;
}

Buf Builder::alloc(size_t floats) {
  Buf b;
  b.kind = Buf::WS;
  b.off = ws;
  ws += (floats * sizeof(float) + 255) / 256 * 256;
  if (plan) plan->allocs.emplace_back(b.off, floats);
  return b;
}

void Builder::segment(bool twin) {
  if (!plan) return;
  plan->seg_end.push_back(plan->steps.size());
  plan->seg_twin.push_back(twin ? 1 : 0);
}

namespace {
// the allocation (Plan::allocs entry) holding workspace byte offset `off`, or SIZE_MAX
size_t alloc_of(const Plan& p, size_t off) {
  size_t best = SIZE_MAX;
  for (const auto& a : p.allocs)
    if (a.first <= off && off < a.first + std::max<size_t>(a.second, 1) * sizeof(float)) best = a.first;
  return best;
}
}  // namespace

void Builder::record_write(const Buf& b, Grow g) {
  if (!plan || b.kind != Buf::WS) return;
  const size_t a = alloc_of(*plan, b.off);
  if (a == SIZE_MAX) throw SpkError(SPK_E_INVALID, "internal: write outside every workspace allocation");
  alloc_writers[a] |= 1 << g;
}

void Builder::check_operand(const std::string& name, const Buf& b) const {
  if (!plan || !scaled || b.kind != Buf::WS) return;   // model input: the range_in step notes it
  const size_t a = alloc_of(*plan, b.off);
  const auto it = alloc_writers.find(a);
  const int w = a == SIZE_MAX || it == alloc_writers.end() ? 0 : it->second;
  if (!w || (w & (1 << AUX)))
    throw SpkError(SPK_E_INVALID, "internal: scaled-split operand of " + name +
                                      " has no declared NOTED / BOUNDED producer (runtime.h Builder::writes)");
}

void Builder::step(const std::string& name, Step s, const std::string& kernel, double bytes) {
  const bool declared = writes_declared;
  const std::vector<Write> w = std::move(pending_writes);
  pending_writes.clear();
  writes_declared = false;
  if (!plan) return;
  if (scaled && !declared)
    throw SpkError(SPK_E_INVALID, "internal: step " + name + " of a scaled plan without declared writes");
  for (const Write& x : w) record_write(x.buf, x.grow);
  plan->steps.push_back(std::move(s));
  plan->names.push_back(name);
  plan->kernels.push_back(kernel.empty() ? name : kernel);
  plan->bytes.push_back(bytes);
  plan->flops.push_back(2.0 * (macs_per_utt - macs_at_last_step) * B);
  macs_at_last_step = macs_per_utt;
}

int pre_range_bits(const Packed& pre) {
  const double P = std::max(pre.l1max, pre.bmax / kRangeLimit);
  int b = 0;
  while (b < 126 && P > 1.3 * std::ldexp(1.0, b)) ++b;
  return b;
}

void Builder::conv(const std::string& name, ConvDesc d, const Packed& p, const ConvIO& io, bool use_bias) {
  if (!plan) return;
  if (io.pre) {
    // the affine times 2^-b, the weights times 2^b (common.h range guard): every kernel that
    // takes a pre-activation (tiled fp16x3 / fp16 / exact fp32) computes the same products
    const bool s2 = io.pre->pre_bits > 0;
    if (p.wexp != io.pre->pre_bits)
      throw SpkError(SPK_E_INVALID, "internal: " + name + " weights not packed for its pre-activation scale");
    d.s0.pre_scale = m.dptr(s2 ? io.pre->ps2_off : io.pre->ps_off);
    d.s0.pre_shift = m.dptr(s2 ? io.pre->pt2_off : io.pre->pt_off);
  } else if (d.s0.pre_scale) {
    // the operand bound of the scaled split needs the pre-activation's host-side extremes
    throw SpkError(SPK_E_INVALID, "internal: pre-activation without its packed affine: " + name);
  }
  d.N = p.N; d.K = p.K; d.Kp = p.Kp;
  d.kcb = p.kcb;
  if (p.kcb && (d.s0.kh * d.s0.kw * d.s0.cin != d.K || d.s0.cin % 32 || io.s1))
    throw SpkError(SPK_E_INVALID, "internal: channel-block K order on an unsupported conv: " + name);
  d.w = m.dptr(p.w_off);
  d.wh = exact ? nullptr : m.dhi(p.w_off);   // no split planes: the exact-fp32 kernels are chosen
  d.wl = exact ? nullptr : m.dlo(p.w_off);
  d.wf = (exact || !m.dfrag || p.f_off == SIZE_MAX) ? nullptr : m.dfrag + p.f_off;
  const bool guard = !exact;   // producers note fp16x3 range overflows in the forward's word
  const bool scale_in = !exact && scaled;
  d.x1 = (!exact && m.fp16 && x1_scope) ? 1 : 0;
  d.wbig = p.wmax >= kX3WeightLimit ? 1 : 0;
  d.bias = (use_bias && p.has_bias) ? m.dptr(p.b_off) : nullptr;
  const int M = d.nimg * d.Ho * d.Wo;
  // split-K for skinny, deep GEMMs (e.g. the 20480 -> 192 embedding layer)
  const int nblk = conv_tile_blocks(d);
  const int nkt = d.Kp / 32;
  Buf partial;
  if (nblk < 128 && nkt >= 32 && !io.affx && !io.gate) {
    d.ksplit = std::max(1, std::min(nkt / 8, (256 + nblk - 1) / nblk));
    if (d.ksplit > 1) partial = alloc((size_t)d.ksplit * M * d.N);
  }
  ConvIO cio = io;
  cio.partial = partial;
  ConvDesc probe = d;   // kernel label: same tile choice as launch_conv
  probe.s1.cin = io.s1 ? d.s1.cin : 0;
  probe.s0.ld2 = io.s0b ? std::max(d.s0.ld2, 1) : 0;
  static const int kDummyLen = 0;   // naming probe only: marks the ragged masks as present
  probe.rowlen = io.rowlen ? &kDummyLen : nullptr;
  probe.s0.vlen = io.vlen ? &kDummyLen : nullptr;
  // algorithmic HBM bytes (SURVEY §8(d) pricing: every operand once, fp32): the input
  // pixels the conv reads (all of them for a k > 1 window, the strided subset for a 1x1),
  // the Res2Net addend, the K-concatenated second operand, weights, output, residual and
  // the two AFF operands
  const double px_out = (double)M;
  const double a_px = (d.s0.kh == 1 && d.s0.kw == 1) ? px_out : (double)d.nimg * d.s0.H * d.s0.W;
  double bytes = 4.0 * a_px * d.s0.cin * (io.s0b ? 2.0 : 1.0) + 4.0 * (double)d.N * d.K + 4.0 * px_out * d.N;
  if (io.s1) bytes += 4.0 * px_out * d.s1.cin;
  if (io.res) bytes += 4.0 * px_out * d.N;
  if (io.affx) bytes += 8.0 * px_out * d.N;
  check_operand(name, io.s0);
  check_operand(name, io.s0b);
  check_operand(name, io.s1);
  // the epilogue notes the output in the range word whenever the plan is not exact
  writes({Write{io.out, guard ? NOTED : AUX}});
  step(name, [d, cio, guard, scale_in](const Ctx& c) mutable {
    d.range_flag = guard ? c.flag : nullptr;
    d.range_in = scale_in ? c.flag : nullptr;
    d.s0.p = c.resolve(cio.s0);
    d.s0.p2 = c.resolve(cio.s0b);
    d.s1.p = c.resolve(cio.s1);
    d.out = c.resolve(cio.out);
    d.res = c.resolve(cio.res);
    d.affx = c.resolve(cio.affx);
    d.affy = c.resolve(cio.affy);
    d.gate = c.resolve(cio.gate);
    d.partial = c.resolve(cio.partial);
    d.rowbias = c.resolve(cio.rowbias);
    d.rowlen = c.resolve_i(cio.rowlen);
    d.s0.vlen = c.resolve_i(cio.vlen);
    return launch_conv(d, c.stream);
  }, conv_kernel_name(probe), bytes);
}

}  // namespace spk

// ============================================================================ C ABI
using namespace spk;

struct spk_model {
  Model m;
};

namespace {

FbankTables* g_tables[64] = {nullptr};
int g_tables_mels[64] = {0};
int g_tables_nb[64] = {0};
std::mutex g_tables_mu;

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const SpkError& e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_error(std::string("internal error: ") + e.what());
    return SPK_E_INVALID;
  }
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return SPK_OK;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  return SPK_E_HIP;
}

}  // namespace

bool spk::PlanPair::idle() const {
  for (const auto& e : last)
    if (hipEventQuery(e.second) != hipSuccess) return false;
  return true;
}

hipError_t spk::PlanPair::mark(hipStream_t s) {
  // one event per stream; an entry whose replay has completed is reused for a new stream, so
  // the list stays as long as the number of streams with a replay in flight
  hipEvent_t* ev = nullptr;
  for (auto& e : last)
    if (e.first == s) ev = &e.second;
  if (!ev)
    for (auto& e : last)
      if (hipEventQuery(e.second) == hipSuccess) {
        e.first = s;
        ev = &e.second;
        break;
      }
  if (!ev) {
    hipEvent_t e = nullptr;
    if (hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming); r != hipSuccess) return r;
    last.emplace_back(s, e);
    ev = &last.back().second;
  }
  return hipEventRecord(*ev, s);
}

spk::PlanPair::~PlanPair() {
  // reached only for an idle pair (Model::retired sweep, handle destruction): no device-wide
  // synchronisation here, which would stall every stream and break a caller's stream capture
  for (auto& kv : graphs) (void)hipGraphExecDestroy(kv.second);
  for (auto& e : last) (void)hipEventDestroy(e.second);
}

namespace {

// SPK_RANGE_MODE=twin: ECAPA / CAM++ keep the gated exact twin instead of the scaled split (A/B)
static bool range_scaled() {
  static const bool on = [] {
    const char* e = std::getenv("SPK_RANGE_MODE");
    return !(e && std::string(e) == "twin");
  }();
  return on;
}

std::unique_ptr<Plan> build_plan(spk_model_t* h, int B, int T, bool ragged, bool exact) {
  auto plan = std::make_unique<Plan>();
  Builder b(h->m, plan.get(), B, ragged, exact);
  // ECAPA / CAM++: unbounded activations everywhere (ReLU -> BN), so the whole plan would need
  // the exact twin; instead every split GEMM scales its operand by the range word (common.h)
  const int arch = h->m.cfg.arch;
  b.scaled = !exact && range_scaled() && (arch == SPK_ARCH_ECAPA || arch == SPK_ARCH_CAMPPLUS);
  plan->scaled = b.scaled;
  if (!exact) {
    // fp16x3 range guard on the model input (common.h)
    const size_t n = (size_t)B * T * h->m.cfg.feat_dim;
    b.writes({}).step("range_in", [n](const Ctx& c) { return launch_range_check(c.in, n, c.flag, c.stream); });
  }
  switch (h->m.cfg.arch) {
    case SPK_ARCH_ERES2NETV2: build_eres2net(b, T, true); break;
    case SPK_ARCH_ERES2NET: build_eres2net(b, T, false); break;
    case SPK_ARCH_ECAPA: build_ecapa(b, T); break;
    case SPK_ARCH_CAMPPLUS: build_campplus(b, T); break;
    case SPK_ARCH_RESNET: build_resnet(b, T, false); break;
    case SPK_ARCH_RES2NET: build_resnet(b, T, true); break;
    default: throw SpkError(SPK_E_UNSUPPORTED, "unknown arch");
  }
  plan->ws_bytes = (b.ws + 255) / 256 * 256;
  return plan;
}

std::shared_ptr<PlanPair> get_pair(spk_model_t* h, int B, int T, bool ragged = false) {
  std::lock_guard<std::mutex> lk(h->m.mu);
  const bool exact_only = h->m.force_exact || !conv_use_x3();
  const auto key = std::make_tuple(B, T, (int)ragged);
  h->m.plan_use[key] = ++h->m.plan_clock;
  auto it = h->m.plans.find(key);
  if (it != h->m.plans.end()) return it->second;
  if (ragged && h->m.cfg.arch != SPK_ARCH_CAMPPLUS && h->m.cfg.arch != SPK_ARCH_ECAPA)
    throw SpkError(SPK_E_UNSUPPORTED, "per-utterance lengths are implemented for CAM++ and ECAPA-TDNN only");
  // drop retired pairs that no forward holds any more and whose last replay has completed
  auto& rt = h->m.retired;
  rt.erase(std::remove_if(rt.begin(), rt.end(),
                          [](const std::shared_ptr<PlanPair>& p) { return p.use_count() == 1 && p->idle(); }),
           rt.end());
  if (h->m.plans.size() >= Model::kMaxPlans) {
    // evict the least recently used pair into the retired list: forwards still holding it,
    // and replays of its graphs still on a stream, keep its graphs alive until they are done
    auto victim = h->m.plans.begin();
    for (auto p = h->m.plans.begin(); p != h->m.plans.end(); ++p)
      if (h->m.plan_use[p->first] < h->m.plan_use[victim->first]) victim = p;
    h->m.plan_use.erase(victim->first);
    rt.push_back(victim->second);
    h->m.plans.erase(victim);
  }
  auto pair = std::make_shared<PlanPair>();
  if (!exact_only) pair->x3 = build_plan(h, B, T, ragged, false);
  pair->ex = build_plan(h, B, T, ragged, true);
  // shared layout: intermediates, then staging (input features, lengths, embeddings) and the
  // range word, all past both plans' intermediates
  size_t ws = std::max(pair->x3 ? pair->x3->ws_bytes : 0, pair->ex->ws_bytes);
  pair->in_bytes = (size_t)B * T * h->m.cfg.feat_dim * sizeof(float);
  pair->out_bytes = (size_t)B * h->m.cfg.embed_dim * sizeof(float);
  pair->len_bytes = ragged ? (size_t)B * sizeof(int32_t) : 0;
  pair->stage_in = ws;
  ws += (pair->in_bytes + 255) / 256 * 256;
  pair->stage_out = ws;
  ws += (pair->out_bytes + 255) / 256 * 256;
  pair->stage_len = ws;
  ws += (pair->len_bytes + 255) / 256 * 256;
  pair->stage_flag = ws;
  ws += 256;
  pair->ws_bytes = ws;
  h->m.plans.emplace(key, pair);
  return pair;
}

// the plan a measurement / introspection call describes: the fp16x3 one unless exact only
Plan* main_plan(const std::shared_ptr<PlanPair>& p) { return p->x3 ? p->x3.get() : p->ex.get(); }

}  // namespace

extern "C" {

int spk_version(void) { return 2; }   // include/spk_hip.h: ABI revision

const char* spk_last_error(void) { return g_last_error.c_str(); }

static int fbank_impl(const float* wav, const int64_t* wav_offsets, int32_t n_utt, float* feats,
                      const int64_t* frame_offsets, int32_t n_mels, int32_t mean_nor, void* stream, int32_t t_max) {
  return guarded([&]() -> int {
    if (n_utt < 0 || n_mels <= 3 || n_mels > 128 || (n_utt > 0 && (!wav || !wav_offsets || !feats || !frame_offsets))) {
      set_error("spk_fbank_f32: invalid argument");
      return SPK_E_INVALID;
    }
    int dev = 0;
    if (int rc = hip_check(hipGetDevice(&dev), "hipGetDevice")) return rc;
    if (dev < 0 || dev >= 64) return SPK_E_DEVICE;
    FbankTables* tab = nullptr;
    int mel_nb = 0;
    {
      std::lock_guard<std::mutex> lk(g_tables_mu);
      if (!g_tables[dev] || g_tables_mels[dev] != n_mels) {
        FbankTables host;
        std::memset(&host, 0, sizeof(host));
        if (build_fbank_tables(&host, n_mels, 16000.0) < 0) {
          set_error("spk_fbank_f32: unsupported n_mels");
          return SPK_E_UNSUPPORTED;
        }
        if (!g_tables[dev]) {
          if (int rc = hip_check(hipMalloc(&g_tables[dev], sizeof(FbankTables)), "hipMalloc(fbank tables)")) return rc;
        }
        if (int rc = hip_check(hipMemcpy(g_tables[dev], &host, sizeof(host), hipMemcpyHostToDevice), "hipMemcpy"))
          return rc;
        g_tables_mels[dev] = n_mels;
        g_tables_nb[dev] = host.mel_nb;
      }
      tab = g_tables[dev];
      mel_nb = g_tables_nb[dev];
    }
    return hip_check(launch_fbank(wav, wav_offsets, n_utt, feats, frame_offsets, n_mels, mean_nor, tab, mel_nb,
                                  reinterpret_cast<hipStream_t>(stream), t_max),
                     "fbank launch");
  });
}

int spk_fbank_f32(const float* wav, const int64_t* wav_offsets, int32_t n_utt, float* feats,
                  const int64_t* frame_offsets, int32_t n_mels, int32_t mean_nor, void* stream) {
  return fbank_impl(wav, wav_offsets, n_utt, feats, frame_offsets, n_mels, mean_nor, stream, 0);
}

int spk_fbank_f32_padded(const float* wav, const int64_t* wav_offsets, int32_t n_utt, float* feats,
                         const int64_t* frame_offsets, int32_t t_max, int32_t n_mels, int32_t mean_nor, void* stream) {
  if (t_max <= 0) {
    set_error("spk_fbank_f32_padded: t_max must be > 0");
    return SPK_E_INVALID;
  }
  return fbank_impl(wav, wav_offsets, n_utt, feats, frame_offsets, n_mels, mean_nor, stream, t_max);
}

int spk_model_create(const spk_model_config_t* cfg, const spk_weight_t* weights, int32_t n_weights, spk_model_t** out) {
  return guarded([&]() -> int {
    if (!cfg || !out || (n_weights > 0 && !weights)) {
      set_error("spk_model_create: null argument");
      return SPK_E_INVALID;
    }
    if (cfg->precision != SPK_PRECISION_FP32 && cfg->precision != SPK_PRECISION_FP16) {
      set_error("spk_model_create: precision must be SPK_PRECISION_FP32 or SPK_PRECISION_FP16");
      return SPK_E_INVALID;
    }
    auto h = std::make_unique<spk_model>();
    h->m.cfg = *cfg;
    h->m.fp16 = cfg->precision == SPK_PRECISION_FP16;
    if (int rc = hip_check(hipGetDevice(&h->m.device), "hipGetDevice")) return rc;
    for (int i = 0; i < n_weights; ++i) {
      const spk_weight_t& w = weights[i];
      if (!w.name || w.ndim < 0 || w.ndim > 4) {
        set_error("spk_model_create: bad weight descriptor");
        return SPK_E_INVALID;
      }
      std::vector<int64_t> shape(w.shape, w.shape + w.ndim);
      h->m.shapes[w.name] = shape;
      if (!w.data) continue;
      size_t n = 1;
      for (auto d : shape) n *= (size_t)d;
      Model::HostT t;
      t.shape = shape;
      t.data.assign(w.data, w.data + n);
      h->m.W[w.name] = std::move(t);
    }
    // pack every layer (a plan-less build), then upload once
    {
      // pack every weight either plan reads (the fused fp16x3 plan and the exact-fp32 one of
      // the range guard may use different layouts of the same tensor)
      for (const bool exact : {false, true}) {
        Builder b(h->m, nullptr, 1, false, exact);
        switch (cfg->arch) {
          case SPK_ARCH_ERES2NETV2: build_eres2net(b, 200, true); break;
          case SPK_ARCH_ERES2NET: build_eres2net(b, 200, false); break;
          case SPK_ARCH_ECAPA: build_ecapa(b, 200); break;
          case SPK_ARCH_CAMPPLUS: build_campplus(b, 200); break;
          case SPK_ARCH_RESNET: build_resnet(b, 200, false); break;
          case SPK_ARCH_RES2NET: build_resnet(b, 200, true); break;
          default: set_error("spk_model_create: unknown arch"); return SPK_E_UNSUPPORTED;
        }
      }
    }
    h->m.dweights_bytes = h->m.arena.size() * sizeof(float);
    if (int rc = hip_check(hipMalloc(&h->m.dweights, std::max<size_t>(h->m.dweights_bytes, 256)), "hipMalloc(weights)"))
      return rc;
    if (int rc = hip_check(hipMemcpy(h->m.dweights, h->m.arena.data(), h->m.dweights_bytes, hipMemcpyHostToDevice),
                           "hipMemcpy(weights)")) {
      (void)hipFree(h->m.dweights);
      return rc;
    }
    {
      // fp16 hi / lo planes of every packed weight for the fp16x3 GEMM (split on the device)
      const size_t n = h->m.dweights_bytes / sizeof(float);
      if (int rc = hip_check(hipMalloc(&h->m.dsplit, std::max<size_t>(2 * n * sizeof(uint16_t), 256)),
                             "hipMalloc(split weights)")) {
        (void)hipFree(h->m.dweights);
        return rc;
      }
      if (int rc = hip_check(launch_split_f16(h->m.dweights, h->m.dsplit, h->m.dsplit + n, n, nullptr),
                             "split_f16"))
        return rc;
      // the same planes in MFMA fragment order for the LDS-DMA GEMM (conv_gemm_f.hip): every
      // matrix wide enough for its 128-column tiles
      size_t fh = 0;
      for (auto& kv : h->m.packed)
        if (kv.second.N > 64 && kv.second.Kp > 0 && kv.second.Kp % 32 == 0) {
          kv.second.f_off = fh;
          fh += frag_halves(kv.second.N, kv.second.Kp);
        }
      if (fh) {
        if (int rc = hip_check(hipMalloc(&h->m.dfrag, fh * sizeof(uint16_t)), "hipMalloc(fragment weights)")) return rc;
        for (auto& kv : h->m.packed)
          if (kv.second.f_off != SIZE_MAX)
            if (int rc = hip_check(launch_pack_frag(h->m.dhi(kv.second.w_off), h->m.dlo(kv.second.w_off), kv.second.N,
                                                    kv.second.Kp, h->m.dfrag + kv.second.f_off, nullptr),
                                   "pack_frag"))
              return rc;
      }
      if (int rc = hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize")) return rc;
    }
    {
      // fp16x3 range guard (common.h): a weight past fp16's range forces the exact path
      // (the activations' range word lives in each forward's workspace)
      h->m.force_exact = !(h->m.gemm_wmax < 65504.0f);   // the split GEMM operands only
    }
    h->m.uploaded = true;
    h->m.arena.clear();
    h->m.arena.shrink_to_fit();
    h->m.W.clear();
    *out = h.release();
    return SPK_OK;
  });
}

int spk_model_destroy(spk_model_t* model) {
  if (!model) return SPK_OK;
  // the caller guarantees no forward of this handle is still being enqueued; replays already
  // on a stream must finish before their executable graphs go
  bool busy = false;
  for (auto& kv : model->m.plans) busy = busy || !kv.second->idle();
  for (auto& p : model->m.retired) busy = busy || !p->idle();
  if (busy) (void)hipDeviceSynchronize();
  if (model->m.dweights) (void)hipFree(model->m.dweights);
  if (model->m.dsplit) (void)hipFree(model->m.dsplit);
  if (model->m.dfrag) (void)hipFree(model->m.dfrag);
  delete model;
  return SPK_OK;
}

int spk_model_workspace_bytes(spk_model_t* model, int32_t B, int32_t T, size_t* bytes) {
  return guarded([&]() -> int {
    if (!model || !bytes || B <= 0 || T <= 0) {
      set_error("spk_model_workspace_bytes: invalid argument");
      return SPK_E_INVALID;
    }
    *bytes = get_pair(model, B, T)->ws_bytes;
    return SPK_OK;
  });
}

int spk_model_flops(spk_model_t* model, int32_t T, double* flops) {
  return guarded([&]() -> int {
    if (!model || !flops || T <= 0) {
      set_error("spk_model_flops: invalid argument");
      return SPK_E_INVALID;
    }
    Builder b(model->m, nullptr, 1);
    switch (model->m.cfg.arch) {
      case SPK_ARCH_ERES2NETV2: build_eres2net(b, T, true); break;
      case SPK_ARCH_ERES2NET: build_eres2net(b, T, false); break;
      case SPK_ARCH_ECAPA: build_ecapa(b, T); break;
      case SPK_ARCH_CAMPPLUS: build_campplus(b, T); break;
      case SPK_ARCH_RESNET: build_resnet(b, T, false); break;
      case SPK_ARCH_RES2NET: build_resnet(b, T, true); break;
      default: return SPK_E_UNSUPPORTED;
    }
    *flops = 2.0 * b.macs_per_utt;
    return SPK_OK;
  });
}

// SPK_GRAPH=0 launches every step directly instead of replaying a captured hipGraph
static bool use_graphs() {
  static const bool on = [] {
    const char* e = std::getenv("SPK_GRAPH");
    return !(e && std::string(e) == "0");
  }();
  return on;
}

// Both plans of the pair are cut into the same segments, every segment ends on the last
// step, and they lay the workspace out alike (a twin then writes exactly the buffers its
// split segment wrote); SPK_GUARD_SEGMENTS=0 forces the whole-plan twin (A/B, diagnostics)
static bool segmented(const PlanPair& pp) {
  static const bool on = [] {
    const char* e = std::getenv("SPK_GUARD_SEGMENTS");
    return !(e && std::string(e) == "0");
  }();
  const Plan &x = *pp.x3, &e = *pp.ex;
  return on && !x.seg_end.empty() && x.seg_end.size() == e.seg_end.size() && x.seg_end.back() == x.steps.size() &&
         e.seg_end.back() == e.steps.size() && x.allocs == e.allocs;
}

// Enqueue one forward: the range word is zeroed, the fp16x3 plan runs (its producers note
// range overflows in the word), then the exact-fp32 plan runs with every launch gated on the
// word (common.h SPK_GATE): a batch whose activations left fp16's range is recomputed on the
// exact kernels and overwrites the embeddings, all on `stream`, with no host round trip.
// `exact` runs the exact plan alone (spk_model_forward_exact).
static int enqueue_steps(const char* fn, const PlanPair& pp, const Ctx& base, bool exact) {
  auto run = [&](const Plan& p, size_t i0, size_t i1, int* flag, const int* gate) -> int {
    Ctx c = base;
    c.flag = flag;
    GateScope g(gate);
    for (size_t i = i0; i < i1; ++i) {
      hipError_t e = p.steps[i](c);
      if (e != hipSuccess) {
        set_error(std::string(fn) + ": step '" + p.names[i] + "': " + hipGetErrorString(e));
        return SPK_E_HIP;
      }
    }
    return SPK_OK;
  };
  if (exact || !pp.x3) return run(*pp.ex, 0, pp.ex->steps.size(), nullptr, nullptr);
  int* word = reinterpret_cast<int*>(base.ws + pp.stage_flag);
  // diagnostics (tools/race_probe.py): SPK_WORD_RESET=memset zeroes the word with a
  // 4-byte hipMemsetAsync (a memset node in the captured graph) instead of the kernel node
  static const bool memset_reset = [] {
    const char* e = std::getenv("SPK_WORD_RESET");
    return e && std::string(e) == "memset";
  }();
  if (memset_reset) {
    if (int rc = hip_check(hipMemsetAsync(word, 0, sizeof(int), base.stream), "range word memset")) return rc;
  } else if (int rc = hip_check(launch_word_reset(word, base.stream), "range word reset")) {
    return rc;
  }
  static const bool no_rerun = std::getenv("SPK_DIAG_NO_RERUN") != nullptr;   // diagnostics only
  if (pp.x3->scaled) return run(*pp.x3, 0, pp.x3->steps.size(), word, nullptr);   // no twin
  if (segmented(pp)) {
    // segment by segment: a segment's exact twin, gated on the word, follows it only where one
    // of its split-GEMM operands is not statically bounded below kRangeLimit (Builder::segment);
    // a flagged segment is recomputed before any later segment reads its outputs
    const Plan &x = *pp.x3, &e = *pp.ex;
    for (size_t sgi = 0; sgi < x.seg_end.size(); ++sgi) {
      const size_t x0 = sgi ? x.seg_end[sgi - 1] : 0, e0 = sgi ? e.seg_end[sgi - 1] : 0;
      if (int rc = run(x, x0, x.seg_end[sgi], word, nullptr)) return rc;
      if (x.seg_twin[sgi] && !no_rerun)
        if (int rc = run(e, e0, e.seg_end[sgi], nullptr, word)) return rc;
    }
    return SPK_OK;
  }
  if (int rc = run(*pp.x3, 0, pp.x3->steps.size(), word, nullptr)) return rc;
  if (no_rerun) return SPK_OK;
  return run(*pp.ex, 0, pp.ex->steps.size(), nullptr, word);
}

// Replay the forward as one hipGraph: inputs are copied into the workspace's staging regions,
// the graph (captured once per workspace address on a private stream) runs on the caller's
// stream, and the embeddings are copied out.  Removes the per-kernel launch cost (CAM++ has
// ~280 launches per forward).
static int run_graph(const char* fn, spk_model_t* model, PlanPair& pp, const float* feats, const int32_t* lengths,
                     char* ws, float* emb_out, hipStream_t stream, bool exact) {
  char* in_s = ws + pp.stage_in;
  char* out_s = ws + pp.stage_out;
  char* len_s = ws + pp.stage_len;
  if (int rc = hip_check(hipMemcpyAsync(in_s, feats, pp.in_bytes, hipMemcpyDeviceToDevice, stream), "stage in"))
    return rc;
  if (lengths && pp.len_bytes)
    if (int rc = hip_check(hipMemcpyAsync(len_s, lengths, pp.len_bytes, hipMemcpyDeviceToDevice, stream),
                           "stage lengths"))
      return rc;
  // the exact-only replay (spk_model_forward_exact) is keyed apart from the guarded one
  const void* key = exact ? static_cast<const void*>(ws + 1) : static_cast<const void*>(ws);
  hipGraphExec_t exec = nullptr;
  {
    std::lock_guard<std::mutex> lk(model->m.mu);
    auto it = pp.graphs.find(key);
    if (it != pp.graphs.end()) exec = it->second;
  }
  if (!exec) {
    hipStream_t cap = nullptr;
    if (int rc = hip_check(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking), "hipStreamCreate")) return rc;
    Ctx c{ws, reinterpret_cast<const float*>(in_s), reinterpret_cast<float*>(out_s), cap,
          lengths ? reinterpret_cast<const int*>(len_s) : nullptr};
    hipGraph_t graph = nullptr;
    int rc = hip_check(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
    if (rc == SPK_OK) rc = enqueue_steps(fn, pp, c, exact);
    const hipError_t ee = hipStreamEndCapture(cap, &graph);
    if (rc == SPK_OK) rc = hip_check(ee, "hipStreamEndCapture");
    // diagnostics (the memset-node evidence): SPK_GRAPH_DOT=<path> writes the captured
    // graph's nodes and dependency edges (hipGraphDebugDotPrint) before it is instantiated
    if (rc == SPK_OK)
      if (const char* dot = std::getenv("SPK_GRAPH_DOT"))
        rc = hip_check(hipGraphDebugDotPrint(graph, dot, hipGraphDebugDotFlagsVerbose), "hipGraphDebugDotPrint");
    if (rc == SPK_OK) rc = hip_check(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0), "hipGraphInstantiate");
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipStreamDestroy(cap);
    if (rc != SPK_OK) return rc;
    std::lock_guard<std::mutex> lk(model->m.mu);
    auto ins = pp.graphs.emplace(key, exec);
    if (!ins.second) {   // another thread captured the same one first
      (void)hipGraphExecDestroy(exec);
      exec = ins.first->second;
    }
  }
  if (int rc = hip_check(hipGraphLaunch(exec, stream), "hipGraphLaunch")) return rc;
  if (int rc = hip_check(hipMemcpyAsync(emb_out, out_s, pp.out_bytes, hipMemcpyDeviceToDevice, stream), "stage out"))
    return rc;
  // completion marker of this replay on this stream (PlanPair::last): an evicted pair is
  // freed only after the replays on every stream are done
  {
    std::lock_guard<std::mutex> lk(model->m.mu);
    return hip_check(pp.mark(stream), "hipEventRecord");
  }
}

static int run_forward(const char* fn, spk_model_t* model, const float* feats, int32_t B, int32_t T,
                       const int32_t* lengths, void* workspace, size_t workspace_bytes, float* emb_out, void* stream,
                       bool exact = false) {
  if (!model || !feats || !emb_out || B <= 0 || T <= 0) {
    set_error(std::string(fn) + ": invalid argument");
    return SPK_E_INVALID;
  }
  int dev = 0;
  if (int rc = hip_check(hipGetDevice(&dev), "hipGetDevice")) return rc;
  if (dev != model->m.device) {
    set_error(std::string(fn) + ": handle belongs to another device");
    return SPK_E_DEVICE;
  }
  const std::shared_ptr<PlanPair> pp = get_pair(model, B, T, lengths != nullptr);
  if (workspace_bytes < pp->ws_bytes || !workspace) {
    set_error(std::string(fn) + ": workspace too small (need " + std::to_string(pp->ws_bytes) + " bytes)");
    return SPK_E_WORKSPACE;
  }
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (use_graphs())
    return run_graph(fn, model, *pp, feats, lengths, reinterpret_cast<char*>(workspace), emb_out, s, exact);
  Ctx c{reinterpret_cast<char*>(workspace), feats, emb_out, s, lengths};
  return enqueue_steps(fn, *pp, c, exact);
}

int spk_model_forward(spk_model_t* model, const float* feats, int32_t B, int32_t T, void* workspace,
                      size_t workspace_bytes, float* emb_out, void* stream) {
  return guarded([&]() -> int {
    return run_forward("spk_model_forward", model, feats, B, T, nullptr, workspace, workspace_bytes, emb_out, stream);
  });
}

int spk_model_workspace_bytes_lengths(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, size_t* bytes) {
  return guarded([&]() -> int {
    if (!model || !bytes || B <= 0 || T <= 0) {
      set_error("spk_model_workspace_bytes_lengths: invalid argument");
      return SPK_E_INVALID;
    }
    *bytes = get_pair(model, B, T, ragged != 0)->ws_bytes;
    return SPK_OK;
  });
}

int spk_model_forward_lengths(spk_model_t* model, const float* feats, int32_t B, int32_t T, const int32_t* lengths,
                              void* workspace, size_t workspace_bytes, float* emb_out, void* stream) {
  return guarded([&]() -> int {
    return run_forward("spk_model_forward_lengths", model, feats, B, T, lengths, workspace, workspace_bytes, emb_out,
                       stream);
  });
}

int spk_model_guard_plan(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, int32_t* n_segments,
                         int32_t* n_twin_segments, int32_t* n_gated_steps) {
  return guarded([&]() -> int {
    if (!model || B <= 0 || T <= 0 || !n_segments || !n_twin_segments || !n_gated_steps) {
      set_error("spk_model_guard_plan: invalid argument");
      return SPK_E_INVALID;
    }
    std::shared_ptr<PlanPair> pp = get_pair(model, B, T, ragged != 0);
    *n_segments = *n_twin_segments = *n_gated_steps = 0;
    if (!pp->x3) return SPK_OK;
    if (pp->x3->scaled) {   // scaled split: one segment, nothing gated behind it
      *n_segments = 1;
      return SPK_OK;
    }
    if (!segmented(*pp)) {
      *n_segments = *n_twin_segments = 1;
      *n_gated_steps = (int32_t)pp->ex->steps.size();
      return SPK_OK;
    }
    const Plan& e = *pp->ex;
    *n_segments = (int32_t)e.seg_end.size();
    for (size_t i = 0; i < e.seg_end.size(); ++i)
      if (pp->x3->seg_twin[i]) {
        ++*n_twin_segments;
        *n_gated_steps += (int32_t)(e.seg_end[i] - (i ? e.seg_end[i - 1] : 0));
      }
    return SPK_OK;
  });
}

int spk_model_forward_exact(spk_model_t* model, const float* feats, int32_t B, int32_t T, const int32_t* lengths,
                            void* workspace, size_t workspace_bytes, float* emb_out, void* stream) {
  return guarded([&]() -> int {
    return run_forward("spk_model_forward_exact", model, feats, B, T, lengths, workspace, workspace_bytes, emb_out,
                       stream, true);
  });
}

int spk_model_range_check(spk_model_t* model, int32_t B, int32_t T, int32_t ragged, const void* workspace,
                          void* stream, int32_t* overflowed) {
  return guarded([&]() -> int {
    if (!model || !overflowed || !workspace || B <= 0 || T <= 0) {
      set_error("spk_model_range_check: invalid argument");
      return SPK_E_INVALID;
    }
    const auto pp = get_pair(model, B, T, ragged != 0);
    *overflowed = 0;
    if (!pp->x3) return SPK_OK;   // exact-only handle: nothing is guarded
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    int v = 0;
    const char* word = reinterpret_cast<const char*>(workspace) + pp->stage_flag;
    if (int rc = hip_check(hipMemcpyAsync(&v, word, sizeof(int), hipMemcpyDeviceToHost, s), "range word")) return rc;
    if (int rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize")) return rc;
    *overflowed = v != 0;
    return SPK_OK;
  });
}

// Diagnostics (tools/race_probe*.py; not in include/spk_hip.h): run the first `nsteps` steps
// of the fp16x3 (exact = 0) or exact (exact = 1) plan directly on `stream`, the range word
// being the workspace slot of a guarded forward (not reset here).
int spk_diag_run_prefix(spk_model_t* model, const float* feats, int32_t B, int32_t T, void* workspace,
                        size_t workspace_bytes, float* emb_out, void* stream, int32_t nsteps, int32_t exact) {
  return guarded([&]() -> int {
    if (!model || !feats || !emb_out || !workspace || B <= 0 || T <= 0) return SPK_E_INVALID;
    const auto pp = get_pair(model, B, T);
    if (workspace_bytes < pp->ws_bytes) return SPK_E_WORKSPACE;
    Plan* p = exact || !pp->x3 ? pp->ex.get() : pp->x3.get();
    Ctx c{reinterpret_cast<char*>(workspace), feats, emb_out, reinterpret_cast<hipStream_t>(stream)};
    c.flag = exact ? nullptr : reinterpret_cast<int*>(c.ws + pp->stage_flag);
    for (int i = 0; i < nsteps && i < (int)p->steps.size(); ++i) {
      hipError_t e = p->steps[i](c);
      if (e != hipSuccess) {
        set_error("step '" + p->names[i] + "': " + hipGetErrorString(e));
        return SPK_E_HIP;
      }
    }
    return SPK_OK;
  });
}

int spk_model_plan_size(spk_model_t* model, int32_t B, int32_t T, int32_t* n_steps) {
  return guarded([&]() -> int {
    if (!model || !n_steps || B <= 0 || T <= 0) return SPK_E_INVALID;
    *n_steps = (int32_t)main_plan(get_pair(model, B, T))->steps.size();
    return SPK_OK;
  });
}

int spk_model_plan_step(spk_model_t* model, int32_t B, int32_t T, int32_t i, char* name, int32_t name_len,
                        char* kernel, int32_t kernel_len, double* flops) {
  return guarded([&]() -> int {
    if (!model || B <= 0 || T <= 0) return SPK_E_INVALID;
    const auto pp = get_pair(model, B, T);
    Plan* p = main_plan(pp);
    if (i < 0 || i >= (int)p->steps.size()) return SPK_E_INVALID;
    if (name && name_len > 0) { std::strncpy(name, p->names[i].c_str(), name_len - 1); name[name_len - 1] = 0; }
    if (kernel && kernel_len > 0) {
      std::strncpy(kernel, p->kernels[i].c_str(), kernel_len - 1);
      kernel[kernel_len - 1] = 0;
    }
    if (flops) *flops = p->flops[i];
    return SPK_OK;
  });
}

int spk_model_plan_step_bytes(spk_model_t* model, int32_t B, int32_t T, int32_t i, double* bytes) {
  return guarded([&]() -> int {
    if (!model || !bytes || B <= 0 || T <= 0) return SPK_E_INVALID;
    const auto pp = get_pair(model, B, T);
    Plan* p = main_plan(pp);
    if (i < 0 || i >= (int)p->steps.size()) return SPK_E_INVALID;
    *bytes = p->bytes[i];
    return SPK_OK;
  });
}

int spk_model_forward_timed(spk_model_t* model, const float* feats, int32_t B, int32_t T, void* workspace,
                            size_t workspace_bytes, float* emb_out, void* stream, float* step_ms, int32_t max_steps) {
  return guarded([&]() -> int {
    if (!model || !feats || !emb_out || !step_ms || B <= 0 || T <= 0) return SPK_E_INVALID;
    const auto pp = get_pair(model, B, T);
    Plan* plan = main_plan(pp);
    const int n = (int)plan->steps.size();
    if (max_steps < n) { set_error("spk_model_forward_timed: step_ms too short"); return SPK_E_INVALID; }
    if (workspace_bytes < pp->ws_bytes) return SPK_E_WORKSPACE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::vector<hipEvent_t> ev(n + 1);
    for (auto& e : ev)
      if (int rc = hip_check(hipEventCreate(&e), "hipEventCreate")) return rc;
    Ctx c{reinterpret_cast<char*>(workspace), feats, emb_out, s};
    c.flag = pp->x3 ? reinterpret_cast<int*>(c.ws + pp->stage_flag) : nullptr;   // no exact re-run here
    int rc = SPK_OK;
    (void)hipEventRecord(ev[0], s);
    for (int i = 0; i < n && rc == SPK_OK; ++i) {
      hipError_t e = plan->steps[i](c);
      if (e != hipSuccess) {
        set_error("step '" + plan->names[i] + "': " + hipGetErrorString(e));
        rc = SPK_E_HIP;
      }
      (void)hipEventRecord(ev[i + 1], s);
    }
    if (rc == SPK_OK) rc = hip_check(hipEventSynchronize(ev[n]), "hipEventSynchronize");
    for (int i = 0; i < n && rc == SPK_OK; ++i) (void)hipEventElapsedTime(&step_ms[i], ev[i], ev[i + 1]);
    for (auto& e : ev) (void)hipEventDestroy(e);
    return rc;
  });
}

}  // extern "C"
