// ERes2Net / ERes2NetV2 launch plan.
//
// Reference forwards: ERes2NetV2.py:65-91 (BasicBlockERes2NetV2), :132-159 (…AFF),
// :235-254 (model); ERes2Net.py:61-87, :125-152, :208-231; fusion.py:22-28 (AFF);
// pooling_layers.py:47-55 (TSTP).
//
// Data layout (workspace, channels-last [B, F, T, C]):
//   * every block output is dense C = planes*expansion;
//   * the conv1 output "T1" and the Res2Net concat buffer "CAT" hold `scale` slices of
//     `width` channels, each zero-padded to a multiple of 4 (width 26 -> 28) so float4
//     loads stay aligned; torch.split / torch.cat are just slice offsets.  T1 is planar
//     (slice i is its own dense [px][wp] plane, written by conv1's split epilogue): the 3x3
//     conv of a slice then reads whole cache lines instead of 112 of every 224 bytes;
//     CAT stays interleaved, the K operand conv3 reads in one piece;
//   * conv3 + bn3 + shortcut conv + its BN + residual add + Hardtanh are ONE GEMM: the
//     shortcut input is K-concatenated as a second operand with its own stride;
//   * `sp + spx` is fused into the 3x3 conv's operand load; AFF is two GEMMs, the second
//     applying x*(1+tanh a) + y*(1-tanh a) in its epilogue.
#include <cmath>
#include <cstdlib>
#include <string>

#include "aff.h"
#include "misc.h"
#include "res2block.h"
#include "runtime.h"

namespace spk {

namespace {

struct T4 {
  Buf buf;
  int ld = 0, H = 0, W = 0, C = 0;   // C = physical channels
};

ConvSrc src_of(const Ctx*, const T4& t, int cin, int k, int stride, int pad) {
  ConvSrc s;
  s.ld = t.ld; s.H = t.H; s.W = t.W; s.cin = cin;
  s.kh = s.kw = k; s.sh = s.sw = stride; s.ph = s.pw = pad;
  return s;
}

int count_blocks(const Model& m, const std::string& layer) {
  int n = 0;
  while (m.has(layer + "." + std::to_string(n) + ".conv1.weight")) ++n;
  return n;
}

struct ERes2Builder {
  Builder& b;
  Model& m;
  bool v2;
  int scale, expansion;
  double base_width;
  Buf T1, CAT, MID, FB;   // block scratch, sized for the largest layer
  // fp16x3 range guard by segment (runtime.h Plan::seg_end): the plan is cut after every block
  // and once at the end; a segment needs its gated exact twin only if a split-GEMM operand in
  // it has no static bound below kRangeLimit.  Bounds: Hardtanh(0, 20) outputs (every block
  // output and every in-block activation), |AFF| <= 2 max(|x|, |y|), a conv's |W x + b| <=
  // max_n sum_k |w_nk| |x|max + |b|max from the packed weights; the stem output (ReLU of the
  // model input's conv) has none, so the first block's segment keeps its twin.
  static constexpr double kHt = 20.0;
  bool seg_hot = false;
  void need(double bound) {
    if (!(bound < (double)kRangeLimit)) seg_hot = true;
  }
  void close_segment() {
    b.segment(seg_hot);
    seg_hot = false;
  }

  ERes2Builder(Builder& bb, bool isv2) : b(bb), m(bb.m), v2(isv2) {
    // ERes2Net (ERes2Net.py) fixes scale 2 / expansion 2 / baseWidth 32; ERes2Net_huge
    // (ERes2Net_huge.py:30-152) uses 3 / 4 / 24 — taken from the config when given.
    scale = m.cfg.scale ? m.cfg.scale : 2;
    expansion = m.cfg.expansion ? m.cfg.expansion : 2;
    base_width = m.cfg.base_width ? m.cfg.base_width : (v2 ? 26 : 32);
    if (scale < 1 || expansion < 1) throw SpkError(SPK_E_INVALID, "bad scale/expansion");
  }

  double pix(const T4& t) const { return (double)t.H * t.W; }

  // ASTP (pooling_layers.py:93-104, global_context_att=False) of x [B, F, T, C] into stats
  // [B, 2*F*C] ((f, c) order, as TSTP): linear1 over the reference's (C*F) channels is a conv
  // whose kernel spans the F frequency rows (weight [bottleneck, C*F] read as [bottleneck][C][F]
  // -- the same memory -- so tap f, channel c is reference channel c*F + f), + tanh; linear2
  // writes its C*F logits in (f, c) order; one pass then pools every (f, c) over time.
  void astp(const T4& x, const Buf& stats) {
    const int B = b.B, F = x.H, T = x.W, C = x.C;
    const std::string w1 = "pool.linear1.weight", w1cf = "pool.linear1.weight#cf";
    const int nb = (int)m.dim(w1, 0);
    if (m.dim(w1, 1) != (int64_t)C * F || m.dim("pool.linear2.weight", 0) != (int64_t)C * F)
      throw SpkError(SPK_E_WEIGHTS, "pool.linear1/2: in_dim != channels x frequency rows of the pooled map");
    if (!m.uploaded && !m.W.count(w1cf)) {
      Model::HostT t = m.get(w1);
      t.shape = {nb, C, F, 1};
      m.W[w1cf] = std::move(t);
    }
    const ChanMap bott = ChanMap::dense(nb);
    const Packed& p1 = m.pack("pool.linear1", bott, {Part{w1cf, "pool.linear1.bias", "", ChanMap::dense(C, 1), 0, 0}}, F * C);
    ChanMap fc;   // linear2 output: reference channel c*F + f -> column f*C + c
    fc.n_phys = F * C;
    fc.phys.resize((size_t)F * C);
    for (int c = 0; c < C; ++c)
      for (int f = 0; f < F; ++f) fc.phys[(size_t)c * F + f] = f * C + c;
    const Packed& p2 = m.pack("pool.linear2", fc, {Part{"pool.linear2.weight", "pool.linear2.bias", "", bott, 0, 0}}, nb);
    b.macs_per_utt += 2.0 * T * (double)C * F * nb;
    if (!b.plan) return;
    const int ldb = bott.n_phys;
    const Buf A = b.alloc((size_t)B * T * ldb), L = b.alloc((size_t)B * T * F * C);
    ConvDesc d1;
    d1.nimg = B; d1.Ho = 1; d1.Wo = T;
    d1.s0.ld = x.ld; d1.s0.H = F; d1.s0.W = T; d1.s0.cin = C;
    d1.s0.kh = F; d1.s0.kw = 1;
    d1.ldo = ldb; d1.act = ACT_TANH;
    Builder::ConvIO io1; io1.s0 = x.buf; io1.out = A;
    b.conv("pool.linear1", d1, p1, io1);
    ConvDesc d2;
    d2.nimg = B; d2.Ho = 1; d2.Wo = T;
    d2.s0.ld = ldb; d2.s0.H = 1; d2.s0.W = T; d2.s0.cin = ldb;
    d2.ldo = F * C;
    Builder::ConvIO io2; io2.s0 = A; io2.out = L;
    b.conv("pool.linear2", d2, p2, io2);
    const T4 xx = x;
    b.step("pool", [=](const Ctx& c) {
      return launch_astp_pool(c.resolve(L), F * C, c.resolve(xx.buf), xx.ld, B, F, T, C, c.resolve(stats), c.stream);
    });
  }

  // AFF bottleneck layout: C/4 channels, up to 64 of them padded to a multiple of 32 (the
  // fused kernel's MFMA tiles; for the two-conv form the second conv's K-tile is one whole
  // tap, so the buffer-resource loader applies); padding channels have zero weights and
  // bias, so they hold silu(0) = 0.
  static ChanMap aff_mid(int C) { return ChanMap::dense(C / 4, C / 4 <= 64 ? 32 : 4); }

  // AFF(x, y) -> out (fusion.py:22-28); x, y, out share geometry, C logical channels each.
  // |x| <= bx, |y| <= by; returns the bound of |out|.
  double aff(const std::string& p, const T4& x, const T4& y, int C, const T4& out, double bx, double by) {
    const int inter = C / 4;
    const ChanMap xin = ChanMap::dense(C);
    const int cp = xin.n_phys;
    const ChanMap mid = aff_mid(C);
    const Packed& a0 = m.pack(p + ".la0", mid,
                              {Part{p + ".local_att.0.weight", p + ".local_att.0.bias", p + ".local_att.1", xin, 0, 0},
                               Part{p + ".local_att.0.weight", p + ".local_att.0.bias", p + ".local_att.1", xin, C, cp}},
                              2 * cp);
    const Packed& a1 = m.pack(p + ".la3", xin,
                              {Part{p + ".local_att.3.weight", p + ".local_att.3.bias", p + ".local_att.4", mid, 0, 0}},
                              mid.n_phys);
    const double m0 = pix(x) * 2.0 * C * inter, m3 = pix(x) * (double)inter * C;
    const double bin = std::max(bx, by);
    need(bin);                                  // local_att.0 reads cat(x, y)
    need(Builder::bound(a0, bin));              // local_att.3 reads SiLU(BN(local_att.0)): |silu z| <= |z|
    const double bout = 2.0 * bin;
    if (!b.plan) {
      b.macs_per_utt += m0 + m3;
      return bout;
    }
    if (b.x3() && aff_x3_supported(cp, mid.n_phys)) {
      // one fused kernel (aff.hip): x and y read once, h never leaves registers
      b.macs_per_utt += m0 + m3;
      AffDesc ad;
      ad.M = b.B * x.H * x.W;
      ad.cp = cp; ad.nmid = mid.n_phys;
      ad.ldx = x.ld; ad.ldy = y.ld; ad.ldo = out.ld;
      ad.w1 = m.dptr(a0.w_off); ad.w1h = m.dhi(a0.w_off); ad.w1l = m.dlo(a0.w_off);
      ad.b1 = m.dptr(a0.b_off); ad.kp1 = a0.Kp;
      ad.w2 = m.dptr(a1.w_off); ad.w2h = m.dhi(a1.w_off); ad.w2l = m.dlo(a1.w_off);
      ad.b2 = m.dptr(a1.b_off); ad.kp2 = a1.Kp;
      if (!a0.has_bias || !a1.has_bias) throw SpkError(SPK_E_WEIGHTS, p + ": AFF convs without bias");
      const double bytes = 4.0 * ad.M * (3.0 * C) + 4.0 * ((double)a0.N * a0.K + (double)a1.N * a1.K);
      const Buf xb = x.buf, yb = y.buf, ob = out.buf;
      b.step(p + ".aff", [ad, xb, yb, ob](const Ctx& c) mutable {
        ad.x = c.resolve(xb);
        ad.y = c.resolve(yb);
        ad.out = c.resolve(ob);
        ad.range_flag = c.flag;
        return launch_aff_x3(ad, c.stream);
      }, aff_x3_kernel_name(cp, mid.n_phys), bytes);
      return bout;
    }
    b.macs_per_utt += m0;
    ConvDesc d;
    d.nimg = b.B; d.Ho = x.H; d.Wo = x.W;
    d.s0 = src_of(nullptr, x, cp, 1, 1, 0);
    d.s1 = src_of(nullptr, y, cp, 1, 1, 0);
    d.ldo = mid.n_phys;
    d.act = ACT_SILU;
    Builder::ConvIO io;
    io.s0 = x.buf; io.s1 = y.buf; io.out = MID;
    b.conv(p + ".local_att.0", d, a0, io);
    ConvDesc e;
    e.nimg = b.B; e.Ho = x.H; e.Wo = x.W;
    T4 midt{MID, mid.n_phys, x.H, x.W, mid.n_phys};
    e.s0 = src_of(nullptr, midt, mid.n_phys, 1, 1, 0);
    e.ldo = out.ld; e.ldx = x.ld; e.ldy = y.ld;
    Builder::ConvIO io2;
    io2.s0 = MID; io2.out = out.buf; io2.affx = x.buf; io2.affy = y.buf;
    b.macs_per_utt += m3;
    b.conv(p + ".local_att.3", e, a1, io2);
    return bout;
  }

  // The whole block as one fused kernel (res2block.hip), scale 2, fp16x3 path, uniform
  // lengths: stage 1 (slices <= 32 wide, 128 output channels) -- identity shortcut from 128
  // channels, or the stage's first block with a 1x1 stride-1 projection shortcut from 64.
  // (ERes2Net's BasicBlockERes2Net, ERes2Net.py:61-87, has the forward of ERes2NetV2's block,
  // ERes2NetV2.py:65-91: ERes2Net-large's stage 1 -- width 32 -- takes the same kernel.)
  // Stage 2 runs as four kernels (1x1 GEMM, two halo 3x3 convs, 1x1 + residual): a fused
  // stage-2 kernel (rounds 3-4) measured slower than those after the round-4 epilogue work
  // (ERes2NetV2 layer2 6.77 vs 5.91 ms) and was removed in round 5.
  bool fusable(const std::string& p, const T4& x, int stride, int width, int Cout, bool use_aff) const {
    const bool sc = m.has(p + ".shortcut.0.weight");
    const bool common = !use_aff && scale == 2 && x.ld == x.C && !b.ragged && b.x3() &&
                        std::getenv("SPK_NO_BLOCK_FUSION") == nullptr;
    // stage 1 (res2block.hip): slices <= 32, 128 output channels, identity or 64 -> 128 projection
    const bool s1 = stride == 1 && width <= 32 && Cout == 128 &&
                    (sc ? (x.C == 64 && std::getenv("SPK_NO_PROJ_FUSION") == nullptr) : x.C == 128);
    return common && s1;
  }

  bool fused_block(const std::string& p, const T4& x, int stride, int width, int Cout, Buf outbuf, T4& out) {
    const ChanMap xin = ChanMap::dense(x.C);
    const ChanMap om = ChanMap::dense(Cout);
    const int sw = 32;                      // padded slice width of the fused kernel
    const ChanMap sl = ChanMap::slices(width, 2, sw);
    const ChanMap wsw = ChanMap::dense(width, sw);
    const bool proj = m.has(p + ".shortcut.0.weight");
    const Packed& c1 = m.pack(p + ".conv1#fused", sl, {Part{p + ".conv1.weight", "", p + ".bn1", xin, 0, 0}}, x.C);
    const Packed& ca = m.pack(p + ".convs.0#fused", wsw, {Part{p + ".convs.0.weight", "", p + ".bns.0", wsw, 0, 0}}, 9 * sw);
    const Packed& cb = m.pack(p + ".convs.1#fused", wsw, {Part{p + ".convs.1.weight", "", p + ".bns.1", wsw, 0, 0}}, 9 * sw);
    std::vector<Part> parts3{Part{p + ".conv3.weight", "", p + ".bn3", sl, 0, 0}};
    if (proj) parts3.push_back(Part{p + ".shortcut.0.weight", "", p + ".shortcut.1", xin, 0, 2 * sw});
    const Packed& c3 = m.pack(p + ".conv3#fused", om, parts3, 2 * sw + (proj ? x.C : 0));
    const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
    const double px = (double)Ho * Wo;   // output pixels (a strided block reads only those inputs)
    b.macs_per_utt += px * x.C * (double)width * 2 + 2.0 * px * 9.0 * width * width + px * (double)width * 2 * Cout +
                      (proj ? px * x.C * (double)Cout : 0.0);
    out = T4{outbuf, Cout, Ho, Wo, Cout};
    if (b.plan) {
      Res2Desc d;
      d.nimg = b.B; d.H = Ho; d.W = Wo; d.C = x.C; d.width = width;
      d.stride = stride; d.Hin = x.H; d.Win = x.W;
      d.Cout = Cout; d.proj = proj;
      d.w1h = m.dhi(c1.w_off); d.w1l = m.dlo(c1.w_off); d.b1 = m.dptr(c1.b_off);
      d.wah = m.dhi(ca.w_off); d.wal = m.dlo(ca.w_off); d.ba = m.dptr(ca.b_off);
      d.wbh = m.dhi(cb.w_off); d.wbl = m.dlo(cb.w_off); d.bb = m.dptr(cb.b_off);
      d.w3h = m.dhi(c3.w_off); d.w3l = m.dlo(c3.w_off); d.b3 = m.dptr(c3.b_off);
      d.w1 = m.dptr(c1.w_off); d.wa = m.dptr(ca.w_off); d.wb = m.dptr(cb.w_off); d.w3 = m.dptr(c3.w_off);
      const double bytes = 4.0 * b.B * px * (x.C + Cout) +
                           4.0 * ((double)c1.N * c1.K + (double)ca.N * ca.K + (double)cb.N * cb.K + (double)c3.N * c3.K);
      const Buf xb = x.buf, ob = outbuf;
      b.step(p + ".fused", [d, xb, ob](const Ctx& c) mutable {
        d.x = c.resolve(xb);
        d.out = c.resolve(ob);
        return launch_res2_block(d, c.stream);
      }, res2_block_kernel_name(d), bytes);
    }
    return true;
  }

  // |x| <= bx; the block's output is Hardtanh-bounded (kHt)
  T4 block(const std::string& p, const T4& x, int stride, int width, int planes, bool use_aff, Buf outbuf, double bx) {
    const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
    const int Cout = planes * expansion;
    need(bx);                                   // conv1 and the shortcut read x; T1 / CAT are Hardtanh outputs
    T4 fo;
    if (fusable(p, x, stride, width, Cout, use_aff) && fused_block(p, x, stride, width, Cout, outbuf, fo)) return fo;
    const ChanMap sl = ChanMap::slices(width, scale);
    const int wp = sl.n_phys / scale;
    const int ldt = sl.n_phys;
    const size_t t1_plane = (size_t)b.B * Ho * Wo * wp;   // floats per T1 slice plane
    const ChanMap xin = ChanMap::dense(x.C);
    const double px = (double)Ho * Wo;

    // conv1 (1x1, stride) + bn1 + Hardtanh -> T1 (scale slices)
    const Packed& c1 = m.pack(p + ".conv1", sl, {Part{p + ".conv1.weight", "", p + ".bn1", xin, 0, 0}}, x.C);
    b.macs_per_utt += px * x.C * (double)width * scale;
    if (b.plan) {
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src_of(nullptr, x, x.C, 1, stride, 0);
      d.ldo = wp; d.osplit = wp; d.oplane = (long long)t1_plane;
      d.act = ACT_HTANH;
      Builder::ConvIO io; io.s0 = x.buf; io.out = T1;
      b.conv(p + ".conv1", d, c1, io);
    }
    const T4 cat{CAT, ldt, Ho, Wo, ldt};
    for (int i = 0; i < scale; ++i) {
      T4 in{T1.at((size_t)i * t1_plane), wp, Ho, Wo, wp};
      Buf addend;
      int add_ld = 0;
      if (i > 0) {
        T4 prev{CAT.at((size_t)(i - 1) * wp), ldt, Ho, Wo, wp};
        if (use_aff) {
          T4 f{FB, wp, Ho, Wo, wp};
          aff(p + ".fuse_models." + std::to_string(i - 1), prev, in, width, f, kHt, kHt);
          in = f;
        } else {
          addend = prev.buf;
          add_ld = ldt;
        }
      }
      const ChanMap one = ChanMap::dense(width);
      const std::string ci = std::to_string(i);
      const Packed& cv = m.pack(p + ".convs." + ci, one,
                                {Part{p + ".convs." + ci + ".weight", "", p + ".bns." + ci, one, 0, 0}}, 9 * wp);
      b.macs_per_utt += px * 9.0 * width * width;
      if (b.plan) {
        ConvDesc d;
        d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
        d.s0 = src_of(nullptr, in, wp, 3, 1, 1);
        if (addend) d.s0.ld2 = add_ld;
        d.ldo = ldt; d.act = ACT_HTANH;
        Builder::ConvIO io; io.s0 = in.buf; io.s0b = addend; io.out = CAT.at((size_t)i * wp);
        b.conv(p + ".convs." + ci, d, cv, io);
      }
    }
    // conv3 + bn3 (+ shortcut conv + bn, K-concatenated) + residual + Hardtanh
    const bool has_sc = m.has(p + ".shortcut.0.weight");
    const ChanMap om = ChanMap::dense(Cout);
    std::vector<Part> parts{Part{p + ".conv3.weight", "", p + ".bn3", sl, 0, 0}};
    int K = ldt;
    if (has_sc) {
      parts.push_back(Part{p + ".shortcut.0.weight", "", p + ".shortcut.1", xin, 0, ldt});
      K += x.C;
    } else if (stride != 1 || x.C != Cout) {
      throw SpkError(SPK_E_WEIGHTS, p + ": missing shortcut for a shape-changing block");
    }
    const Packed& c3 = m.pack(p + ".conv3", om, parts, K);
    b.macs_per_utt += px * (double)width * scale * Cout + (has_sc ? px * x.C * (double)Cout : 0.0);
    T4 out{outbuf, om.n_phys, Ho, Wo, om.n_phys};
    if (b.plan) {
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src_of(nullptr, cat, ldt, 1, 1, 0);
      Builder::ConvIO io; io.s0 = CAT; io.out = outbuf;
      if (has_sc) {
        d.s1 = src_of(nullptr, x, x.C, 1, stride, 0);
        io.s1 = x.buf;
      } else {
        d.ldr = x.ld;
        io.res = x.buf;
      }
      d.ldo = out.ld; d.act = ACT_HTANH;
      b.conv(p + ".conv3", d, c3, io);
    }
    return out;
  }

  void run(int T) {
    const int B = b.B;
    const int F = m.cfg.feat_dim;
    const int mc = m.cfg.m_channels;
    if (mc % 4) throw SpkError(SPK_E_UNSUPPORTED, "m_channels must be a multiple of 4");
    // ---- stem conv 3x3 1->mc + bn1 + relu (ERes2NetV2.py:238)
    const Packed& stem = m.pack("conv1", ChanMap::dense(mc), {Part{"conv1.weight", "", "bn1", ChanMap::dense(1, 1), 0, 0}}, 9);
    T4 x{b.alloc((size_t)B * F * T * mc), mc, F, T, mc};
    double bx = INFINITY;   // ReLU(BN(conv(input))): no static bound
    b.macs_per_utt += (double)F * T * mc * 9;
    if (b.plan) {
      const float* w = m.dptr(stem.w_off);
      const float* bias = m.dptr(stem.b_off);
      const int kp = stem.Kp;
      const Buf xo = x.buf;
      const int ld = x.ld;
      const bool flag = !b.exact;
      b.step("stem", [=](const Ctx& c) {
        return launch_stem_conv3x3(c.in, B, T, F, w, bias, mc, ACT_RELU, kp, c.resolve(xo), ld, c.stream, nullptr, flag ? c.flag : nullptr);
      });
    }
    // ---- scratch for the block internals, sized by the largest layer
    size_t t1_max = 0, mid_max = 0, fb_max = 0;
    {
      int H = F, W = T;
      for (int li = 0; li < 4; ++li) {
        const int stride = li ? 2 : 1;
        H = (H - 1) / stride + 1; W = (W - 1) / stride + 1;
        const int width = (int)std::floor((mc << li) * (base_width / 64.0));
        const size_t px = (size_t)B * H * W;
        t1_max = std::max(t1_max, px * ChanMap::slices(width, scale).n_phys);
        mid_max = std::max(mid_max, px * ChanMap::dense(width / 4).n_phys);
        fb_max = std::max(fb_max, px * ChanMap::dense(width).n_phys);
        const int C = (mc << li) * expansion;   // model-level AFF at this resolution
        mid_max = std::max(mid_max, px * aff_mid(C).n_phys);
      }
    }
    T1 = b.alloc(t1_max);
    CAT = b.alloc(t1_max);
    MID = b.alloc(mid_max);
    FB = b.alloc(fb_max);

    T4 outs[4];
    for (int li = 0; li < 4; ++li) {
      const std::string layer = "layer" + std::to_string(li + 1);
      const int planes = mc << li;
      const int width = (int)std::floor(planes * (base_width / 64.0));
      const int stride = li ? 2 : 1;
      const int nb = count_blocks(m, layer);
      if (nb == 0) throw SpkError(SPK_E_WEIGHTS, "no blocks in " + layer);
      const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
      const size_t osz = (size_t)B * Ho * Wo * ChanMap::dense(planes * expansion).n_phys;
      Buf pp[2] = {b.alloc(osz), b.alloc(osz)};
      for (int bi = 0; bi < nb; ++bi) {
        x = block(layer + "." + std::to_string(bi), x, bi ? 1 : stride, width, planes, li >= 2, pp[bi & 1], bx);
        bx = kHt;
        close_segment();   // the stem's segment ends with layer1.0
      }
      outs[li] = x;
    }

    T4 fused;
    double bnd = 0.0;   // bound of the last downsample / fuse output
    auto downsample = [&](const std::string& key, const T4& in, double bin) {
      const int Cout = (int)m.dim(key, 0);
      const ChanMap om = ChanMap::dense(Cout);
      const Packed& p = m.pack(key, om, {Part{key, "", "", ChanMap::dense(in.C), 0, 0}}, 9 * in.C);
      const int Ho = (in.H - 1) / 2 + 1, Wo = (in.W - 1) / 2 + 1;
      T4 out{b.alloc((size_t)B * Ho * Wo * om.n_phys), om.n_phys, Ho, Wo, om.n_phys};
      need(bin);
      bnd = p.l1max * bin;   // no bias
      b.macs_per_utt += (double)Ho * Wo * Cout * in.C * 9.0;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = Ho; d.Wo = Wo;
        d.s0 = src_of(nullptr, in, in.C, 3, 2, 1);
        d.ldo = out.ld;
        Builder::ConvIO io; io.s0 = in.buf; io.out = out.buf;
        b.conv(key, d, p, io, /*use_bias=*/false);
      }
      return out;
    };
    auto fuse = [&](const std::string& key, const T4& a, const T4& y, double by) {
      T4 out{b.alloc((size_t)B * a.H * a.W * a.C), a.C, a.H, a.W, a.C};
      bnd = aff(key, a, y, a.C, out, kHt, by);
      return out;
    };
    if (v2) {
      const T4 ds = downsample("layer3_ds.weight", outs[2], kHt);
      fused = fuse("fuse34", outs[3], ds, bnd);
    } else {
      const T4 d1 = downsample("layer1_downsample.weight", outs[0], kHt);
      const T4 f12 = fuse("fuse_mode12", outs[1], d1, bnd);
      const T4 d2 = downsample("layer2_downsample.weight", f12, bnd);
      const T4 f123 = fuse("fuse_mode123", outs[2], d2, bnd);
      const T4 d3 = downsample("layer3_downsample.weight", f123, bnd);
      fused = fuse("fuse_mode1234", outs[3], d3, bnd);
    }
    const double bfused = bnd;   // pooled statistics (mean, std, attention-weighted too) stay below it

    // ---- TSTP (pooling_layers.py:47-55) -> stats [B, 2*H*C] in (h, c) order; TAP / TSDP
    //      (:10-35, pooling_func) keep only the mean / the std part; ASTP (:58-104) pools
    //      with attention weights into the same (h, c) order
    const int pool = m.cfg.pooling;
    if (pool < SPK_POOL_TSTP || pool > SPK_POOL_ASTP) throw SpkError(SPK_E_UNSUPPORTED, "pooling must be TSTP, TAP, TSDP or ASTP");
    const int parts = pool == SPK_POOL_TAP ? 1 : pool == SPK_POOL_TSDP ? 2 : 3;
    const int nst = parts == 3 ? 2 : 1;
    const int H4 = fused.H, C4 = fused.C;
    const int S = nst * H4 * C4;
    const Buf stats = b.alloc((size_t)B * S);
    need(bfused);   // ASTP linear1 (its linear2 reads tanh outputs) or seg_1 reads the pooled stats
    if (pool == SPK_POOL_ASTP) {
      astp(fused, stats);
    } else if (b.plan) {
      const T4 f = fused;
      b.step("pool", [=](const Ctx& c) {
        return launch_tstp(c.resolve(f.buf), B, f.H, f.W, f.C, f.ld, 1e-8f, 1, c.resolve(stats), c.stream, parts);
      });
    }
    // reference flattens (C, F): index c*H + h  -> our h*C + c
    ChanMap perm;
    perm.phys.resize(S);
    perm.n_phys = S;
    for (int part = 0; part < nst; ++part)
      for (int c = 0; c < C4; ++c)
        for (int h = 0; h < H4; ++h) perm.phys[part * H4 * C4 + c * H4 + h] = part * H4 * C4 + h * C4 + c;
    const int E = (int)m.dim("seg_1.weight", 0);
    if (E % 4) throw SpkError(SPK_E_UNSUPPORTED, "embedding_size must be a multiple of 4");
    if (m.dim("seg_1.weight", 1) != S) throw SpkError(SPK_E_WEIGHTS, "seg_1 in_features != pooled stats size");
    const bool two = m.cfg.two_emb_layer != 0;
    const ChanMap em = ChanMap::dense(E, 1);
    const Packed& seg1 = m.pack("seg_1", em, {Part{"seg_1.weight", "seg_1.bias", "", perm, 0, 0}}, S);
    b.macs_per_utt += (double)S * E;
    const T4 st{stats, S, 1, 1, S};
    Buf e1 = two ? b.alloc((size_t)B * E) : Buf{Buf::OUT, 0, nullptr};
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = 1;
      d.s0 = src_of(nullptr, st, S, 1, 1, 0);
      d.ldo = E;
      if (two) {
        const Packed& pa = m.pack_post_affine("seg_bn_1", "seg_bn_1", em);
        d.act = ACT_RELU;
        d.post_scale = m.dptr(pa.ps_off);
        d.post_shift = m.dptr(pa.pt_off);
      }
      Builder::ConvIO io; io.s0 = stats; io.out = e1;
      b.conv("seg_1", d, seg1, io);
    } else if (two) {
      m.pack_post_affine("seg_bn_1", "seg_bn_1", em);
    }
    if (two) {
      const Packed& seg2 = m.pack("seg_2", em, {Part{"seg_2.weight", "seg_2.bias", "", ChanMap::dense(E, 1), 0, 0}}, E);
      // seg_2 reads seg_bn_1(ReLU(seg_1(stats)))
      need(Builder::bound(m.pack_post_affine("seg_bn_1", "seg_bn_1", em), Builder::bound(seg1, bfused)));
      b.macs_per_utt += (double)E * E;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = 1;
        const T4 t{e1, E, 1, 1, E};
        d.s0 = src_of(nullptr, t, E, 1, 1, 0);
        d.ldo = E;
        Builder::ConvIO io; io.s0 = e1; io.out = Buf{Buf::OUT, 0, nullptr};
        b.conv("seg_2", d, seg2, io);
      }
    }
    close_segment();
  }
};

}  // namespace

void build_eres2net(Builder& b, int T, bool v2) {
  ERes2Builder eb(b, v2);
  eb.run(T);
}

}  // namespace spk
