// CAM++ launch plan.
//
// Reference: speakerlab/models/campplus/DTDNN.py (FCM :13-48, CAMPPlus :50-115) and
// layers.py (TDNNLayer :40-67, CAMLayer :70-110, CAMDenseTDNNLayer :113-149,
// CAMDenseTDNNBlock :152-180, TransitLayer :183-196, DenseLayer :199-215,
// BasicResBlock :218-253, statistics_pooling :26-37).
//
// Mapping onto the fused GEMM (channels-last everywhere):
//   * FCM: 3x3 convs with frequency-only stride; BasicResBlock = 2 GEMMs, the shortcut conv
//     K-concatenated into the second one (or the identity residual in its epilogue);
//   * the FCM -> TDNN reshape (C, F) -> C*F needs no data movement: xvector.tdnn is run as
//     a 2-D conv whose kernel spans the whole frequency axis (kh = F/8, kw = 5, stride (1,2))
//     over the [B, F/8, T, 32] FCM output, with the weight re-indexed on the host;
//   * a dense layer's BN-ReLU pre-activation is applied in the operand loader (pre_scale),
//     its second BN-ReLU is folded into linear1's epilogue;
//   * CAMLayer's context branch (mean + 100-frame segment means -> linear1 -> ReLU ->
//     linear2 -> sigmoid) is one kernel per utterance (cam_gate, tdnn_ops.hip): the context
//     is constant inside a segment, so both 1x1 layers run once per segment -- the
//     reference's per-frame computation without the repetition; the gate multiplies
//     linear_local's output in its epilogue;
//   * torch.cat growth is an in-place write into the block's preallocated channel buffer;
//     transit layers write straight into the next block's buffer; out_nonlinear is folded
//     into the last transit's epilogue; dense + BN(affine=False) is one small GEMM.
#include "misc.h"
#include "runtime.h"
#include "tdnn_ops.h"

namespace spk {

namespace {

struct A4 {
  Buf buf;
  int ld = 0, H = 0, W = 0, C = 0;
};

ConvSrc src2d(const A4& t, int cin, int kh, int kw, int sh, int sw, int ph, int pw, int dw = 1) {
  ConvSrc s;
  s.ld = t.ld; s.H = t.H; s.W = t.W; s.cin = cin;
  s.kh = kh; s.kw = kw; s.sh = sh; s.sw = sw; s.ph = ph; s.pw = pw; s.dw = dw;
  return s;
}

}  // namespace

void build_campplus(Builder& b, int T) {
  // reduced-precision mode: only the dense blocks' GEMMs (the bulk of the FLOPs) run as single
  // products; the FCM head, the TDNN layer, transits and the embedding layer stay fp16x3
  b.x1_scope = false;
  Model& m = b.m;
  const int B = b.B;
  const int F = m.cfg.feat_dim;
  const int mc = (int)m.dim("head.conv1.weight", 0);
  if (F % 8 || mc % 4) throw SpkError(SPK_E_UNSUPPORTED, "CAM++: feat_dim % 8 and m_channels % 4 required");
  // ---- FCM stem
  const Packed& stem = m.pack("head.conv1", ChanMap::dense(mc),
                              {Part{"head.conv1.weight", "", "head.bn1", ChanMap::dense(1, 1), 0, 0}}, 9);
  A4 x{b.alloc((size_t)B * F * T * mc), mc, F, T, mc};
  b.macs_per_utt += (double)F * T * mc * 9;
  if (b.plan) {
    const float* w = m.dptr(stem.w_off);
    const float* bias = m.dptr(stem.b_off);
    const int kp = stem.Kp;
    const Buf xo = x.buf;
    const bool rg = b.ragged;
    const bool flag = !b.exact;
    b.writes({{xo, Builder::NOTED}}).step("head.stem", [=](const Ctx& c) {
      return launch_stem_conv3x3(c.in, B, T, F, w, bias, mc, ACT_RELU, kp, c.resolve(xo), mc, c.stream,
                                 rg ? c.lens : nullptr, flag ? c.flag : nullptr);
    });
  }
  const ChanMap cm = ChanMap::dense(mc);
  // ragged batches: outputs past an utterance's valid frames are written as zero, so every
  // conv sees the zero padding of that utterance alone; BN-ReLU'd inputs are masked on load
  const Buf LENS = b.ragged ? Buf{Buf::LEN, 0, nullptr} : Buf{};
  // FCM BasicResBlocks
  for (int li = 1; li <= 2; ++li) {
    for (int bi = 0; bi < 2; ++bi) {
      const std::string p = "head.layer" + std::to_string(li) + "." + std::to_string(bi);
      if (!m.has(p + ".conv1.weight")) throw SpkError(SPK_E_WEIGHTS, p + " missing");
      const int stride = bi == 0 ? 2 : 1;
      const int Ho = (x.H + 2 - 3) / stride + 1;
      A4 y1{b.alloc((size_t)B * Ho * T * mc), mc, Ho, T, mc};
      A4 out{b.alloc((size_t)B * Ho * T * mc), mc, Ho, T, mc};
      const Packed& c1 = m.pack(p + ".conv1", cm, {Part{p + ".conv1.weight", "", p + ".bn1", cm, 0, 0}}, 9 * mc);
      const bool sc = m.has(p + ".shortcut.0.weight");
      // the projection shortcut (1x1, frequency stride 2, + BN) is its own small GEMM whose
      // output conv2 adds as a residual: conv2 is then a plain stride-1 3x3 conv that the
      // halo kernel takes, instead of an implicit GEMM with a K-concatenated operand on
      // 32-wide tiles
      const Packed& c2 = m.pack(p + ".conv2", cm, {Part{p + ".conv2.weight", "", p + ".bn2", cm, 0, 0}}, 9 * mc);
      const Packed* csc = sc ? &m.pack(p + ".shortcut", cm, {Part{p + ".shortcut.0.weight", "", p + ".shortcut.1", cm, 0, 0}}, mc)
                             : nullptr;
      A4 scb{sc ? b.alloc((size_t)B * Ho * T * mc) : Buf{}, mc, Ho, T, mc};
      const double macs1 = (double)Ho * T * mc * mc * 9;
      const double macs_sc = sc ? (double)Ho * T * mc * mc : 0.0;
      b.macs_per_utt += macs1;
      if (!b.plan) b.macs_per_utt += macs1 + macs_sc;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = Ho; d.Wo = T;
        d.s0 = src2d(x, mc, 3, 3, stride, 1, 1, 1);
        d.ldo = mc; d.act = ACT_RELU;
        Builder::ConvIO io; io.s0 = x.buf; io.out = y1.buf; io.rowlen = LENS;
        b.conv(p + ".conv1", d, c1, io);
        if (sc) {
          b.macs_per_utt += macs_sc;
          ConvDesc f;
          f.nimg = B; f.Ho = Ho; f.Wo = T;
          f.s0 = src2d(x, mc, 1, 1, stride, 1, 0, 0);
          f.ldo = mc;
          Builder::ConvIO ios; ios.s0 = x.buf; ios.out = scb.buf;
          b.conv(p + ".shortcut", f, *csc, ios);
        }
        b.macs_per_utt += macs1;
        ConvDesc e;
        e.nimg = B; e.Ho = Ho; e.Wo = T;
        e.s0 = src2d(y1, mc, 3, 3, 1, 1, 1, 1);
        Builder::ConvIO io2; io2.s0 = y1.buf; io2.out = out.buf; io2.rowlen = LENS;
        const A4& resid = sc ? scb : x;
        e.ldr = resid.ld;
        io2.res = resid.buf;
        e.ldo = mc; e.act = ACT_RELU;
        b.conv(p + ".conv2", e, c2, io2);
      }
      x = out;
    }
  }
  // head.conv2 3x3 stride (2,1) + bn2 + relu
  {
    const int Ho = (x.H + 2 - 3) / 2 + 1;
    A4 z{b.alloc((size_t)B * Ho * T * mc), mc, Ho, T, mc};
    const Packed& c = m.pack("head.conv2", cm, {Part{"head.conv2.weight", "", "head.bn2", cm, 0, 0}}, 9 * mc);
    b.macs_per_utt += (double)Ho * T * mc * mc * 9;
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = Ho; d.Wo = T;
      d.s0 = src2d(x, mc, 3, 3, 2, 1, 1, 1);
      d.ldo = mc; d.act = ACT_RELU;
      Builder::ConvIO io; io.s0 = x.buf; io.out = z.buf; io.rowlen = LENS;
      b.conv("head.conv2", d, c, io);
    }
    x = z;
  }
  const int Fh = x.H;   // F / 8
  // ---- xvector.tdnn: Conv1d(mc*Fh -> C0, k5, s2, p2) as a full-height 2-D conv
  const std::string tk = "xvector.tdnn.linear.weight";
  const int C0 = (int)m.dim(tk, 0);
  const int K5 = (int)m.dim(tk, 2);
  if (m.dim(tk, 1) != (int64_t)mc * Fh) throw SpkError(SPK_E_WEIGHTS, "CAM++: tdnn input != FCM output channels");
  const std::string tk2 = tk + "#2d";
  if (!m.uploaded && !m.W.count(tk2)) {
    const Model::HostT& w = m.get(tk);
    Model::HostT t;
    t.shape = {C0, mc, Fh, K5};
    t.data.resize((size_t)C0 * mc * Fh * K5);
    for (int co = 0; co < C0; ++co)
      for (int c = 0; c < mc; ++c)
        for (int f = 0; f < Fh; ++f)
          for (int k = 0; k < K5; ++k)
            t.data[(((size_t)co * mc + c) * Fh + f) * K5 + k] = w.data[((size_t)co * mc * Fh + c * Fh + f) * K5 + k];
    m.W[tk2] = t;
    m.shapes[tk2] = t.shape;
  }
  const int T2 = (T + 2 * (K5 / 2) - K5) / 2 + 1;
  // valid frames after the stride-2 TDNN, per utterance (ragged batches)
  Buf LEN2;
  if (b.ragged) {
    LEN2 = b.alloc((size_t)B);
    if (b.plan) {
      const int pad = K5 / 2, k5 = K5;
      b.writes({{LEN2, Builder::AUX}}).step("xvector.tdnn.lengths", [=](const Ctx& c) {
        return launch_derive_len(c.lens, c.resolve_i(LEN2), B, pad, k5, 2, c.stream);
      });
    }
  }
  const double T2d = T2;
  const int nseg = (T2 + 99) / 100;
  // dense blocks: sizes
  struct Blk { int n, d, c_in, c_fin; Buf buf; };
  std::vector<Blk> blks;
  {
    int c = C0;
    for (int i = 1;; ++i) {
      const std::string p = "xvector.block" + std::to_string(i);
      if (!m.has(p + ".tdnnd1.linear1.weight")) break;
      int n = 0;
      while (m.has(p + ".tdnnd" + std::to_string(n + 1) + ".linear1.weight")) ++n;
      const int growth = (int)m.dim(p + ".tdnnd1.cam_layer.linear_local.weight", 0);
      // dilation from the registry (12/24/16 layers with dilations 1/2/2, DTDNN.py:77-78)
      const int dil = i == 1 ? 1 : 2;
      Blk bk{n, dil, c, c + n * growth, Buf{}};
      bk.buf = b.alloc((size_t)B * T2 * bk.c_fin);
      blks.push_back(bk);
      c = (int)m.dim("xvector.transit" + std::to_string(i) + ".linear.weight", 0);
    }
    if (blks.empty()) throw SpkError(SPK_E_WEIGHTS, "CAM++: no dense blocks");
  }
  {
    const ChanMap om = ChanMap::dense(C0);
    const Packed& p = m.pack("xvector.tdnn", om, {Part{tk2, "", "xvector.tdnn.nonlinear.batchnorm", cm, 0, 0}},
                             Fh * K5 * mc);
    b.macs_per_utt += T2d * C0 * mc * Fh * K5;
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = T2;
      d.s0 = src2d(x, mc, Fh, K5, 1, 2, 0, K5 / 2);
      d.ldo = blks[0].c_fin; d.act = ACT_RELU;
      Builder::ConvIO io; io.s0 = x.buf; io.out = blks[0].buf; io.rowlen = LEN2;
      b.conv("xvector.tdnn", d, p, io);
    }
  }
  const int bnc = (int)m.dim("xvector.block1.tdnnd1.linear1.weight", 0);   // bn_channels (128)
  const int red = (int)m.dim("xvector.block1.tdnnd1.cam_layer.linear1.weight", 0);
  const Buf Hh = b.alloc((size_t)B * T2 * bnc);
  const Buf GATE = b.alloc((size_t)B * nseg * 64);
  const Buf SEGSUM = b.alloc((size_t)B * nseg * bnc);
  Buf xo_final;
  int c_final = 0;
  for (size_t bi = 0; bi < blks.size(); ++bi) {
    const Blk& bk = blks[bi];
    b.x1_scope = true;
    const std::string p = "xvector.block" + std::to_string(bi + 1);
    for (int l = 0; l < bk.n; ++l) {
      const std::string q = p + ".tdnnd" + std::to_string(l + 1);
      const int cin = bk.c_in + l * (int)m.dim(q + ".cam_layer.linear_local.weight", 0);
      const int growth = (int)m.dim(q + ".cam_layer.linear_local.weight", 0);
      if (cin % 4 || growth % 4 || bnc % 4 || red % 4 || growth > 64)
        throw SpkError(SPK_E_UNSUPPORTED, q + ": channel counts must be multiples of 4");
      const Packed* pre = &m.pack_post_affine(q + ".pre", q + ".nonlinear1.batchnorm", ChanMap::dense(cin));
      const Packed& l1 = m.pack(q + ".linear1", ChanMap::dense(bnc),
                                {Part{q + ".linear1.weight", "", q + ".nonlinear2.batchnorm", ChanMap::dense(cin), 0, 0}}, cin,
                                pre->pre_bits);
      const std::string c = q + ".cam_layer";
      const Packed& cl1 = m.pack(c + ".linear1", ChanMap::dense(red),
                                 {Part{c + ".linear1.weight", c + ".linear1.bias", "", ChanMap::dense(bnc), 0, 0}}, bnc);
      const Packed& cl2 = m.pack(c + ".linear2", ChanMap::dense(growth),
                                 {Part{c + ".linear2.weight", c + ".linear2.bias", "", ChanMap::dense(red), 0, 0}}, red);
      const int ks = (int)m.dim(c + ".linear_local.weight", 2);
      const Packed& loc = m.pack(c + ".linear_local", ChanMap::dense(growth),
                                 {Part{c + ".linear_local.weight", "", "", ChanMap::dense(bnc), 0, 0}}, ks * bnc);
      // reference-algorithmic MACs (the reference runs the CAM linears on every frame)
      const double m_l1 = T2d * bnc * cin, m_c1 = T2d * red * bnc, m_c2 = T2d * growth * red;
      const double m_loc = T2d * growth * bnc * ks;
      if (!b.plan) {
        b.macs_per_utt += m_l1 + m_c1 + m_c2 + m_loc;
        continue;
      }
      const A4 db{bk.buf, bk.c_fin, 1, T2, bk.c_fin};
      {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T2;
        d.s0 = src2d(db, cin, 1, 1, 1, 1, 0, 0);
        d.ldo = bnc; d.act = ACT_RELU;
        Builder::ConvIO io; io.s0 = bk.buf; io.out = Hh; io.vlen = LEN2; io.rowlen = LEN2; io.pre = pre;
        b.macs_per_utt += m_l1;
        b.conv(q + ".linear1", d, l1, io);
      }
      {
        // context -> linear1 -> ReLU -> linear2 -> sigmoid, once per (utterance, segment)
        const float* w1 = m.dptr(cl1.w_off);
        const float* b1 = cl1.has_bias ? m.dptr(cl1.b_off) : nullptr;
        const float* w2 = m.dptr(cl2.w_off);
        const float* b2 = cl2.has_bias ? m.dptr(cl2.b_off) : nullptr;
        const int k1p = cl1.Kp, k2p = cl2.Kp;
        b.macs_per_utt += m_c1 + m_c2;
        b.writes({{GATE, Builder::AUX}, {SEGSUM, Builder::AUX}}).step(c + ".gate", [=](const Ctx& cx) {
          return launch_cam_gate(cx.resolve(Hh), B, T2, bnc, bnc, 100, nseg, w1, k1p, b1, red, w2, k2p, b2, growth,
                                 cx.resolve(GATE), growth, cx.resolve(SEGSUM), cx.stream, cx.resolve_i(LEN2));
        }, "cam_gate_kernel", 4.0 * B * T2 * bnc);
      }
      {
        const A4 hh{Hh, bnc, 1, T2, bnc};
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T2;
        d.s0 = src2d(hh, bnc, 1, ks, 1, 1, 0, (ks - 1) / 2 * bk.d, bk.d);
        d.ldo = bk.c_fin;
        d.gate_ld = growth; d.gate_seg = 100; d.gate_nseg = nseg;
        Builder::ConvIO io; io.s0 = Hh; io.out = bk.buf.at((size_t)cin); io.gate = GATE; io.rowlen = LEN2;
        b.macs_per_utt += m_loc;
        b.conv(c + ".linear_local", d, loc, io);
      }
    }
    b.x1_scope = false;
    // transit: BN-ReLU (pre) -> 1x1 (no bias); the last one also folds out_nonlinear
    const std::string t = "xvector.transit" + std::to_string(bi + 1);
    const int cout = (int)m.dim(t + ".linear.weight", 0);
    const bool last = bi + 1 == blks.size();
    const Packed* pre = &m.pack_post_affine(t + ".pre", t + ".nonlinear.batchnorm", ChanMap::dense(bk.c_fin));
    const Packed& tp = m.pack(t, ChanMap::dense(cout),
                              {Part{t + ".linear.weight", "", last ? "xvector.out_nonlinear.batchnorm" : "",
                                    ChanMap::dense(bk.c_fin), 0, 0}},
                              bk.c_fin, pre->pre_bits);
    b.macs_per_utt += T2d * cout * bk.c_fin;
    Buf dst;
    int ldd;
    if (last) {
      dst = b.alloc((size_t)B * T2 * cout);
      ldd = cout;
      xo_final = dst;
      c_final = cout;
    } else {
      if (blks[bi + 1].c_in != cout) throw SpkError(SPK_E_WEIGHTS, t + ": channel mismatch with next block");
      dst = blks[bi + 1].buf;
      ldd = blks[bi + 1].c_fin;
    }
    if (b.plan) {
      const A4 db{bk.buf, bk.c_fin, 1, T2, bk.c_fin};
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = T2;
      d.s0 = src2d(db, bk.c_fin, 1, 1, 1, 1, 0, 0);
      d.ldo = ldd;
      if (last) d.act = ACT_RELU;
      Builder::ConvIO io; io.s0 = bk.buf; io.out = dst; io.vlen = LEN2; io.rowlen = LEN2; io.pre = pre;
      b.conv(t, d, tp, io, /*use_bias=*/last);
    }
  }
  // ---- stats pool + dense (1x1, BN affine=False)
  const Buf ST = b.alloc((size_t)B * 2 * c_final);
  const int E = (int)m.dim("xvector.dense.linear.weight", 0);
  if (E % 4 || c_final % 4) throw SpkError(SPK_E_UNSUPPORTED, "CAM++: embedding_size must be a multiple of 4");
  const Packed& dp = m.pack("xvector.dense", ChanMap::dense(E, 1),
                            {Part{"xvector.dense.linear.weight", "", "xvector.dense.nonlinear.batchnorm",
                                  ChanMap::dense(2 * c_final), 0, 0}},
                            2 * c_final);
  b.macs_per_utt += (double)E * 2 * c_final;
  if (!b.plan) return;
  b.writes({{ST, Builder::BOUNDED}}).step("xvector.stats", [=](const Ctx& c) {
    return launch_stats_pool(c.resolve(xo_final), B, T2, c_final, c_final, c.resolve(ST), c.stream,
                             c.resolve_i(LEN2));
  });
  ConvDesc d;
  d.nimg = B; d.Ho = 1; d.Wo = 1;
  ConvSrc s; s.ld = 2 * c_final; s.cin = 2 * c_final;
  d.s0 = s;
  d.ldo = E;
  Builder::ConvIO io; io.s0 = ST; io.out = Buf{Buf::OUT, 0, nullptr};
  b.conv("xvector.dense", d, dp, io);
}

}  // namespace spk
