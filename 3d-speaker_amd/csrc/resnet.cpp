// ResNet / Res2Net launch plans (the ResNet family of speakerlab/models).
//
// Reference forwards:
//   ResNet   speakerlab/models/resnet/ResNet.py:15-35 (BasicBlock), :86-101 (model)
//   Res2Net  speakerlab/models/res2net/Res2Net.py:27-87 (BasicBlockRes2Net), :128-147 (model)
// Both: stem conv3x3 1->m + BN + ReLU, four stages (stride 1, 2, 2, 2), TSTP, seg_1
// [-> ReLU -> seg_bn_1 -> seg_2].
//
// Layout as csrc/eres2net.cpp (channels-last [B, F, T, C]):
//   * ResNet BasicBlock = two implicit-GEMM convs: conv1 3x3(stride) + bn1 + ReLU -> MID;
//     conv2 3x3 + bn2 with the projection shortcut (1x1 stride conv + BN) K-concatenated as
//     a second operand, or the identity added in the epilogue, then ReLU;
//   * Res2Net block (scale 2): conv1 1x1(stride) + bn1 + Hardtanh writes spx0 into Z1 and
//     spx1 straight into its concat position in Z2; the 3x3 conv writes sp next to it, so
//     torch.cat is free and conv3 reads one operand; the projection shortcut is its own GEMM
//     whose output the conv3 epilogue adds (identity blocks add the input).
#include <cmath>

#include "misc.h"
#include "runtime.h"

namespace spk {

namespace {

struct R4 {
  Buf buf;
  int ld = 0, H = 0, W = 0, C = 0;
};

ConvSrc src(const R4& t, int cin, int k, int stride, int pad) {
  ConvSrc s;
  s.ld = t.ld; s.H = t.H; s.W = t.W; s.cin = cin;
  s.kh = s.kw = k; s.sh = s.sw = stride; s.ph = s.pw = pad;
  return s;
}

int n_blocks(const Model& m, const std::string& layer) {
  int n = 0;
  while (m.has(layer + "." + std::to_string(n) + ".conv1.weight")) ++n;
  return n;
}

struct ResBuilder {
  Builder& b;
  Model& m;
  bool res2;
  Buf MID, Z1, Z2, SC;

  ResBuilder(Builder& bb, bool r2) : b(bb), m(bb.m), res2(r2) {}

  // ---- ResNet BasicBlock (ResNet.py:30-35)
  R4 basic(const std::string& p, const R4& x, int stride, int planes, Buf outbuf) {
    const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
    const ChanMap xin = ChanMap::dense(x.C), pm = ChanMap::dense(planes);
    const double px = (double)Ho * Wo;
    const Packed& c1 = m.pack(p + ".conv1", pm, {Part{p + ".conv1.weight", "", p + ".bn1", xin, 0, 0}}, 9 * x.C);
    b.macs_per_utt += px * 9.0 * x.C * planes;
    const R4 mid{MID, pm.n_phys, Ho, Wo, pm.n_phys};
    if (b.plan) {
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src(x, x.C, 3, stride, 1);
      d.ldo = mid.ld; d.act = ACT_RELU;
      Builder::ConvIO io; io.s0 = x.buf; io.out = MID;
      b.conv(p + ".conv1", d, c1, io);
    }
    const bool sc = m.has(p + ".shortcut.0.weight");
    if (!sc && (stride != 1 || x.C != planes))
      throw SpkError(SPK_E_WEIGHTS, p + ": missing shortcut for a shape-changing block");
    std::vector<Part> parts{Part{p + ".conv2.weight", "", p + ".bn2", pm, 0, 0}};
    int K = 9 * pm.n_phys;
    if (sc) {
      parts.push_back(Part{p + ".shortcut.0.weight", "", p + ".shortcut.1", xin, 0, K});
      K += x.C;
    }
    const Packed& c2 = m.pack(p + ".conv2", pm, parts, K);
    b.macs_per_utt += px * 9.0 * planes * planes + (sc ? px * x.C * (double)planes : 0.0);
    R4 out{outbuf, pm.n_phys, Ho, Wo, pm.n_phys};
    if (b.plan) {
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src(mid, pm.n_phys, 3, 1, 1);
      Builder::ConvIO io; io.s0 = MID; io.out = outbuf;
      if (sc) {
        d.s1 = src(x, x.C, 1, stride, 0);
        io.s1 = x.buf;
      } else {
        d.ldr = x.ld;
        io.res = x.buf;
      }
      d.ldo = out.ld; d.act = ACT_RELU;
      b.conv(p + ".conv2", d, c2, io);
    }
    return out;
  }

  // ---- BasicBlockRes2Net (Res2Net.py:59-87), scale 2: conv1 -> [spx0 | spx1];
  //   sp = Ht(bn(conv3x3(spx0))); out = Ht(bn3(conv3(cat(sp, spx1))) + shortcut).
  // conv1's split epilogue writes spx0 into Z1 and spx1 straight into the second half of
  // Z2's rows (two output planes, one plane stride apart); the 3x3 conv writes sp into the
  // first half of Z2, so conv3 reads the concat as ONE operand of 2 x wp channels.
  R4 res2block(const std::string& p, const R4& x, int stride, int planes, Buf outbuf) {
    const int scale = m.cfg.scale ? m.cfg.scale : 2, expansion = m.cfg.expansion ? m.cfg.expansion : 2;
    if (scale != 2) throw SpkError(SPK_E_UNSUPPORTED, "Res2Net: the executor implements scale 2 (the reference default)");
    const double bw = m.cfg.base_width ? m.cfg.base_width : 32;
    const int width = (int)std::floor(planes * (bw / 64.0)), Cout = planes * expansion;
    const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
    const ChanMap xin = ChanMap::dense(x.C), sl = ChanMap::slices(width, 2), one = ChanMap::dense(width);
    const int wp = sl.n_phys / 2, ldz = 2 * wp;
    const double px = (double)Ho * Wo;
    const Packed& c1 = m.pack(p + ".conv1", sl, {Part{p + ".conv1.weight", "", p + ".bn1", xin, 0, 0}}, x.C);
    b.macs_per_utt += px * x.C * (double)width * 2;
    if (b.plan) {
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src(x, x.C, 1, stride, 0);
      d.ldo = ldz; d.osplit = wp;
      d.oplane = (long long)((Z2.off - Z1.off) / sizeof(float)) + wp;   // plane 1 -> Z2[:, wp:]
      d.act = ACT_HTANH;
      Builder::ConvIO io; io.s0 = x.buf; io.out = Z1;
      b.conv(p + ".conv1", d, c1, io);
    }
    const Packed& cv = m.pack(p + ".convs.0", one, {Part{p + ".convs.0.weight", "", p + ".bns.0", one, 0, 0}}, 9 * wp);
    b.macs_per_utt += px * 9.0 * width * width;
    if (b.plan) {
      const R4 in{Z1, ldz, Ho, Wo, wp};
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src(in, wp, 3, 1, 1);
      d.ldo = ldz; d.act = ACT_HTANH;
      Builder::ConvIO io; io.s0 = Z1; io.out = Z2;
      b.conv(p + ".convs.0", d, cv, io);
    }
    // shortcut: projection GEMM into SC (added by the conv3 epilogue) or the identity
    const bool sc = m.has(p + ".shortcut.0.weight");
    if (!sc && (stride != 1 || x.C != Cout))
      throw SpkError(SPK_E_WEIGHTS, p + ": missing shortcut for a shape-changing block");
    const ChanMap om = ChanMap::dense(Cout);
    if (sc) {
      const Packed& s = m.pack(p + ".shortcut", om, {Part{p + ".shortcut.0.weight", "", p + ".shortcut.1", xin, 0, 0}},
                               x.C);
      b.macs_per_utt += px * x.C * (double)Cout;
      if (b.plan) {
        ConvDesc d;
        d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
        d.s0 = src(x, x.C, 1, stride, 0);
        d.ldo = om.n_phys;
        Builder::ConvIO io; io.s0 = x.buf; io.out = SC;
        b.conv(p + ".shortcut", d, s, io);
      }
    }
    const Packed& c3 = m.pack(p + ".conv3", om, {Part{p + ".conv3.weight", "", p + ".bn3", sl, 0, 0}}, ldz);
    b.macs_per_utt += px * (double)width * 2 * Cout;
    R4 out{outbuf, om.n_phys, Ho, Wo, om.n_phys};
    if (b.plan) {
      const R4 cat{Z2, ldz, Ho, Wo, ldz};
      ConvDesc d;
      d.nimg = b.B; d.Ho = Ho; d.Wo = Wo;
      d.s0 = src(cat, ldz, 1, 1, 0);
      Builder::ConvIO io; io.s0 = Z2; io.out = outbuf;
      if (sc) {
        d.ldr = om.n_phys;
        io.res = SC;
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
    const int B = b.B, F = m.cfg.feat_dim, mc = m.cfg.m_channels;
    if (mc % 4 || F % 8) throw SpkError(SPK_E_UNSUPPORTED, "m_channels % 4 and feat_dim % 8 required");
    const int expansion = res2 ? (m.cfg.expansion ? m.cfg.expansion : 2) : 1;
    // ---- stem conv3x3 1 -> m + bn1 + ReLU (ResNet.py:89, Res2Net.py:131)
    const Packed& stem = m.pack("conv1", ChanMap::dense(mc), {Part{"conv1.weight", "", "bn1", ChanMap::dense(1, 1), 0, 0}}, 9);
    R4 x{b.alloc((size_t)B * F * T * mc), mc, F, T, mc};
    b.macs_per_utt += (double)F * T * mc * 9;
    if (b.plan) {
      const float* w = m.dptr(stem.w_off);
      const float* bias = m.dptr(stem.b_off);
      const int kp = stem.Kp;
      const Buf xo = x.buf;
      const bool flag = !b.exact;
      b.step("stem", [=](const Ctx& c) {
        return launch_stem_conv3x3(c.in, B, T, F, w, bias, mc, ACT_RELU, kp, c.resolve(xo), mc, c.stream, nullptr, flag ? c.flag : nullptr);
      });
    }
    // ---- block scratch sized by the largest stage
    size_t mid = 0, z = 0, scb = 0;
    {
      int H = F, W = T;
      for (int li = 0; li < 4; ++li) {
        if (li) { H = (H - 1) / 2 + 1; W = (W - 1) / 2 + 1; }
        const size_t px = (size_t)B * H * W;
        const int planes = mc << li;
        mid = std::max(mid, px * ChanMap::dense(planes).n_phys);
        if (res2) {
          const int width = (int)std::floor(planes * ((m.cfg.base_width ? m.cfg.base_width : 32) / 64.0));
          z = std::max(z, px * ChanMap::slices(width, 2).n_phys);
          scb = std::max(scb, px * ChanMap::dense(planes * expansion).n_phys);
        }
      }
    }
    if (res2) {
      Z1 = b.alloc(z);
      Z2 = b.alloc(z);
      SC = b.alloc(scb);
    } else {
      MID = b.alloc(mid);
    }
    for (int li = 0; li < 4; ++li) {
      const std::string layer = "layer" + std::to_string(li + 1);
      const int planes = mc << li, stride = li ? 2 : 1;
      const int nb = n_blocks(m, layer);
      if (nb == 0) throw SpkError(SPK_E_WEIGHTS, "no blocks in " + layer);
      const int Ho = (x.H - 1) / stride + 1, Wo = (x.W - 1) / stride + 1;
      const size_t osz = (size_t)B * Ho * Wo * ChanMap::dense(planes * expansion).n_phys;
      Buf pp[2] = {b.alloc(osz), b.alloc(osz)};
      for (int bi = 0; bi < nb; ++bi) {
        const std::string p = layer + "." + std::to_string(bi);
        x = res2 ? res2block(p, x, bi ? 1 : stride, planes, pp[bi & 1]) : basic(p, x, bi ? 1 : stride, planes, pp[bi & 1]);
      }
    }
    head(x);
  }

  // ---- TSTP (pooling_layers.py:47-55) -> seg_1 [-> ReLU -> seg_bn_1 -> seg_2]
  void head(const R4& f) {
    const int B = b.B, H4 = f.H, C4 = f.C, S = 2 * H4 * C4;
    const Buf stats = b.alloc((size_t)B * S);
    if (b.plan) {
      const R4 ff = f;
      b.step("pool", [=](const Ctx& c) {
        return launch_tstp(c.resolve(ff.buf), B, ff.H, ff.W, ff.C, ff.ld, 1e-8f, 1, c.resolve(stats), c.stream);
      });
    }
    ChanMap perm;                                    // reference flattens (C, F): c*H + h -> ours h*C + c
    perm.phys.resize(S);
    perm.n_phys = S;
    for (int part = 0; part < 2; ++part)
      for (int c = 0; c < C4; ++c)
        for (int h = 0; h < H4; ++h) perm.phys[part * H4 * C4 + c * H4 + h] = part * H4 * C4 + h * C4 + c;
    const int E = (int)m.dim("seg_1.weight", 0);
    if (E % 4) throw SpkError(SPK_E_UNSUPPORTED, "embedding_size must be a multiple of 4");
    if (m.dim("seg_1.weight", 1) != S) throw SpkError(SPK_E_WEIGHTS, "seg_1 in_features != pooled stats size");
    const bool two = m.cfg.two_emb_layer != 0;
    const ChanMap em = ChanMap::dense(E, 1);
    const Packed& seg1 = m.pack("seg_1", em, {Part{"seg_1.weight", "seg_1.bias", "", perm, 0, 0}}, S);
    b.macs_per_utt += (double)S * E;
    Buf e1 = two ? b.alloc((size_t)B * E) : Buf{Buf::OUT, 0, nullptr};
    const Packed* pa = two ? &m.pack_post_affine("seg_bn_1", "seg_bn_1", em) : nullptr;
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = 1;
      const R4 st{stats, S, 1, 1, S};
      d.s0 = src(st, S, 1, 1, 0);
      d.ldo = E;
      if (two) {
        d.act = ACT_RELU;
        d.post_scale = m.dptr(pa->ps_off);
        d.post_shift = m.dptr(pa->pt_off);
      }
      Builder::ConvIO io; io.s0 = stats; io.out = e1;
      b.conv("seg_1", d, seg1, io);
    }
    if (two) {
      const Packed& seg2 = m.pack("seg_2", em, {Part{"seg_2.weight", "seg_2.bias", "", ChanMap::dense(E, 1), 0, 0}}, E);
      b.macs_per_utt += (double)E * E;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = 1;
        const R4 t{e1, E, 1, 1, E};
        d.s0 = src(t, E, 1, 1, 0);
        d.ldo = E;
        Builder::ConvIO io; io.s0 = e1; io.out = Buf{Buf::OUT, 0, nullptr};
        b.conv("seg_2", d, seg2, io);
      }
    }
  }
};

}  // namespace

void build_resnet(Builder& b, int T, bool res2) {
  ResBuilder rb(b, res2);
  rb.run(T);
}

}  // namespace spk
