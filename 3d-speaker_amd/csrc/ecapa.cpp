// ECAPA-TDNN launch plan.
//
// Reference: speakerlab/models/ecapa_tdnn/ECAPA_TDNN.py — Conv1d 'same'/reflect :42-106,
// TDNNBlock :127-151 (conv -> ReLU -> BN), Res2NetBlock :154-191, SEBlock :194-222,
// AttentiveStatisticsPooling :225-287, SERes2NetBlock :290-347, ECAPA_TDNN :350-463.
//
// Layout: channels-last [B, T, C].  Mapping onto the fused GEMM:
//   * reflect padding is done by the operand loader (no padded copy);
//   * BN after ReLU is the GEMM's post-affine epilogue (not foldable into the weights);
//   * Res2Net: chunk j (j >= 2) reads `x_j + y_{j-1}` through the dual-operand load; y_0 is
//     x_0 itself, so tdnn2 K-concatenates [h1 chunk 0 | y_1..y_7] instead of copying;
//   * the three SE-Res2Net block outputs are written straight into the MFA input buffer
//     (torch.cat(xl[1:]) costs nothing);
//   * ASP global context: W [x; mean; std] = W_x x + (W_m mean + W_s std), and the second
//     term is constant over time, so it is one [B, 6144] x [6144, 128] GEMM whose result
//     is added per utterance (rowbias) to the [B*T, 3072] x [3072, 128] GEMM;
//   * asp_bn is folded into fc on the input side.
#include "runtime.h"
#include "tdnn_ops.h"

namespace spk {

namespace {

ConvSrc src1d(int ld, int T, int cin, int k = 1, int dil = 1, bool reflect = false) {
  ConvSrc s;
  s.ld = ld; s.H = 1; s.W = T; s.cin = cin;
  s.kh = 1; s.kw = k; s.dw = dil;
  s.pw = reflect ? dil * (k - 1) / 2 : 0;
  // a one-tap conv has no padding to reflect: flagging it would keep the 3072-deep MFA GEMM
  // off the buffer-resource loader (conv_buf_loader_ok) for nothing
  s.reflect = reflect && k > 1 ? 1 : 0;
  return s;
}

ConvSrc src_vec(int cin) {   // [B, cin] as B images of one pixel
  ConvSrc s;
  s.ld = cin; s.H = 1; s.W = 1; s.cin = cin;
  return s;
}

}  // namespace

void build_ecapa(Builder& b, int T) {
  Model& m = b.m;
  const int B = b.B;
  const int F = m.cfg.feat_dim;
  int C[5], K[5], D[5];
  for (int i = 0; i < 5; ++i) {
    C[i] = m.cfg.channels[i] ? m.cfg.channels[i] : (i < 4 ? 512 : 1536);
    K[i] = m.cfg.kernel_sizes[i] ? m.cfg.kernel_sizes[i] : (i == 0 ? 5 : (i < 4 ? 3 : 1));
    D[i] = m.cfg.dilations[i] ? m.cfg.dilations[i] : (i == 4 ? 1 : i + 1);
  }
  if (F % 4) throw SpkError(SPK_E_UNSUPPORTED, "ECAPA input_size must be a multiple of 4");
  for (int i = 0; i < 5; ++i)
    if (C[i] % 32) throw SpkError(SPK_E_UNSUPPORTED, "ECAPA channels must be multiples of 32");
  const int pad0 = D[0] * (K[0] - 1) / 2;
  if (T <= pad0 || T <= D[1] || T <= D[2] || T <= D[3]) throw SpkError(SPK_E_INVALID, "utterance too short for reflect padding");
  const int catC = C[1] + C[2] + C[3];
  if (catC != C[4]) throw SpkError(SPK_E_WEIGHTS, "ECAPA: mfa input must be the concatenation of the 3 blocks");
  const double Td = T;
  // forward(x, lengths) (ECAPA_TDNN.py:430-454): the convolutions run over the whole padded
  // [B, T] input exactly like the reference (no masking there); only the SE squeeze means
  // and the attentive-pooling statistics are restricted to each utterance's valid frames
  const Buf LENS = b.ragged ? Buf{Buf::LEN, 0, nullptr} : Buf{};
  int cmax = std::max(std::max(C[0], C[1]), std::max(C[2], C[3]));

  auto post = [&](const std::string& bn, int n) { return &m.pack_post_affine(bn, bn, ChanMap::dense(n)); };
  auto set_post = [&](ConvDesc& d, const Packed* p) {
    d.post_scale = m.dptr(p->ps_off);
    d.post_shift = m.dptr(p->pt_off);
  };

  // ---- blocks.0: TDNNBlock(F -> C0, k5) on the input features [B, T, F]
  const Buf X0 = b.alloc((size_t)B * T * C[0]);
  {
    const Packed& p = m.pack("blocks.0", ChanMap::dense(C[0]),
                             {Part{"blocks.0.conv.conv.weight", "blocks.0.conv.conv.bias", "", ChanMap::dense(F), 0, 0}},
                             K[0] * F);
    const Packed* pa = post("blocks.0.norm.norm", C[0]);
    b.macs_per_utt += Td * C[0] * F * K[0];
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = T;
      d.s0 = src1d(F, T, F, K[0], D[0], true);
      d.ldo = C[0]; d.act = ACT_RELU;
      set_post(d, pa);
      Builder::ConvIO io; io.s0 = Buf{Buf::IN, 0, nullptr}; io.out = X0;
      b.conv("blocks.0", d, p, io);
    }
  }
  const Buf CATB = b.alloc((size_t)B * T * catC);
  const Buf H = b.alloc((size_t)B * T * cmax), R = b.alloc((size_t)B * T * cmax), H2 = b.alloc((size_t)B * T * cmax);
  const Buf SC = b.alloc((size_t)B * T * cmax);
  const Buf S = b.alloc((size_t)B * cmax), S1 = b.alloc((size_t)B * 512), G = b.alloc((size_t)B * cmax);

  Buf xin = X0;
  int xin_ld = C[0], xin_c = C[0];
  int cat_off = 0;
  for (int i = 1; i <= 3; ++i) {
    const std::string p = "blocks." + std::to_string(i);
    const int Ci = C[i];
    int scale = 1;
    while (m.has(p + ".res2net_block.blocks." + std::to_string(scale - 1) + ".conv.conv.weight")) ++scale;
    if (scale < 2 || Ci % scale) throw SpkError(SPK_E_WEIGHTS, p + ": bad res2net scale");
    const int w = Ci / scale;
    if (w % 4) throw SpkError(SPK_E_UNSUPPORTED, p + ": res2net width must be a multiple of 4");
    // residual (shortcut conv when channels change)
    Buf res = xin;
    int res_ld = xin_ld;
    if (m.has(p + ".shortcut.conv.weight")) {
      const Packed& ps = m.pack(p + ".shortcut", ChanMap::dense(Ci),
                               {Part{p + ".shortcut.conv.weight", p + ".shortcut.conv.bias", "", ChanMap::dense(xin_c), 0, 0}},
                               xin_c);
      b.macs_per_utt += Td * Ci * xin_c;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T;
        d.s0 = src1d(xin_ld, T, xin_c);
        d.ldo = Ci;
        Builder::ConvIO io; io.s0 = xin; io.out = SC;
        b.conv(p + ".shortcut", d, ps, io);
      }
      res = SC;
      res_ld = Ci;
    }
    // tdnn1
    {
      const Packed& pp = m.pack(p + ".tdnn1", ChanMap::dense(Ci),
                                {Part{p + ".tdnn1.conv.conv.weight", p + ".tdnn1.conv.conv.bias", "", ChanMap::dense(xin_c), 0, 0}},
                                xin_c);
      const Packed* pa = post(p + ".tdnn1.norm.norm", Ci);
      b.macs_per_utt += Td * Ci * xin_c;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T;
        d.s0 = src1d(xin_ld, T, xin_c);
        d.ldo = Ci; d.act = ACT_RELU;
        set_post(d, pa);
        Builder::ConvIO io; io.s0 = xin; io.out = H;
        b.conv(p + ".tdnn1", d, pp, io);
      }
    }
    // res2net chain: y_1 = tdnn(x_1); y_j = tdnn(x_j + y_{j-1})
    for (int j = 1; j < scale; ++j) {
      const std::string q = p + ".res2net_block.blocks." + std::to_string(j - 1);
      const Packed& pp = m.pack(q, ChanMap::dense(w),
                                {Part{q + ".conv.conv.weight", q + ".conv.conv.bias", "", ChanMap::dense(w), 0, 0}}, K[i] * w);
      const Packed* pa = post(q + ".norm.norm", w);
      b.macs_per_utt += Td * w * w * K[i];
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T;
        d.s0 = src1d(Ci, T, w, K[i], D[i], true);
        Builder::ConvIO io;
        io.s0 = H.at((size_t)j * w);
        if (j >= 2) {
          d.s0.ld2 = Ci;
          io.s0b = R.at((size_t)(j - 1) * w);
        }
        d.ldo = Ci; d.act = ACT_RELU;
        set_post(d, pa);
        io.out = R.at((size_t)j * w);
        b.conv(q, d, pp, io);
      }
    }
    // tdnn2 over [h chunk 0 | y_1 .. y_{scale-1}]
    {
      const std::string q = p + ".tdnn2";
      const Packed& pp = m.pack(q, ChanMap::dense(Ci),
                                {Part{q + ".conv.conv.weight", q + ".conv.conv.bias", "", ChanMap::dense(w), 0, 0},
                                 Part{q + ".conv.conv.weight", q + ".conv.conv.bias", "", ChanMap::dense(Ci - w), w, w}},
                                Ci);
      const Packed* pa = post(q + ".norm.norm", Ci);
      b.macs_per_utt += Td * Ci * Ci;
      if (b.plan) {
        ConvDesc d;
        d.nimg = B; d.Ho = 1; d.Wo = T;
        d.s0 = src1d(Ci, T, w);
        d.s1 = src1d(Ci, T, Ci - w);
        d.ldo = Ci; d.act = ACT_RELU;
        set_post(d, pa);
        Builder::ConvIO io; io.s0 = H; io.s1 = R.at((size_t)w); io.out = H2;
        b.conv(q, d, pp, io);
      }
    }
    // SE: s = mean_T -> relu(conv1) -> sigmoid(conv2) ; out = h2 * s + residual
    {
      const std::string q = p + ".se_block";
      const int se = (int)m.dim(q + ".conv1.conv.weight", 0);
      if (se % 4 || se > 512) throw SpkError(SPK_E_UNSUPPORTED, q + ": se_channels must be a multiple of 4 <= 512");
      const Packed& p1 = m.pack(q + ".conv1", ChanMap::dense(se),
                                {Part{q + ".conv1.conv.weight", q + ".conv1.conv.bias", "", ChanMap::dense(Ci), 0, 0}}, Ci);
      const Packed& p2 = m.pack(q + ".conv2", ChanMap::dense(Ci),
                                {Part{q + ".conv2.conv.weight", q + ".conv2.conv.bias", "", ChanMap::dense(se), 0, 0}}, se);
      b.macs_per_utt += 2.0 * Ci * se;
      if (b.plan) {
        b.writes({{S, Builder::BOUNDED}}).step(q + ".mean", [=](const Ctx& c) { return launch_time_mean(c.resolve(H2), B, T, Ci, Ci, c.resolve(S), Ci, c.stream, c.resolve_i(LENS)); });
        ConvDesc d1;
        d1.nimg = B; d1.Ho = 1; d1.Wo = 1;
        d1.s0 = src_vec(Ci);
        d1.ldo = se; d1.act = ACT_RELU;
        Builder::ConvIO io1; io1.s0 = S; io1.out = S1;
        b.conv(q + ".conv1", d1, p1, io1);
        ConvDesc d2;
        d2.nimg = B; d2.Ho = 1; d2.Wo = 1;
        d2.s0 = src_vec(se);
        d2.ldo = Ci; d2.act = ACT_SIGMOID;
        Builder::ConvIO io2; io2.s0 = S1; io2.out = G;
        b.conv(q + ".conv2", d2, p2, io2);
        const Buf out = CATB.at((size_t)cat_off);
        b.writes({{out, Builder::NOTED}}).step(p + ".se_apply", [=](const Ctx& c) {
          return launch_se_apply(c.resolve(H2), Ci, c.resolve(G), Ci, c.resolve(res), res_ld, c.resolve(out), catC, B, T,
                                 Ci, c.stream, c.flag);
        });
      }
    }
    xin = CATB.at((size_t)cat_off);
    xin_ld = catC;
    xin_c = Ci;
    cat_off += Ci;
  }

  // ---- MFA: TDNNBlock(3072 -> 3072, k1)
  const int Cm = C[4];
  const Buf A = b.alloc((size_t)B * T * Cm);
  {
    const Packed& pp = m.pack("mfa", ChanMap::dense(Cm),
                              {Part{"mfa.conv.conv.weight", "mfa.conv.conv.bias", "", ChanMap::dense(catC), 0, 0}}, catC * K[4]);
    const Packed* pa = post("mfa.norm.norm", Cm);
    b.macs_per_utt += Td * Cm * catC * K[4];
    if (b.plan) {
      ConvDesc d;
      d.nimg = B; d.Ho = 1; d.Wo = T;
      d.s0 = src1d(catC, T, catC, K[4], D[4], true);
      d.ldo = Cm; d.act = ACT_RELU;
      set_post(d, pa);
      Builder::ConvIO io; io.s0 = CATB; io.out = A;
      b.conv("mfa", d, pp, io);
    }
  }
  // ---- attentive statistics pooling (global context)
  const int att = (int)m.dim("asp.tdnn.conv.conv.weight", 0);
  if (att % 4) throw SpkError(SPK_E_UNSUPPORTED, "attention_channels must be a multiple of 4");
  if (m.dim("asp.tdnn.conv.conv.weight", 1) != 3 * Cm) throw SpkError(SPK_E_UNSUPPORTED, "ASP global_context=False");
  const Buf MS = b.alloc((size_t)B * 2 * Cm), CB = b.alloc((size_t)B * att), HA = b.alloc((size_t)B * T * att);
  const Buf L = b.alloc((size_t)B * T * Cm), P = b.alloc((size_t)B * 2 * Cm);
  const Packed& pctx = m.pack("asp.tdnn.ctx", ChanMap::dense(att),
                              {Part{"asp.tdnn.conv.conv.weight", "", "", ChanMap::dense(2 * Cm), Cm, 0}}, 2 * Cm);
  const Packed& patt = m.pack("asp.tdnn.x", ChanMap::dense(att),
                              {Part{"asp.tdnn.conv.conv.weight", "asp.tdnn.conv.conv.bias", "", ChanMap::dense(Cm), 0, 0}}, Cm);
  const Packed* pan = post("asp.tdnn.norm.norm", att);
  const Packed& patt2 = m.pack("asp.conv", ChanMap::dense(Cm),
                               {Part{"asp.conv.conv.weight", "asp.conv.conv.bias", "", ChanMap::dense(att), 0, 0}}, att);
  // reference-algorithmic MACs (the context half of asp.tdnn is computed once per utterance)
  const double macs_ctx = Td * att * 2.0 * Cm, macs_att = Td * att * (double)Cm, macs_conv = Td * Cm * (double)att;
  const int E = (int)m.dim("fc.conv.weight", 0);
  if (E % 4) throw SpkError(SPK_E_UNSUPPORTED, "lin_neurons must be a multiple of 4");
  Part fcp{"fc.conv.weight", "fc.conv.bias", "", ChanMap::dense(2 * Cm), 0, 0};
  fcp.bn_in = "asp_bn.norm";
  const Packed& pfc = m.pack("fc", ChanMap::dense(E, 1), {fcp}, 2 * Cm);
  const double macs_fc = (double)E * 2 * Cm;
  if (!b.plan) {
    b.macs_per_utt += macs_ctx + macs_att + macs_conv + macs_fc;
    return;
  }
  b.writes({{MS, Builder::BOUNDED}}).step("asp.stats", [=](const Ctx& c) { return launch_asp_stats(c.resolve(A), B, T, Cm, Cm, 1e-12f, c.resolve(MS), c.stream, c.resolve_i(LENS)); });
  {
    ConvDesc d;
    d.nimg = B; d.Ho = 1; d.Wo = 1;
    d.s0 = src_vec(2 * Cm);
    d.ldo = att;
    Builder::ConvIO io; io.s0 = MS; io.out = CB;
    b.macs_per_utt += macs_ctx;
    b.conv("asp.tdnn.ctx", d, pctx, io, /*use_bias=*/false);
  }
  {
    ConvDesc d;
    d.nimg = B; d.Ho = 1; d.Wo = T;
    d.s0 = src1d(Cm, T, Cm);
    d.ldo = att; d.act = ACT_RELU; d.act2 = ACT_TANH;
    d.rowbias_ld = att;
    set_post(d, pan);
    Builder::ConvIO io; io.s0 = A; io.out = HA; io.rowbias = CB;
    b.macs_per_utt += macs_att;
    b.conv("asp.tdnn", d, patt, io);
  }
  {
    ConvDesc d;
    d.nimg = B; d.Ho = 1; d.Wo = T;
    d.s0 = src1d(att, T, att);
    d.ldo = Cm;
    Builder::ConvIO io; io.s0 = HA; io.out = L;
    b.macs_per_utt += macs_conv;
    b.conv("asp.conv", d, patt2, io);
  }
  b.writes({{P, Builder::BOUNDED}}).step("asp.pool", [=](const Ctx& c) {
    return launch_attn_pool(c.resolve(L), Cm, c.resolve(A), Cm, B, T, Cm, 1e-12f, c.resolve(P), c.stream,
                            c.resolve_i(LENS));
  });
  {
    ConvDesc d;
    d.nimg = B; d.Ho = 1; d.Wo = 1;
    d.s0 = src_vec(2 * Cm);
    d.ldo = E;
    Builder::ConvIO io; io.s0 = P; io.out = Buf{Buf::OUT, 0, nullptr};
    b.macs_per_utt += macs_fc;
    b.conv("fc", d, pfc, io);
  }
}

}  // namespace spk
