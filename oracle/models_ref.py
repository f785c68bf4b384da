"""ORACLE (test infrastructure only) — functional fp32/fp64 CPU restatement of the four
speaker-embedding forwards on the north-star path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product modules in ``3d-speaker_amd/speakerlab/models`` run the
HIP executor and never call into here.

Every function takes a plain ``state_dict`` (key -> torch tensor, the reference's key
layout) and restates the reference forward op for op with ``torch.nn.functional``:

* ERes2NetV2   — ``speakerlab/models/eres2net/ERes2NetV2.py:31-254``
* ERes2Net     — ``speakerlab/models/eres2net/ERes2Net.py:30-231``
* AFF          — ``speakerlab/models/eres2net/fusion.py:8-28``
* TSTP         — ``speakerlab/models/eres2net/pooling_layers.py:38-55`` (TAP / TSDP :10-35, ASTP :58-104)
* ECAPA_TDNN   — ``speakerlab/models/ecapa_tdnn/ECAPA_TDNN.py:29-463``
* CAMPPlus     — ``speakerlab/models/campplus/DTDNN.py:13-115``, ``layers.py:10-253``
* ResNet34     — ``speakerlab/models/resnet/ResNet.py:15-113``
* Res2Net      — ``speakerlab/models/res2net/Res2Net.py:17-147``

It is pinned against golden embeddings produced by the reference modules themselves
(``tests/golden/make_golden.py``) in ``tests/test_oracle_models.py``.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]


def _bn(x, sd: SD, p: str, eps: float = 1e-5):
    w = sd.get(p + '.weight')
    b = sd.get(p + '.bias')
    return F.batch_norm(x, sd[p + '.running_mean'], sd[p + '.running_var'], w, b, False, 0.0, eps)


def _htanh(x):
    """``ReLU(nn.Hardtanh(0, 20))`` (ERes2NetV2.py:20-28, ERes2Net.py:19-27)."""
    return torch.clamp(x, 0.0, 20.0)


# ----------------------------------------------------------------------------- ERes2Net
def _aff(sd: SD, p: str, x, y):
    """AFF fusion.py:22-28."""
    xa = torch.cat((x, y), 1)
    a = F.conv2d(xa, sd[p + '.local_att.0.weight'], sd[p + '.local_att.0.bias'])
    a = F.silu(_bn(a, sd, p + '.local_att.1'))
    a = F.conv2d(a, sd[p + '.local_att.3.weight'], sd[p + '.local_att.3.bias'])
    a = _bn(a, sd, p + '.local_att.4')
    a = 1.0 + torch.tanh(a)
    return x * a + y * (2.0 - a)


def _eres2_block(sd: SD, p: str, x, stride: int, width: int, scale: int, aff: bool):
    """BasicBlockERes2NetV2(.AFF) ERes2NetV2.py:65-91 / 132-159 (ERes2Net blocks are
    identical in forward, ERes2Net.py:61-87 / 125-152)."""
    out = F.conv2d(x, sd[p + '.conv1.weight'], stride=stride)
    out = _htanh(_bn(out, sd, p + '.bn1'))
    spx = torch.split(out, width, 1)
    outs = []
    sp = None
    for i in range(scale):
        if i == 0:
            sp = spx[0]
        elif aff:
            sp = _aff(sd, f'{p}.fuse_models.{i - 1}', sp, spx[i])
        else:
            sp = sp + spx[i]
        sp = F.conv2d(sp, sd[f'{p}.convs.{i}.weight'], padding=1)
        sp = _htanh(_bn(sp, sd, f'{p}.bns.{i}'))
        outs.append(sp)
    out = torch.cat(outs, 1)
    out = _bn(F.conv2d(out, sd[p + '.conv3.weight']), sd, p + '.bn3')
    if (p + '.shortcut.0.weight') in sd:
        res = _bn(F.conv2d(x, sd[p + '.shortcut.0.weight'], stride=stride), sd, p + '.shortcut.1')
    else:
        res = x
    return _htanh(out + res)


def _tstp(x, pooling='TSTP'):
    """TSTP pooling_layers.py:47-55: mean_T, sqrt(var_T(unbiased) + 1e-8), flatten (C,F);
    TAP (:17-21) keeps the mean part, TSDP (:30-35) the std part."""
    mean = x.mean(dim=-1).flatten(start_dim=1)
    std = torch.sqrt(torch.var(x, dim=-1) + 1e-8).flatten(start_dim=1)
    if pooling == 'TAP':
        return mean
    if pooling == 'TSDP':
        return std
    return torch.cat((mean, std), 1)


def _astp(sd: SD, x, prefix='pool'):
    """ASTP pooling_layers.py:58-104 (global_context_att=False): alpha = softmax_T(linear2(
    tanh(linear1(x)))) over (C*F, T); mean = sum alpha x, std = sqrt(clamp(sum alpha x^2 -
    mean^2, 1e-10)), cat(mean, std)."""
    x = x.reshape(x.shape[0], x.shape[1] * x.shape[2], x.shape[3])
    a = torch.tanh(F.conv1d(x, sd[f'{prefix}.linear1.weight'], sd[f'{prefix}.linear1.bias']))
    a = torch.softmax(F.conv1d(a, sd[f'{prefix}.linear2.weight'], sd[f'{prefix}.linear2.bias']), dim=2)
    mean = torch.sum(a * x, dim=2)
    var = torch.sum(a * (x ** 2), dim=2) - mean ** 2
    return torch.cat([mean, torch.sqrt(var.clamp(min=1e-10))], dim=1)


def _eres2_layer(sd: SD, name: str, x, n_blocks: int, stride: int, width: int, scale: int, aff: bool):
    for b in range(n_blocks):
        x = _eres2_block(sd, f'{name}.{b}', x, stride if b == 0 else 1, width, scale, aff)
    return x


def eres2netv2_forward(sd: SD, x, m_channels=64, base_width=26, scale=2, num_blocks=(3, 4, 6, 3),
                       two_emb_layer=False, pooling='TSTP'):
    """ERes2NetV2.forward ERes2NetV2.py:235-254. x: [B, T, F]."""
    x = x.permute(0, 2, 1).unsqueeze(1)
    out = F.relu(_bn(F.conv2d(x, sd['conv1.weight'], padding=1), sd, 'bn1'))
    widths = [int(math.floor(m_channels * (2 ** i) * (base_width / 64.0))) for i in range(4)]
    out1 = _eres2_layer(sd, 'layer1', out, num_blocks[0], 1, widths[0], scale, False)
    out2 = _eres2_layer(sd, 'layer2', out1, num_blocks[1], 2, widths[1], scale, False)
    out3 = _eres2_layer(sd, 'layer3', out2, num_blocks[2], 2, widths[2], scale, True)
    out4 = _eres2_layer(sd, 'layer4', out3, num_blocks[3], 2, widths[3], scale, True)
    out3_ds = F.conv2d(out3, sd['layer3_ds.weight'], stride=2, padding=1)
    fused = _aff(sd, 'fuse34', out4, out3_ds)
    stats = _astp(sd, fused) if pooling == 'ASTP' else _tstp(fused, pooling)
    emb = F.linear(stats, sd['seg_1.weight'], sd['seg_1.bias'])
    if two_emb_layer:
        emb = F.linear(_bn(F.relu(emb), sd, 'seg_bn_1'), sd['seg_2.weight'], sd['seg_2.bias'])
    return emb


def eres2net_forward(sd: SD, x, m_channels=32, base_width=32, scale=2, num_blocks=(3, 4, 6, 3), two_emb_layer=False):
    """ERes2Net.forward ERes2Net.py:208-231 (baseWidth 32, scale 2, expansion 2); also
    ERes2Net_huge.py:206-232 (baseWidth 24, scale 3, expansion 4)."""
    x = x.permute(0, 2, 1).unsqueeze(1)
    out = F.relu(_bn(F.conv2d(x, sd['conv1.weight'], padding=1), sd, 'bn1'))
    widths = [int(math.floor(m_channels * (2 ** i) * (base_width / 64.0))) for i in range(4)]
    out1 = _eres2_layer(sd, 'layer1', out, num_blocks[0], 1, widths[0], scale, False)
    out2 = _eres2_layer(sd, 'layer2', out1, num_blocks[1], 2, widths[1], scale, False)
    out1_ds = F.conv2d(out1, sd['layer1_downsample.weight'], stride=2, padding=1)
    f12 = _aff(sd, 'fuse_mode12', out2, out1_ds)
    out3 = _eres2_layer(sd, 'layer3', out2, num_blocks[2], 2, widths[2], scale, True)
    f12_ds = F.conv2d(f12, sd['layer2_downsample.weight'], stride=2, padding=1)
    f123 = _aff(sd, 'fuse_mode123', out3, f12_ds)
    out4 = _eres2_layer(sd, 'layer4', out3, num_blocks[3], 2, widths[3], scale, True)
    f123_ds = F.conv2d(f123, sd['layer3_downsample.weight'], stride=2, padding=1)
    f1234 = _aff(sd, 'fuse_mode1234', out4, f123_ds)
    emb = F.linear(_tstp(f1234), sd['seg_1.weight'], sd['seg_1.bias'])
    if two_emb_layer:
        emb = F.linear(_bn(F.relu(emb), sd, 'seg_bn_1'), sd['seg_2.weight'], sd['seg_2.bias'])
    return emb


# ----------------------------------------------------------------------------- ResNet / Res2Net
def _stem(sd: SD, x):
    x = x.permute(0, 2, 1).unsqueeze(1)
    return F.relu(_bn(F.conv2d(x, sd['conv1.weight'], padding=1), sd, 'bn1'))


def _head(sd: SD, out, two_emb_layer):
    emb = F.linear(_tstp(out), sd['seg_1.weight'], sd['seg_1.bias'])
    if two_emb_layer:
        emb = F.linear(_bn(F.relu(emb), sd, 'seg_bn_1'), sd['seg_2.weight'], sd['seg_2.bias'])
    return emb


def _shortcut(sd: SD, p: str, x, stride):
    if p + '.shortcut.0.weight' in sd:
        return _bn(F.conv2d(x, sd[p + '.shortcut.0.weight'], stride=stride), sd, p + '.shortcut.1')
    return x


def _resnet_block(sd: SD, p: str, x, stride):
    """BasicBlock ResNet.py:30-35."""
    out = F.relu(_bn(F.conv2d(x, sd[p + '.conv1.weight'], stride=stride, padding=1), sd, p + '.bn1'))
    out = _bn(F.conv2d(out, sd[p + '.conv2.weight'], padding=1), sd, p + '.bn2')
    return F.relu(out + _shortcut(sd, p, x, stride))


def resnet_forward(sd: SD, x, num_blocks=(3, 4, 6, 3), two_emb_layer=True):
    """ResNet.forward ResNet.py:86-101 (TSTP pooling)."""
    out = _stem(sd, x)
    for li, n in enumerate(num_blocks):
        for b in range(n):
            out = _resnet_block(sd, f'layer{li + 1}.{b}', out, (2 if li else 1) if b == 0 else 1)
    return _head(sd, out, two_emb_layer)


def _res2net_block(sd: SD, p: str, x, stride, width, scale):
    """BasicBlockRes2Net Res2Net.py:59-87: the last split passes through to the concat."""
    out = _htanh(_bn(F.conv2d(x, sd[p + '.conv1.weight'], stride=stride), sd, p + '.bn1'))
    spx = torch.split(out, width, 1)
    nums = scale - 1
    outs = []
    sp = None
    for i in range(nums):
        sp = spx[i] if i == 0 else sp + spx[i]
        sp = _htanh(_bn(F.conv2d(sp, sd[f'{p}.convs.{i}.weight'], padding=1), sd, f'{p}.bns.{i}'))
        outs.append(sp)
    out = torch.cat(outs + [spx[nums]], 1)
    out = _bn(F.conv2d(out, sd[p + '.conv3.weight']), sd, p + '.bn3')
    return _htanh(out + _shortcut(sd, p, x, stride))


def res2net_forward(sd: SD, x, m_channels=32, base_width=32, scale=2, num_blocks=(3, 4, 6, 3), two_emb_layer=False):
    """Res2Net.forward Res2Net.py:128-147 (TSTP pooling)."""
    out = _stem(sd, x)
    for li, n in enumerate(num_blocks):
        width = int(math.floor(m_channels * (2 ** li) * (base_width / 64.0)))
        for b in range(n):
            out = _res2net_block(sd, f'layer{li + 1}.{b}', out, (2 if li else 1) if b == 0 else 1, width, scale)
    return _head(sd, out, two_emb_layer)


# ----------------------------------------------------------------------------- ECAPA
def _same_reflect_conv1d(x, w, b, dilation=1):
    """speechbrain-style ``Conv1d(padding='same', padding_mode='reflect')``
    ECAPA_TDNN.py:29-39 (get_padding_elem, stride 1) and :95-106."""
    k = w.shape[-1]
    L = x.shape[-1]
    l_out = (L - dilation * (k - 1) - 1) + 1
    pad = (L - l_out) // 2
    if pad > 0:
        x = F.pad(x, [pad, pad], mode='reflect')
    return F.conv1d(x, w, b, dilation=dilation)


def _tdnn_block(sd: SD, p: str, x, dilation=1):
    """TDNNBlock ECAPA_TDNN.py:127-151: conv -> ReLU -> BN (post-activation BN)."""
    y = _same_reflect_conv1d(x, sd[p + '.conv.conv.weight'], sd[p + '.conv.conv.bias'], dilation)
    return _bn(F.relu(y), sd, p + '.norm.norm')


def _length_mask(lengths, L):
    """length_to_mask(lengths * L, max_len=L) ECAPA_TDNN.py:11-27, as [B, 1, L] in the dtype
    of ``lengths`` (float32 for the reference's default ``torch.ones``), like the reference."""
    m = torch.arange(L, dtype=lengths.dtype).expand(len(lengths), L) < (lengths * L).unsqueeze(1)
    return m.to(lengths.dtype).unsqueeze(1)


def _seres2net_block(sd: SD, p: str, x, dilation, scale=8, lengths=None):
    """SERes2NetBlock ECAPA_TDNN.py:290-347 with Res2NetBlock :154-191 and SEBlock :194-222
    (masked squeeze mean with relative ``lengths``, :209-216)."""
    residual = x
    if (p + '.shortcut.conv.weight') in sd:
        residual = _same_reflect_conv1d(x, sd[p + '.shortcut.conv.weight'], sd[p + '.shortcut.conv.bias'])
    x = _tdnn_block(sd, p + '.tdnn1', x)
    ys = []
    y_i = None
    for i, x_i in enumerate(torch.chunk(x, scale, dim=1)):
        if i == 0:
            y_i = x_i
        elif i == 1:
            y_i = _tdnn_block(sd, f'{p}.res2net_block.blocks.{i - 1}', x_i, dilation)
        else:
            y_i = _tdnn_block(sd, f'{p}.res2net_block.blocks.{i - 1}', x_i + y_i, dilation)
        ys.append(y_i)
    x = torch.cat(ys, 1)
    x = _tdnn_block(sd, p + '.tdnn2', x)
    if lengths is not None:
        mask = _length_mask(lengths, x.shape[-1])
        s = (x * mask).sum(dim=2, keepdim=True) / mask.sum(dim=2, keepdim=True)
    else:
        s = x.mean(dim=2, keepdim=True)
    s = F.relu(F.conv1d(s, sd[p + '.se_block.conv1.conv.weight'], sd[p + '.se_block.conv1.conv.bias']))
    s = torch.sigmoid(F.conv1d(s, sd[p + '.se_block.conv2.conv.weight'], sd[p + '.se_block.conv2.conv.bias']))
    return s * x + residual


def _asp(sd: SD, p: str, x, eps=1e-12, lengths=None):
    """AttentiveStatisticsPooling ECAPA_TDNN.py:243-287, global_context=True; relative
    ``lengths`` mask the global statistics and the softmax (-inf fill)."""
    L = x.shape[-1]
    if lengths is None:
        lengths = torch.ones(x.shape[0])
    mask = _length_mask(lengths, L)
    m = mask / mask.sum(dim=2, keepdim=True).float()     # float32 weights, as the reference

    def stats(x, m):
        mean = (m * x).sum(2)
        std = torch.sqrt((m * (x - mean.unsqueeze(2)).pow(2)).sum(2).clamp(eps))
        return mean, std

    mean, std = stats(x, m)
    attn = torch.cat([x, mean.unsqueeze(2).repeat(1, 1, L), std.unsqueeze(2).repeat(1, 1, L)], 1)
    attn = torch.tanh(_tdnn_block(sd, p + '.tdnn', attn))
    attn = F.conv1d(attn, sd[p + '.conv.conv.weight'], sd[p + '.conv.conv.bias'])
    attn = attn.masked_fill(mask == 0, float('-inf'))
    attn = F.softmax(attn, dim=2)
    mean, std = stats(x, attn)
    return torch.cat((mean, std), 1).unsqueeze(2)


def ecapa_forward(sd: SD, x, dilations=(1, 2, 3, 4, 1), lengths=None):
    """ECAPA_TDNN.forward ECAPA_TDNN.py:430-463. x: [B, T, F] -> [B, lin_neurons];
    ``lengths``: relative lengths (masked SE / ASP statistics)."""
    x = x.transpose(1, 2)
    xl = []
    x = _tdnn_block(sd, 'blocks.0', x, dilations[0])
    xl.append(x)
    i = 1
    while f'blocks.{i}.tdnn1.conv.conv.weight' in sd:
        x = _seres2net_block(sd, f'blocks.{i}', x, dilations[i], lengths=lengths)
        xl.append(x)
        i += 1
    x = torch.cat(xl[1:], 1)
    x = _tdnn_block(sd, 'mfa', x)
    x = _asp(sd, 'asp', x, lengths=lengths)
    x = _bn(x, sd, 'asp_bn.norm')
    x = F.conv1d(x, sd['fc.conv.weight'], sd['fc.conv.bias'])
    return x.transpose(1, 2).squeeze(1)


# ----------------------------------------------------------------------------- CAM++
def _bn_relu(sd: SD, p: str, x):
    """get_nonlinear('batchnorm-relu') layers.py:10-24."""
    return F.relu(_bn(x, sd, p + '.batchnorm'))


def _cam_dense_layer(sd: SD, p: str, x, dilation):
    """CAMDenseTDNNLayer layers.py:113-149 + CAMLayer :70-110 (kernel 3)."""
    h = F.conv1d(_bn_relu(sd, p + '.nonlinear1', x), sd[p + '.linear1.weight'])
    h = _bn_relu(sd, p + '.nonlinear2', h)
    c = p + '.cam_layer'
    y = F.conv1d(h, sd[c + '.linear_local.weight'], padding=dilation, dilation=dilation)
    seg = F.avg_pool1d(h, kernel_size=100, stride=100, ceil_mode=True)
    shape = seg.shape
    seg = seg.unsqueeze(-1).expand(*shape, 100).reshape(*shape[:-1], -1)[..., :h.shape[-1]]
    ctx = h.mean(-1, keepdim=True) + seg
    ctx = F.relu(F.conv1d(ctx, sd[c + '.linear1.weight'], sd[c + '.linear1.bias']))
    m = torch.sigmoid(F.conv1d(ctx, sd[c + '.linear2.weight'], sd[c + '.linear2.bias']))
    return y * m


def _basic_res_block(sd: SD, p: str, x, stride):
    """BasicResBlock layers.py:218-253 (stride on the frequency axis only)."""
    out = F.relu(_bn(F.conv2d(x, sd[p + '.conv1.weight'], stride=(stride, 1), padding=1), sd, p + '.bn1'))
    out = _bn(F.conv2d(out, sd[p + '.conv2.weight'], padding=1), sd, p + '.bn2')
    if (p + '.shortcut.0.weight') in sd:
        out = out + _bn(F.conv2d(x, sd[p + '.shortcut.0.weight'], stride=(stride, 1)), sd, p + '.shortcut.1')
    else:
        out = out + x
    return F.relu(out)


def campplus_forward(sd: SD, x, block_layers=(12, 24, 16), dilations=(1, 2, 2)):
    """CAMPPlus.forward DTDNN.py:111-115 with FCM :39-48. x: [B, T, F]."""
    x = x.permute(0, 2, 1).unsqueeze(1)
    h = 'head'
    out = F.relu(_bn(F.conv2d(x, sd[h + '.conv1.weight'], padding=1), sd, h + '.bn1'))
    for layer in ('layer1', 'layer2'):
        for b in range(2):
            out = _basic_res_block(sd, f'{h}.{layer}.{b}', out, 2 if b == 0 else 1)
    out = F.relu(_bn(F.conv2d(out, sd[h + '.conv2.weight'], stride=(2, 1), padding=1), sd, h + '.bn2'))
    s = out.shape
    x = out.reshape(s[0], s[1] * s[2], s[3])
    xv = 'xvector'
    x = F.conv1d(x, sd[xv + '.tdnn.linear.weight'], stride=2, padding=2)
    x = _bn_relu(sd, xv + '.tdnn.nonlinear', x)
    for bi, (n, d) in enumerate(zip(block_layers, dilations)):
        for li in range(n):
            y = _cam_dense_layer(sd, f'{xv}.block{bi + 1}.tdnnd{li + 1}', x, d)
            x = torch.cat([x, y], 1)
        x = _bn_relu(sd, f'{xv}.transit{bi + 1}.nonlinear', x)
        x = F.conv1d(x, sd[f'{xv}.transit{bi + 1}.linear.weight'])
    x = _bn_relu(sd, xv + '.out_nonlinear', x)
    stats = torch.cat([x.mean(dim=-1), x.std(dim=-1, unbiased=True)], -1)
    x = F.conv1d(stats.unsqueeze(-1), sd[xv + '.dense.linear.weight']).squeeze(-1)
    return _bn(x, sd, xv + '.dense.nonlinear.batchnorm')


# ----------------------------------------------------------------------------- registry
ARCHS = {
    # name: (forward, reference ctor kwargs used by the registry in infer_sv_batch.py:46-120)
    'eres2netv2': (eres2netv2_forward, dict(feat_dim=80, embedding_size=192)),
    'eres2net_large': (lambda sd, x: eres2net_forward(sd, x, m_channels=64),
                       dict(feat_dim=80, embedding_size=192, m_channels=64)),
    'ecapa': (ecapa_forward, dict(input_size=80, lin_neurons=192, channels=[1024, 1024, 1024, 1024, 3072])),
    'campplus': (campplus_forward, dict(feat_dim=80, embedding_size=512)),
    'eres2net_huge': (lambda sd, x: eres2net_forward(sd, x, m_channels=64, base_width=24, scale=3),
                      dict(feat_dim=80, embedding_size=192)),
    'eres2netv2_w24s4ep4': (lambda sd, x: eres2netv2_forward(sd, x, base_width=24, scale=4),
                            dict(feat_dim=80, embedding_size=192, baseWidth=24, scale=4, expansion=4)),
    'campplus_192': (campplus_forward, dict(feat_dim=80, embedding_size=192)),
    'eres2net_base': (lambda sd, x: eres2net_forward(sd, x, m_channels=32), dict(feat_dim=80, embedding_size=512,
                                                                                  m_channels=32)),
    'resnet34': (resnet_forward, dict(feat_dim=80, embedding_size=192)),
    'res2net': (res2net_forward, dict(feat_dim=80, embedding_size=192)),
}


def forward(arch: str, sd: SD, feats: torch.Tensor) -> torch.Tensor:
    with torch.no_grad():
        return ARCHS[arch][0](sd, feats)
