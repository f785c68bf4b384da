"""Scaled split behind an amplifying operand loader.

CAM++'s dense layers and transits apply their BN-ReLU pre-activation (`nonlinear1`,
layers.py:113-149; the transits' `nonlinear`, layers.py:183-196) inside the GEMM's operand
loader, after the producer of x noted its largest output in the range word.  relu(psc x + psh)
can exceed the 2x growth bound the word assumes, by up to P = max_c max(|psc|, |psh| / 2^14), so
those GEMMs scale their operand by a further 2^-b with P <= 1.3 * 2^b (common.h,
runtime.cpp pre_range_bits): the affine is packed times 2^-b and the GEMM's weights times 2^b
(the products unchanged), so no kernel sees the bits.  The construction below (TDNN output BN scaled, block1.tdnnd1's
nonlinear1 running_var shrunk to 1e-2, so psc ~ 12) drives the scaled operand past fp16's
65504 under the word-only scale, both with the word clear (activations just below 2^14) and
set; the CPU test pins that arithmetic, the GPU test the forward against fp64."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import helpers
from oracle import models_ref as R

RANGE_LIMIT = 2.0 ** 14
TDNN_BN = 'xvector.tdnn.nonlinear.batchnorm.weight'
PRE_BN = 'xvector.block1.tdnnd1.nonlinear1.batchnorm'


def _hot_state(factor, dtype=torch.float64):
    m = helpers.loaded_module('campplus')
    sd = m.state_dict()
    sd[TDNN_BN].mul_(factor)
    sd[PRE_BN + '.running_var'].fill_(1e-2)
    return m, {k: v.to(dtype) if v.is_floating_point() else v for k, v in sd.items()}


def _pre_range_bits(P):
    """runtime.cpp pre_range_bits: smallest b >= 0 with P <= 1.3 * 2^b."""
    b = 0
    while P > 1.3 * 2.0 ** b:
        b += 1
    return b


def _word_scale_exp(word):
    """common.h range_scale without the extra bits: s with word * 2^-s in [2^13, 2^14)."""
    return int(np.floor(np.log2(word))) - 13 if word >= RANGE_LIMIT else 0


def _block1_operand(sd, feats):
    """The largest activation written before block1.tdnnd1.linear1 and that GEMM's operand
    relu(BN(x)) (DTDNN.py:39-48, 111-115 up to the first dense layer)."""
    x = feats.permute(0, 2, 1).unsqueeze(1)
    out = F.relu(R._bn(F.conv2d(x, sd['head.conv1.weight'], padding=1), sd, 'head.bn1'))
    word = out.abs().max().item()
    for layer in ('layer1', 'layer2'):
        for b in range(2):
            out = R._basic_res_block(sd, f'head.{layer}.{b}', out, 2 if b == 0 else 1)
            word = max(word, out.abs().max().item())
    out = F.relu(R._bn(F.conv2d(out, sd['head.conv2.weight'], stride=(2, 1), padding=1), sd, 'head.bn2'))
    s = out.shape
    x = F.conv1d(out.reshape(s[0], s[1] * s[2], s[3]), sd['xvector.tdnn.linear.weight'], stride=2, padding=2)
    x = R._bn_relu(sd, 'xvector.tdnn.nonlinear', x)
    word = max(word, x.abs().max().item())
    return word, R._bn_relu(sd, 'xvector.block1.tdnnd1.nonlinear1', x)


@pytest.mark.parametrize('factor', [3e3, 1e4])
def test_construction_overflows_the_word_only_scale(factor):
    _, sd = _hot_state(factor)
    feats = torch.from_numpy(helpers.golden('campplus')['feats2'][:3]).double()
    word, operand = _block1_operand(sd, feats)
    g = sd[PRE_BN + '.weight']
    psc = g / torch.sqrt(sd[PRE_BN + '.running_var'] + 1e-5)
    psh = sd[PRE_BN + '.bias'] - sd[PRE_BN + '.running_mean'] * psc
    P = max(psc.abs().max().item(), psh.abs().max().item() / RANGE_LIMIT)
    amax = operand.abs().max().item()
    s = _word_scale_exp(word)
    assert amax * 2.0 ** -s > 65504            # the round-5 scale saturates this operand
    b = _pre_range_bits(P)
    assert b >= 3
    assert amax * 2.0 ** -(s + b) < 1.95 * 2.0 ** 15   # the pre-activation bits bring it back in range (common.h)
    if factor == 3e3:
        assert word < RANGE_LIMIT               # ... even with the word clear (sc = 1 before)


@pytest.mark.gpu
@pytest.mark.parametrize('factor', [3e3, 1e4])
def test_hot_preactivation_matches_fp64(factor):
    m, sd = _hot_state(factor)
    feats = torch.from_numpy(helpers.golden('campplus')['feats2'][:3])
    ref = R.forward('campplus', sd, feats.double()).numpy()
    # the construction is ill-conditioned: bound by the reference's own fp32 error as well
    ref32 = R.forward('campplus', {k: v.float() if v.is_floating_point() else v for k, v in sd.items()},
                      feats).numpy()
    tol = max(1e-4, 1.5 * helpers.rel_err(ref32, ref).max())
    dev = torch.device('cuda', 0)
    m = m.to(dev)
    with torch.no_grad():
        out = m(feats.to(dev)).cpu().numpy()
    h = m._hip_handle(dev)
    assert not h.last_forward_exact
    assert np.isfinite(out).all()
    err = helpers.rel_err(out, ref).max()
    assert err < tol, (err, tol)


def test_emulated_forward_with_folded_pre_bits():
    """The host emulation (tests/emu) runs the real plan builder and packing: the 2^-b folded
    into block1's packed BN-ReLU affine and the 2^b folded into its weights must cancel, so the
    emulated forward (exact GEMMs) reproduces fp64 like the unmodified model does."""
    from emu_runner import EmuModel
    m, sd = _hot_state(3e3)
    feats = torch.from_numpy(helpers.golden('campplus')['feats2'][:1])
    ref = R.forward('campplus', sd, feats.double()).numpy()
    ref32 = R.forward('campplus', {k: v.float() if v.is_floating_point() else v for k, v in sd.items()},
                      feats).numpy()
    tol = max(1e-4, 1.5 * helpers.rel_err(ref32, ref).max())
    out = EmuModel(m)(feats).numpy()
    assert np.isfinite(out).all()
    assert helpers.rel_err(out, ref).max() < tol
