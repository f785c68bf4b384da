"""Executor plan logic on the host (tests/emu): the real C++ plan builder + weight packing
with emulated kernels must reproduce the oracle.  Catches layout / folding / aliasing bugs
without a GPU; the GPU tests then only have to validate the kernels."""
import numpy as np
import pytest
import torch

import helpers
from emu_runner import EmuModel
from oracle import models_ref

EMU_ARCHS = helpers.ARCHS + helpers.VARIANTS


@pytest.mark.parametrize('arch', EMU_ARCHS)
def test_emulated_plan_matches_oracle(arch):
    g = helpers.golden(arch)
    m = helpers.loaded_module(arch)
    feats = torch.from_numpy(g['feats2'][:1])          # 1 x 98 frames keeps the loops quick
    ref = g['emb64_2'][:1]
    emb = EmuModel(m)(feats).numpy()
    floor = helpers.rel_err(g['emb32_2'][:1], ref).max()     # the reference's own fp32 noise
    assert helpers.rel_err(emb, ref).max() < max(1e-4, 2 * floor)


@pytest.mark.parametrize('arch,gflop', [('eres2netv2', 16.533), ('eres2net_large', 26.747)])
def test_algorithmic_flops_match_survey(arch, gflop):
    """FLOPs per 2 s utterance = 2 x conv/linear MACs (forward hooks)."""
    fl = EmuModel(helpers.loaded_module(arch)).flops(198)
    assert abs(fl / 1e9 - gflop) / gflop < 2e-3, fl


def test_ecapa_flops_match_survey():
    fl = EmuModel(helpers.loaded_module('ecapa')).flops(198)
    assert abs(fl / 1e9 - 7.426) / 7.426 < 2e-3, fl


def test_campplus_flops_match_survey():
    """CAM++(512) = 1.115 GMAC per 2 s utterance."""
    fl = EmuModel(helpers.loaded_module('campplus')).flops(198)
    assert abs(fl / 2e9 - 1.115) / 1.115 < 5e-3, fl


@pytest.mark.parametrize('arch', helpers.ARCHS)
def test_flops_attributed_per_step(arch):
    """Per-step FLOPs (used for the per-kernel roofline) add up to the model total and land
    on the GEMM / conv launch that performs them."""
    em = EmuModel(helpers.loaded_module(arch))
    steps = em.plan(2, 198)
    total = sum(f for _, f, _ in steps)
    assert abs(total - 2 * em.flops(198)) / total < 1e-9
    for name, f, kern in steps:
        if kern.startswith(('conv_gemm', 'conv3x3')):
            assert f > 0, (name, kern)


@pytest.mark.parametrize('arch', ['campplus', 'campplus_192'])
def test_emulated_ragged_campplus_matches_per_utterance(arch):
    """Variable-length batch (config C3): row b of a padded batch with lengths[b] valid
    frames equals the reference forward of that utterance alone; the padding frames hold
    garbage that must not leak in."""
    g = helpers.golden(arch)
    m = helpers.loaded_module(arch)
    sd = helpers.state_dict(arch, torch.float64)
    full = torch.from_numpy(g['feats0'][:3]).float()            # 3 x 198 frames
    lengths = [198, 120, 161]
    feats = full.clone()
    gen = torch.Generator().manual_seed(0)
    for b, n in enumerate(lengths):
        feats[b, n:] = 50 * torch.randn(198 - n, full.shape[2], generator=gen)
    emb = EmuModel(m)(feats, lengths).numpy()
    for b, n in enumerate(lengths):
        ref = models_ref.forward(arch, sd, full[b:b + 1, :n].double()).numpy()
        assert helpers.rel_err(emb[b:b + 1], ref).max() < 1e-5, (b, n)


def test_step_bytes_priced_per_conv():
    """Per-step algorithmic bytes (the byte side of bench.py's per-launch roofline): every
    conv step is priced; ERes2NetV2 layer3.1.conv3 (1x1, 208 -> 512 channels, residual) is
    exactly input + weights + output + residual, fp32, and the fused blocks layer1.1.fused /
    layer1.0.fused / layer2.1.fused are their input + output + the packed weight matrices."""
    m = helpers.loaded_module('eres2netv2')
    em = EmuModel(m)
    B, T = 2, 40
    steps = em.plan(B, T)
    nbytes = em.plan_bytes(B, T)
    assert len(nbytes) == len(steps)
    for (name, _, kern), by in zip(steps, nbytes):
        if kern.startswith(('conv_gemm', 'conv3x3', 'pw_gemm')):
            assert by > 0, name
    names = [name for name, _, _ in steps]
    px3 = B * 20 * (T // 4)
    assert nbytes[names.index("layer3.1.conv3")] == 4.0 * (px3 * 208 + 512 * 208 + px3 * 512 + px3 * 512)
    # the stage-2 blocks run unfused (four kernels measured faster than a fused stage-2 kernel,
    # DESIGN.md §7 round 4): conv3 (1x1, 104 -> 256, residual) priced like layer3's
    px2 = B * 40 * (T // 2)
    assert 'layer2.1.fused' not in names
    assert nbytes[names.index('layer2.1.conv3')] == 4.0 * (px2 * 104 + 256 * 104 + px2 * 256 + px2 * 256)
    px = B * 80 * T
    w = 64 * 128 + 2 * 32 * 288 + 128 * 64
    assert nbytes[names.index('layer1.1.fused')] == 8.0 * px * 128 + 4.0 * w
    # layer1.0 (64 -> 128, projection shortcut K-concatenated with conv3) is fused as well
    w0 = 64 * 64 + 2 * 32 * 288 + 128 * 128
    assert nbytes[names.index('layer1.0.fused')] == 4.0 * px * (64 + 128) + 4.0 * w0
    assert not any(n.startswith('layer1.') and not n.endswith('.fused') for n in names)


def test_emulated_plans_with_channel_block_k_order():
    """ConvDesc::kcb (SPK_KCB=1, read once per process): the permuted weight packing and the
    emulated loader order must still reproduce the oracle; a child process gets the flag."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, SPK_KCB='1')
    r = subprocess.run([sys.executable, '-m', 'pytest', '-q', '-x', '-p', 'no:cacheprovider',
                        os.path.join(here, 'test_emu_plans.py'), '-k',
                        'test_emulated_plan_matches_oracle and (eres2netv2 or ecapa or resnet34)'],
                       env=env, cwd=os.path.dirname(here), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
