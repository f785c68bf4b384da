"""fp16x3 range guard plumbing on the host emulation (tests/emu): a model whose activations
reach the range limit raises the forward's range word (a workspace slot), the forward still
reproduces the oracle (ERes2Net: the gated exact twin of the flagged segment recomputes it;
ECAPA / CAM++: the split GEMMs scale their operands by the word -- the emulated GEMMs are
exact, so here only the plumbing is checked), the word belongs to its workspace (two interleaved forwards with two
workspaces do not see each other's), spk_model_forward_exact runs the exact plan alone, and
weights past fp16's range force the exact path at creation.  The GPU test
(tests/test_gpu_range_guard.py) checks the kernels."""
import ctypes

import numpy as np
import torch

import helpers
from emu_runner import EmuModel, lib, _check
from oracle import models_ref


def _scaled(arch, key, factor):
    m = helpers.loaded_module(arch)
    sd = m.state_dict()
    sd[key].mul_(factor)
    return m


def _flag(em):
    return em.range_word()


def _forward_exact(em, feats):
    B, T, _ = feats.shape
    n = ctypes.c_size_t()
    _check(lib().spk_model_workspace_bytes(em.handle, B, T, ctypes.byref(n)), 'workspace')
    ws = torch.zeros(max(n.value, 256), dtype=torch.uint8)
    out = torch.empty(B, em.embed_dim)
    _check(lib().spk_model_forward_exact(em.handle, feats.data_ptr(), B, T, None, ws.data_ptr(), ws.numel(),
                                         out.data_ptr(), None), 'forward_exact')
    return out


def test_flag_stays_clear_in_range():
    g = helpers.golden('ecapa')
    em = EmuModel(helpers.loaded_module('ecapa'))
    em(torch.from_numpy(g['feats2'][:1]))
    assert _flag(em) == 0


def test_large_activations_flag_and_exact_path():
    g = helpers.golden('ecapa')
    m = _scaled('ecapa', 'blocks.0.norm.norm.weight', 1e5)     # post-ReLU BN: activations ~1e5
    feats = torch.from_numpy(g['feats2'][:1])
    em = EmuModel(m)
    guarded = em(feats).numpy()
    assert _flag(em) == 1
    assert _flag(em) == 1                                       # reading does not clear it
    ref = models_ref.forward('ecapa', {k: v.double() if v.is_floating_point() else v
                                       for k, v in m.state_dict().items()}, feats.double()).numpy()
    assert helpers.rel_err(guarded, ref).max() < 1e-4
    out = _forward_exact(em, feats).numpy()
    assert helpers.rel_err(out, ref).max() < 1e-4


def test_range_word_is_per_workspace():
    """Two forwards interleaved with their own workspaces: only the overflowing one is
    re-run, and a later clean forward on a workspace clears that workspace's word."""
    g = helpers.golden('campplus')
    m = helpers.loaded_module('campplus')
    em = EmuModel(m)
    clean = torch.from_numpy(g['feats2'][:1]).clone()
    hot = clean.clone()
    hot[0, 3, 5] = 40000.0
    B, T, _ = clean.shape
    n = ctypes.c_size_t()
    _check(lib().spk_model_workspace_bytes(em.handle, B, T, ctypes.byref(n)), 'workspace')
    wa, wb = (torch.zeros(n.value, dtype=torch.uint8) for _ in range(2))
    sd = {k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    oa = em(hot, ws=wa).numpy()
    ob = em(clean, ws=wb).numpy()
    assert em.range_word((B, T, 0, wa)) == 1 and em.range_word((B, T, 0, wb)) == 0
    assert helpers.rel_err(oa, models_ref.forward('campplus', sd, hot.double()).numpy()).max() < 1e-4
    assert helpers.rel_err(ob, models_ref.forward('campplus', sd, clean.double()).numpy()).max() < 1e-4
    em(clean, ws=wa)
    assert em.range_word((B, T, 0, wa)) == 0


def test_large_input_flags():
    g = helpers.golden('campplus')
    em = EmuModel(helpers.loaded_module('campplus'))
    feats = torch.from_numpy(g['feats2'][:1]).clone()
    feats[0, 3, 5] = 40000.0
    em(feats)
    assert _flag(em) == 1


def test_weights_out_of_fp16_range_force_exact():
    g = helpers.golden('ecapa')
    m = _scaled('ecapa', 'blocks.1.tdnn1.conv.conv.weight', 1e6)   # packed weights past 65504
    feats = torch.from_numpy(g['feats2'][:1])
    em = EmuModel(m)
    out = em(feats).numpy()
    assert _flag(em) == 0                                        # exact plan: nothing to flag
    ref = models_ref.forward('ecapa', {k: v.double() if v.is_floating_point() else v
                                       for k, v in m.state_dict().items()}, feats.double()).numpy()
    assert helpers.rel_err(out, ref).max() < 1e-4
    steps = em.plan(1, feats.shape[1])
    assert not any(s[0] == 'range_in' for s in steps)           # the exact plan has no input check


def _guard_plan(em, B, T, ragged=0):
    v = [ctypes.c_int32(-1) for _ in range(3)]
    _check(lib().spk_model_guard_plan(em.handle, B, T, ragged, *[ctypes.byref(x) for x in v]), 'guard_plan')
    return [x.value for x in v]


def test_eres2net_guard_segments_only_the_stem_segment_is_twinned():
    """ERes2NetV2: every split-GEMM operand past the stem is bounded statically (Hardtanh(0, 20)
    block outputs, |AFF| <= 2 max(|x|, |y|), weight-norm bounds of the downsample / AFF / seg
    layers), so of the plan's segments (one per block, plus the tail) only the first -- the
    stem and layer1.0, which read the unbounded stem output -- and, where the weight-norm
    bound of fuse34's hidden layer (here 34.8 x 1130) passes 2^14, the tail get a gated
    exact twin: about a dozen no-op launches behind a forward instead of the ~60-step plan."""
    em = EmuModel(helpers.loaded_module('eres2netv2'))
    nseg, ntwin, ngated = _guard_plan(em, 2, 40)
    assert nseg == 3 + 4 + 6 + 3 + 1
    assert 1 <= ntwin <= 2
    assert 0 < ngated <= 14


def test_eres2net_hot_input_reruns_the_stem_segment():
    """An input value that drives the stem output past the range limit sets the word; the
    first segment's exact twin recomputes stem + layer1.0 before layer1.1 reads its output,
    and the embeddings match the fp64 reference."""
    g = helpers.golden('eres2netv2')
    m = helpers.loaded_module('eres2netv2')
    feats = torch.from_numpy(g['feats2'][:1, :40]).clone()
    feats[0, 7, 11] = 3.0e6
    em = EmuModel(m)
    out = em(feats).numpy()
    assert _flag(em) == 1
    sd = {k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    ref = models_ref.forward('eres2netv2', sd, feats.double()).numpy()
    assert helpers.rel_err(out, ref).max() < 1e-4


def test_unbounded_models_scale_instead_of_twin():
    """ECAPA / CAM++ activations are unbounded (ReLU -> BN): their split GEMMs scale the operand
    by the range word (common.h scaled split), so nothing is gated behind the plan."""
    for arch in ('ecapa', 'campplus'):
        em = EmuModel(helpers.loaded_module(arch))
        nseg, ntwin, ngated = _guard_plan(em, 1, 40)
        assert nseg == 1 and ntwin == 0 and ngated == 0
