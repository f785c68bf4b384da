"""fp16x3 range guard plumbing on the host emulation (tests/emu): a model whose activations
reach 2^15 raises the handle's flag (spk_model_range_check reports and clears it), the exact
plan (spk_model_forward_exact) reproduces the oracle, and weights past fp16's range force the
exact path at creation.  The GPU test (tests/test_gpu_range_guard.py) checks the kernels."""
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
    v = ctypes.c_int32(-1)
    _check(lib().spk_model_range_check(em.handle, None, ctypes.byref(v)), 'range_check')
    return v.value


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
    em(feats)
    assert _flag(em) == 1
    assert _flag(em) == 0                                       # cleared by the check
    out = _forward_exact(em, feats).numpy()
    ref = models_ref.forward('ecapa', {k: v.double() if v.is_floating_point() else v
                                       for k, v in m.state_dict().items()}, feats.double()).numpy()
    assert helpers.rel_err(out, ref).max() < 1e-4
    assert _flag(em) == 0                                       # the exact plan does not flag


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
