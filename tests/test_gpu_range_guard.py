"""fp16x3 range guard on the GPU (include/spk_hip.h): models whose activations leave the
range the split-precision GEMMs represent (ECAPA / CAM++ have unbounded ReLU -> BN outputs,
ECAPA_TDNN.py:127-151, layers.py:40-67) still match the fp64 reference forward within the
north-star 1e-4, because the flagged forward is re-run on the exact-fp32 kernels; the fp16x3
result alone would not (the saturation the guard exists for)."""
import ctypes

import numpy as np
import pytest
import torch

import helpers
from oracle import models_ref
from speakerlab import _hip

pytestmark = pytest.mark.gpu


def _scaled(arch, key, factor):
    m = helpers.loaded_module(arch)
    m.state_dict()[key].mul_(factor)
    return m



@pytest.mark.parametrize('arch,key,factor', [('ecapa', 'blocks.0.norm.norm.weight', 1e5),
                                             ('campplus', 'head.layer1.0.bn2.weight', 3e4)])
def test_out_of_range_activations_take_exact_path(arch, key, factor):
    g = helpers.golden(arch)
    m = _scaled(arch, key, factor)
    feats = torch.from_numpy(g['feats2'][:3])
    sd = {k: v.double() if v.is_floating_point() else v for k, v in m.state_dict().items()}
    ref = models_ref.forward(arch, sd, feats.double()).numpy()
    dev = torch.device('cuda', 0)
    m = m.to(dev)
    with torch.no_grad():
        out = m(feats.to(dev)).cpu().numpy()
    h = m._hip_handle(dev)
    assert h.last_forward_exact
    assert helpers.rel_err(out, ref).max() < 1e-4
    # the split-precision forward alone saturates: far off the reference
    B, T, _ = feats.shape
    x = feats.to(dev).contiguous()
    raw = torch.empty(B, h.embed_dim, device=dev)
    ws = torch.empty(h.workspace_bytes(B, T), dtype=torch.uint8, device=dev)
    _hip._check(_hip.lib().spk_model_forward(h.handle, x.data_ptr(), B, T, ws.data_ptr(), ws.numel(),
                                             raw.data_ptr(), _hip._stream(dev)), 'forward')
    flag = ctypes.c_int32(0)
    _hip._check(_hip.lib().spk_model_range_check(h.handle, _hip._stream(dev), ctypes.byref(flag)), 'check')
    assert flag.value == 1
    assert helpers.rel_err(raw.cpu().numpy(), ref).max() > 1e-3


def test_in_range_model_stays_on_split_path():
    g = helpers.golden('ecapa')
    dev = torch.device('cuda', 0)
    m = helpers.loaded_module('ecapa').to(dev)
    with torch.no_grad():
        m(torch.from_numpy(g['feats2'][:2]).to(dev))
    assert not m._hip_handle(dev).last_forward_exact
