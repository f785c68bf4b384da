"""Numerics of the fp16x3 split-precision MFMA scheme (conv_gemm.hip), emulated on the CPU:
every conv / linear operand x -> hi = fp16(x), lo = fp16((x - hi) * 2^11), product
hi*hi + 2^-11 (hi*lo + lo*hi) in fp64.  The resulting embeddings must be at least as close to
the reference's fp64 forward as the reference's own fp32 forward is (tests/golden)."""
import pytest
import torch
import torch.nn.functional as F

import helpers
from oracle import models_ref

S = 2.0 ** 11


def _split(t):
    hi = t.to(torch.float16).to(t.dtype)
    lo = ((t - hi) * S).to(torch.float16).to(t.dtype)
    return hi, lo


def _x3(fn, name):
    def g(x, w, b=None, *a, **k):
        xh, xl = _split(x)
        wh, wl = _split(w)
        y = fn(xh, wh, None, *a, **k) + (fn(xh, wl, None, *a, **k) + fn(xl, wh, None, *a, **k)) / S
        if b is not None:
            y = y + (b if name == 'linear' else b.view(1, -1, *([1] * (y.dim() - 2))))
        return y
    return g


@pytest.mark.parametrize('arch', ['eres2netv2', 'campplus', 'ecapa'])
def test_fp16x3_within_reference_fp32_noise(arch, monkeypatch):
    g = helpers.golden(arch)
    sd = helpers.state_dict(arch, torch.float64)
    for name in ('conv1d', 'conv2d', 'linear'):
        monkeypatch.setattr(F, name, _x3(getattr(F, name), name))
    emb = models_ref.forward(arch, sd, torch.from_numpy(g['feats2']).double()).numpy()
    err = helpers.rel_err(emb, g['emb64_2']).max()
    floor = helpers.rel_err(g['emb32_2'], g['emb64_2']).max()
    assert err < max(floor, 2e-6), (err, floor)
