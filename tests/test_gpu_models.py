"""GPU parity: the HIP embedding forward (through the C ABI) vs the reference's golden
embeddings and vs the CPU oracle.  Tolerance (BASELINE.json north_star): per-embedding
relative L2 error <= 1e-4 in fp32."""
import numpy as np
import pytest
import torch

import helpers
from oracle import models_ref

pytestmark = pytest.mark.gpu
TOL = 1e-4
GPU_ARCHS = helpers.ARCHS + helpers.VARIANTS

_cache = {}


def gpu_module(arch):
    if arch not in _cache:
        _cache[arch] = helpers.loaded_module(arch).to('cuda')
    return _cache[arch]


@pytest.mark.parametrize('arch', GPU_ARCHS)
def test_golden_embeddings(arch):
    g = helpers.golden(arch)
    m = gpu_module(arch)
    for i in range(3):
        with torch.no_grad():
            emb = m(torch.from_numpy(g[f'feats{i}']).cuda()).cpu().numpy()
        assert emb.shape == g[f'emb32_{i}'].shape
        e64 = helpers.rel_err(emb, g[f'emb64_{i}']).max()
        e32 = helpers.rel_err(emb, g[f'emb32_{i}']).max()
        # variants with a reference fp32-vs-fp64 floor above the bar (w24s4ep4: 5e-4 with
        # random weights) are held to 2x that floor; the four north-star models to 1e-4
        tol = max(TOL, 2 * helpers.rel_err(g[f'emb32_{i}'], g[f'emb64_{i}']).max())
        print(f'{arch} set{i}: rel err vs fp64 {e64:.2e}, vs reference fp32 {e32:.2e} (tol {tol:.1e})')
        assert e64 < tol and e32 < tol, (arch, i, e64, e32)


@pytest.mark.parametrize('arch', helpers.ARCHS)
@pytest.mark.parametrize('B,T', [(1, 57), (5, 101), (33, 198)])
def test_ragged_shapes_vs_oracle(arch, B, T):
    torch.manual_seed(B * 1000 + T)
    x = torch.randn(B, T, 80) * 2.0
    sd = helpers.state_dict(arch)
    ref = models_ref.forward(arch, sd, x).numpy()
    with torch.no_grad():
        emb = gpu_module(arch)(x.cuda()).cpu().numpy()
    err = helpers.rel_err(emb, ref).max()
    assert err < TOL, (arch, B, T, err)


def test_batch_independence_eres2netv2():
    """Row i of a batched forward equals the single-utterance forward (no cross-talk)."""
    g = helpers.golden('eres2netv2')
    m = gpu_module('eres2netv2')
    x = torch.from_numpy(g['feats0']).cuda()
    with torch.no_grad():
        full = m(x).cpu().numpy()
        single = np.concatenate([m(x[i:i + 1]).cpu().numpy() for i in range(x.shape[0])])
    # different M picks different tiles / K-steps (fp32 summation order): ~1e-5 noise;
    # cross-talk between utterances would be O(1)
    assert helpers.rel_err(full, single).max() < 5e-5


def test_weight_reload_invalidates_native_handle():
    m = helpers.loaded_module('eres2netv2').to('cuda')
    x = torch.from_numpy(helpers.golden('eres2netv2')['feats2']).cuda()
    with torch.no_grad():
        a = m(x).cpu().numpy()
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        sd['seg_1.bias'] += 1.0
        m.load_state_dict(sd)
        b = m(x).cpu().numpy()
    np.testing.assert_allclose(b - a, 1.0, atol=1e-4)
