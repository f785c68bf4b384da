"""ERes2NetV2 pooling heads TAP / TSDP / ASTP (pooling_layers.py:10-35, 58-104,
ERes2NetV2.py:215-217): the oracle vs reference-generated goldens on the CPU
(tests/golden/make_pooling_golden.py), the executor's plan on the host emulation, the HIP
forward vs the same goldens on the GPU (1e-4), and ASTP's global-context form refused."""
import os

import numpy as np
import pytest
import torch

import helpers
from oracle import models_ref

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'eres2netv2_pool_golden.npz')


def _module(pool):
    from speakerlab.models.eres2net.ERes2NetV2 import ERes2NetV2
    from speakerlab.utils import synthetic
    m = ERes2NetV2(feat_dim=80, embedding_size=192, pooling_func=pool)
    synthetic.load_synthetic_weights(m, seed=0, bn_stats=helpers.bn_stats('eres2netv2'))
    return m.eval()


@pytest.mark.parametrize('pool', ['TAP', 'TSDP', 'ASTP'])
def test_oracle_matches_reference_golden(pool):
    g = np.load(G)
    m = _module(pool)
    sd = {k: v.double() for k, v in m.state_dict().items()}
    with torch.no_grad():
        emb = models_ref.eres2netv2_forward(sd, torch.from_numpy(g['feats']).double(), pooling=pool).numpy()
    assert helpers.rel_err(emb, g[f'emb64_{pool}']).max() < 1e-10


def test_layouts_and_astp():
    from speakerlab.models.eres2net import pooling_layers
    assert _module('TAP').seg_1.in_features == 10 * 1024
    assert _module('TSTP').seg_1.in_features == 2 * 10 * 1024
    a = _module('ASTP')
    assert a.seg_1.in_features == 2 * 10 * 1024
    assert tuple(a.pool.linear1.weight.shape) == (128, 10 * 1024, 1)
    assert tuple(a.pool.linear2.weight.shape) == (10 * 1024, 128, 1)
    with pytest.raises(NotImplementedError):
        pooling_layers.ASTP(in_dim=10240, global_context_att=True)


def test_emulated_plan_astp():
    """The executor's ASTP steps (frequency-tall linear1 conv, permuted linear2, pooling
    kernel contract) on the host emulation vs the reference's fp64 golden."""
    from emu_runner import EmuModel
    g = np.load(G)
    emb = EmuModel(_module('ASTP'))(torch.from_numpy(g['feats'])).numpy()
    assert helpers.rel_err(emb, g['emb64_ASTP']).max() < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize('pool', ['TAP', 'TSDP', 'ASTP'])
def test_gpu_pooling_heads(pool):
    g = np.load(G)
    m = _module(pool).to('cuda')
    with torch.no_grad():
        emb = m(torch.from_numpy(g['feats']).cuda()).cpu().numpy()
    e64 = helpers.rel_err(emb, g[f'emb64_{pool}']).max()
    e32 = helpers.rel_err(emb, g[f'emb32_{pool}']).max()
    print(f'{pool}: rel err vs fp64 {e64:.2e}, vs reference fp32 {e32:.2e}')
    assert e64 < 1e-4 and e32 < 1e-4
