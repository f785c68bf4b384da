"""Pin the CPU oracle (oracle/models_ref.py) against golden embeddings produced by the
reference modules themselves (tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

import helpers
from oracle import models_ref


@pytest.mark.parametrize('arch', helpers.ARCHS + helpers.VARIANTS)
def test_oracle_matches_reference_fp32(arch):
    g = helpers.golden(arch)
    sd = helpers.state_dict(arch)
    for i in range(3):
        emb = models_ref.forward(arch, sd, torch.from_numpy(g[f'feats{i}'])).numpy()
        # same op sequence in fp32: only summation-order noise
        # same op sequence in fp32: only summation-order noise (x reference conditioning)
        floor = helpers.rel_err(g[f'emb32_{i}'], g[f'emb64_{i}']).max()
        assert helpers.rel_err(emb, g[f'emb32_{i}']).max() < max(2e-6, 0.2 * floor), (arch, i)


@pytest.mark.parametrize('arch', ['eres2netv2', 'campplus'])
def test_oracle_matches_reference_fp64(arch):
    g = helpers.golden(arch)
    sd = helpers.state_dict(arch, torch.float64)
    emb = models_ref.forward(arch, sd, torch.from_numpy(g['feats2']).double()).numpy()
    assert helpers.rel_err(emb, g['emb64_2']).max() < 1e-12


def test_oracle_ecapa_lengths_matches_reference():
    """forward(x, lengths): masked SE / ASP statistics (ECAPA_TDNN.py:209-287), pinned by
    tests/golden/make_ecapa_lengths_golden.py (reference module output)."""
    g = dict(np.load(helpers.os.path.join(helpers.GOLDEN, 'ecapa_lengths_golden.npz')))
    lens = torch.from_numpy(g['lengths'])
    with torch.no_grad():
        e32 = models_ref.ecapa_forward(helpers.state_dict('ecapa'), torch.from_numpy(g['feats']), lengths=lens)
        e64 = models_ref.ecapa_forward(helpers.state_dict('ecapa', torch.float64),
                                       torch.from_numpy(g['feats']).double(), lengths=lens)
    assert helpers.rel_err(e32.numpy(), g['emb32']).max() < 2e-6
    assert helpers.rel_err(e64.numpy(), g['emb64']).max() < 1e-12
