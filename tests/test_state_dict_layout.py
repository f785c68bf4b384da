"""Drop-in boundary: this package's modules expose exactly the reference state_dict layout
(strict load_state_dict of reference checkpoints, infer_sv_batch.py:249-252), at the same
dotted paths the registries import (infer_sv_batch.py:46-120)."""
import importlib

import pytest

import helpers


@pytest.mark.parametrize('arch', helpers.ARCHS + helpers.VARIANTS)
def test_keys_and_shapes_match_reference(arch):
    ref = helpers.ref_keys(arch)
    mine = {k: list(v.shape) for k, v in helpers.product_module(arch).state_dict().items()}
    assert set(mine) == set(ref), (set(mine) ^ set(ref))
    for k in ref:
        assert mine[k] == ref[k], k


@pytest.mark.parametrize('dotted', [
    'speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2',
    'speakerlab.models.eres2net.ERes2Net.ERes2Net',
    'speakerlab.models.ecapa_tdnn.ECAPA_TDNN.ECAPA_TDNN',
    'speakerlab.models.campplus.DTDNN.CAMPPlus',
    'speakerlab.models.eres2net.ERes2Net_huge.ERes2Net',
])
def test_registry_dotted_paths_import(dotted):
    mod, _, cls = dotted.rpartition('.')
    assert hasattr(importlib.import_module(mod), cls)


@pytest.mark.parametrize('arch', helpers.ARCHS)
def test_strict_load_of_reference_layout(arch):
    import torch
    m = helpers.product_module(arch)
    sd = {k: torch.zeros(v) if k.split('.')[-1] != 'num_batches_tracked' else torch.tensor(0)
          for k, v in helpers.ref_keys(arch).items()}
    m.load_state_dict(sd, strict=True)


def test_cpu_forward_refuses_without_device():
    """The product path has no CPU fallback: a CPU tensor must raise, not silently compute."""
    import torch
    from speakerlab._hip import HipError
    m = helpers.product_module('eres2netv2').eval()
    with pytest.raises(HipError):
        m(torch.zeros(1, 98, 80))
