"""Config C3 at its configured size (BASELINE.json configs[2]): 1,024 variable-length 1-5 s
utterances through GPU Fbank and the ragged CAM++ forward, bucketed by length exactly as
tools/bench_workloads.py times it.  Rows at the shortest and longest utterance and at every
bucket edge are checked against the per-utterance fp64 oracle (oracle/fbank_ref.py +
oracle/models_ref.py, the same wav alone): the fp16x3 default at the north-star 1e-4, the
reduced-precision single-product mode (C3's bf16-class setting) at cosine >= 0.9999."""
import os
import sys

import numpy as np
import pytest
import torch

import helpers
from oracle import fbank_ref, models_ref

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))


@pytest.fixture(scope='module')
def c3_run():
    import bench_workloads
    dev = torch.device('cuda', 0)
    step, lens, order, host, model = bench_workloads.c3_setup(dev, 'fp32', 4)
    n = len(lens)
    edges = sorted({0, n - 1} | {e for b in np.linspace(0, n, 5).astype(int)[1:-1] for e in (b - 1, b)})
    sd = helpers.state_dict('campplus', torch.float64)
    ref = {}
    for i in edges:
        wav = host[i, :int(lens[order[i]])]
        f = torch.from_numpy(fbank_ref.fbank(wav, 80, True))[None]
        ref[i] = models_ref.forward('campplus', sd, f).numpy()[0]
    with torch.no_grad():
        emb32 = step().cpu().numpy()
        model.set_hip_precision('fp16')
        emb16 = step().cpu().numpy()
        model.set_hip_precision('fp32')
    return edges, ref, emb32, emb16, lens, order


def test_c3_full_batch_rows_match_oracle(c3_run):
    edges, ref, emb32, _, lens, order = c3_run
    assert len(edges) >= 8
    assert np.isfinite(emb32).all()
    for i in edges:
        err = helpers.rel_err(emb32[i:i + 1], ref[i][None]).max()
        print(f'row {i} (utt {order[i]}, {lens[order[i]]} samples): rel err {err:.2e}')
        assert err < 1e-4, (i, err)


def test_c3_full_batch_fp16_mode_cosine(c3_run):
    edges, ref, _, emb16, _, _ = c3_run
    assert np.isfinite(emb16).all()
    for i in edges:
        a, b = emb16[i].astype(np.float64), ref[i]
        cos = float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))
        print(f'row {i}: fp16-mode cosine {cos:.6f}')
        assert cos >= 0.9999, (i, cos)
