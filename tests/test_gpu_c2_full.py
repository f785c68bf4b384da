"""Config C2 at its full size (BASELINE.json configs[1]): ERes2NetV2,
B = 256 x 2 s from wav, the shape bench.py times.  At B = 256 every stage-1 activation
tensor is 128 ch x 80 x 198 x 256 x 4 B = 2.08 GB, past the 2 GiB window of one 32-bit
buffer-resource offset, so the loaders' per-block resource bases are exercised here and
nowhere at the golden-vector sizes.  Rows at both ends and around the middle are checked
against the fp64 oracle (fp64 Fbank + fp64 forward) at the north-star 1e-4, and the tail
rows against a small-batch GPU forward (no cross-talk between utterances)."""
import numpy as np
import pytest
import torch

import helpers
from oracle import fbank_ref, models_ref
from speakerlab import _hip
from speakerlab.utils import synthetic

pytestmark = pytest.mark.gpu

B, L = 256, 32000
ROWS = [0, 1, 127, 128, 254, 255]


def test_c2_full_batch_rows_vs_oracle():
    wavs = synthetic.pcm16_batch(B, L, seed=1)          # bench.py's C2 input
    m = helpers.loaded_module('eres2netv2').to('cuda')
    x = torch.from_numpy(wavs).cuda()
    with torch.no_grad():
        feats = _hip.fbank(x, 80, mean_nor=True)
        assert feats.shape == (B, 198, 80)
        emb = m(feats).cpu().numpy()
        assert not helpers.took_exact_rerun(m)   # the split plan ran: no range-guard re-run
        tail = m(feats[B - 8:].contiguous()).cpu().numpy()
        assert not helpers.took_exact_rerun(m)
    assert np.isfinite(emb).all()
    # tail rows of the 2 GB batch == the same utterances in a batch of 8
    assert helpers.rel_err(emb[B - 8:], tail).max() < 5e-5
    ref_feats = np.stack([fbank_ref.fbank(wavs[r], 80, True) for r in ROWS])
    fe = np.abs(feats[ROWS].cpu().numpy() - ref_feats).max()
    assert fe < 5e-6, fe
    sd = helpers.state_dict('eres2netv2', torch.float64)
    torch.set_num_threads(16)
    ref = models_ref.forward('eres2netv2', sd, torch.from_numpy(ref_feats)).numpy()
    err = helpers.rel_err(emb[ROWS], ref)
    print('C2 rows', ROWS, 'rel err vs fp64 oracle', err)
    assert err.max() < 1e-4, err
