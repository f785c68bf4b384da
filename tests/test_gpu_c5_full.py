"""Config C5 at full size (BASELINE.json configs[4]): the 1 h synthetic meeting of
tools/bench_diarization.py through the GPU pipeline -- energy VAD, post-processing, 1.5 s /
0.75 s chunks, GPU Fbank + ERes2NetV2 embeddings, clustering -- against the ORACLE pipeline's
fixture (tests/golden/make_c5_golden.py: the reference's VAD post-processing and chunking as
loops, fp64 Kaldi Fbank, the op-for-op ERes2NetV2, host clustering):

* the same 3,538 chunks;
* embeddings within the north-star 1e-4 on every 16th chunk (the stored rows);
* the CLI's AHC back-end: the same segments (infer_diarization.py:621-649, 780-797);
* spectral clustering with the oracle speaker count (--speaker_num 4, no centroid merge):
  the same four-speaker partition of the chunks, and the same DER against the generator's
  turns.  (With the synthetic weights the AHC thresholds of the recipe see one speaker; the
  spectral partition is the non-degenerate check.)"""
import os

import numpy as np
import pytest
import torch

import helpers
from speakerlab.bin import infer_diarization as idz
from speakerlab.process import cluster
from speakerlab.utils import der, synthetic, vad_post

pytestmark = pytest.mark.gpu
G = dict(np.load(os.path.join(helpers.GOLDEN, 'c5_golden.npz')))


def _partition(labels):
    """Canonical form of a partition: labels renumbered by first occurrence."""
    seen = {}
    return np.array([seen.setdefault(int(v), len(seen)) for v in labels])


def test_c5_full_meeting_matches_oracle_pipeline():
    minutes, spk, seed, _ = G['meta']
    wav, turns = synthetic.synth_meeting(minutes * 60, int(spk), seed=int(seed))
    diar = idz.Diarization3Dspeaker('cuda', synthetic_weights=True, vad='energy', batch_size=256)
    x = torch.from_numpy(wav)[None]
    flags, xv = diar.do_vad(x)
    _, _, vad_time = diar.postprocess_vad(flags, xv)
    chunks = [c for st, ed in vad_time for c in diar.chunk(st, ed)]
    assert np.array_equal(np.asarray(chunks, np.float64), G['chunks'])
    emb = diar.do_emb_extraction(chunks, x)
    err = helpers.rel_err(emb[G['idx']], G['emb']).max()
    print(f'{len(chunks)} chunks, embeddings vs oracle (every 16th): max rel err {err:.2e}')
    assert err < 1e-4
    np.random.seed(0)
    _, segs = diar.do_clustering(chunks, emb)
    assert np.allclose(np.asarray(segs, np.float64), G['seg_ahc'])
    np.random.seed(0)
    lab = cluster.spectral_labels_gpu(emb, oracle_num=int(spk))
    assert len(np.unique(lab)) == int(spk)
    assert np.array_equal(_partition(lab), _partition(G['labels_spectral']))
    gt = [f'SPEAKER m 0 {a:.3f} {b - a:.3f} <NA> <NA> s{k} <NA> <NA>' for a, b, k in turns]
    rttm = lambda s: [f'SPEAKER m 0 {a:.3f} {b - a:.3f} <NA> <NA> {int(k)} <NA> <NA>' for a, b, k in s]
    ours = der.der(gt, rttm(vad_post.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lab)])))
    ref = der.der(gt, rttm(G['seg_spectral'].tolist()))
    print('spectral (oracle count) DER', ours)
    assert ours == ref
