"""Diarization end to end on the GPU vs the oracle pipeline: the same VAD flags go through
the reference's post-processing loops (oracle/diar_ref.py), its sub-segments through the
fp64 Fbank + fp64 ERes2NetV2 (oracle), then through the same clustering decisions; the
output segments must be identical."""
import json

import numpy as np
import pytest
import torch

import helpers
from oracle import diar_ref, fbank_ref, models_ref
from speakerlab.bin import infer_diarization as idz
from speakerlab.process import cluster
from speakerlab.utils import synthetic
from speakerlab.utils.fileio import write_wav
from speakerlab.utils.utils import circle_pad

pytestmark = pytest.mark.gpu


def _oracle_segments(diar, wav):
    flags, x = diar.do_vad(wav[None])
    proc = diar_ref.post_process_speech_flags(flags)
    mask = diar_ref.flags_to_mask(proc, len(x), 256)
    refined = diar_ref.refine_boundaries(x, mask)
    chunks = [c for st, ed in diar_ref.mask_to_intervals(refined) for c in diar_ref.chunk(st, ed)]
    t = torch.from_numpy(wav)
    pieces = [t[int(st * 16000):int(ed * 16000)] for st, ed in chunks]
    L = max(p.shape[0] for p in pieces)
    batch = torch.stack([circle_pad(p, L) for p in pieces]).numpy()
    sd = diar.embedding_model.state_dict()
    emb = models_ref.forward('eres2netv2', {k: v.cpu() for k, v in sd.items()},
                             torch.from_numpy(fbank_ref.fbank_batch(batch))).numpy()
    return chunks, emb


def test_diarization_matches_oracle(tmp_path):
    wav, turns = synthetic.synth_meeting(24.0, 3, seed=3)
    diar = idz.Diarization3Dspeaker('cuda', synthetic_weights=True, vad='energy')
    out = diar(torch.from_numpy(wav)[None], wav_fs=16000)
    chunks, emb_ref = _oracle_segments(diar, wav)
    emb = diar.do_emb_extraction(chunks, torch.from_numpy(wav)[None])
    assert emb.shape == emb_ref.shape and len(chunks) > 10
    # end to end from wav at the north-star bar (fp64 GPU Fbank, tests/test_gpu_fbank.py)
    assert helpers.rel_err(emb, emb_ref).max() < 1e-4
    # same clustering decisions on the oracle embeddings (host cosine in fp64)
    S = cluster._host_cosine(emb_ref, emb_ref).astype(np.float32)
    lab = cluster.ahc_labels(S, 0.3)
    cc = diar.cluster
    lab = cc.merge_by_cos(cc.filter_minor_cluster(lab, emb_ref, 0), emb_ref, 0.3)
    ref = diar_ref.compressed_seg([[c[0], c[1], int(j)] for c, j in zip(chunks, lab)])
    assert out == ref
    # hence the same DER as the oracle pipeline, scored like the reference recipe (md-eval)
    from speakerlab.utils import der
    gt = [f'SPEAKER m 0 {a:.3f} {b - a:.3f} <NA> <NA> s{k} <NA> <NA>' for a, b, k in turns]
    to_rttm = lambda segs: [f'SPEAKER m 0 {a:.3f} {b - a:.3f} <NA> <NA> {k} <NA> <NA>' for a, b, k in segs]
    assert der.der(gt, to_rttm(out)) == der.der(gt, to_rttm(ref))

    rttm = tmp_path / 'm.rttm'
    diar.save_diar_output(str(rttm), 'm')
    lines = rttm.read_text().splitlines()
    assert len(lines) == len(out) and lines[0].startswith('SPEAKER m 0 ')


def test_diarization_cli_outputs(tmp_path):
    wav, _ = synthetic.synth_meeting(12.0, 2, seed=5)
    p = tmp_path / 'meet.wav'
    write_wav(str(p), wav)
    idz.main(['--wav', str(p), '--out_dir', str(tmp_path / 'out'), '--out_type', 'json', '--synthetic_weights',
              '--vad', 'energy', '--diable_progress_bar', '--nprocs', '1'])
    res = json.loads((tmp_path / 'out' / 'meet.json').read_text())
    assert len(res) >= 1 and all(k.startswith('meet_') for k in res)
    for side in ('meta', 'vad_info', 'pairs'):
        assert (tmp_path / 'out' / f'meet.{side}.json').exists()
    meta = json.loads((tmp_path / 'out' / 'meet.meta.json').read_text())
    assert abs(meta['duration_sec'] - 12.0) < 1e-3
