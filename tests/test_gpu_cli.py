"""infer_sv_batch end to end on the GPU: wav files -> 10 s circle-padded chunks -> GPU Fbank
-> native forward -> per-wav mean, checked against the oracle (fp64 Fbank + fp64 model)
on the same chunks (reference ``speakerlab/bin/infer_sv_batch.py:122-207, 300-330``)."""
import numpy as np
import pytest
import torch

import helpers
from oracle import fbank_ref, models_ref
from speakerlab.bin import infer_sv_batch as isb
from speakerlab.utils import kaldi_io, synthetic
from speakerlab.utils.fileio import write_wav

pytestmark = pytest.mark.gpu

MODEL_ID = 'iic/speech_campplus_sv_zh-cn_16k-common'      # CAM++(192): cheap in the fp64 oracle


def _wavs(tmp_path):
    paths = []
    for i, sec in enumerate([3, 12, 21, 0.5]):
        p = tmp_path / f'spk{i}.wav'
        write_wav(str(p), synthetic.synth_wav(int(sec * 16000), seed=40 + i) / 32768.0)
        paths.append(str(p))
    lst = tmp_path / 'wav.list'
    lst.write_text('\n'.join(paths) + '\n')
    return paths, lst


def _oracle(paths):
    class A:
        synthetic_weights = True
    sd = isb.build_model(isb.supports[MODEL_ID], A, None).state_dict()
    out = {}
    for p in paths:
        chunks = isb.load_wav_chunks(p).numpy()
        feats = torch.from_numpy(fbank_ref.fbank_batch(chunks))
        out[isb.wav_id_of(p)] = models_ref.forward('campplus_192', sd, feats).numpy().mean(0)
    return out


@pytest.mark.parametrize('fmt', ['npy', 'ark'])
def test_infer_sv_batch_matches_oracle(tmp_path, fmt):
    paths, lst = _wavs(tmp_path)
    out_dir = tmp_path / 'emb'
    isb.main(['--model_id', MODEL_ID, '--wavs', str(lst), '--feat_out_dir', str(out_dir), '--synthetic_weights',
              '--feat_out_format', fmt, '--batch_size', '2', '--diable_progress_bar', '--nprocs', '1'])
    if fmt == 'npy':
        got = {isb.wav_id_of(p): np.load(out_dir / f'{isb.wav_id_of(p)}.npy') for p in paths}
    else:
        got = dict(kaldi_io.read_ark(str(out_dir / 'embedding_0.ark')))
    ref = _oracle(paths)
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert got[k].shape == (192,)
        # end to end from wav at the north-star bar (the GPU Fbank computes in fp64)
        assert helpers.rel_err(got[k][None], ref[k][None]).max() < 1e-4, k


def test_runtime_extract_speaker_embedding_cli(tmp_path):
    """Drop-in for the C++ runtime binary (runtime/onnxruntime/bin/extract_speaker_embedding.cpp):
    wav.scp in, one text .embedding per utterance + the embedding scp out, int16/32767 samples."""
    import json

    from speakerlab.bin import extract_speaker_embedding as ese
    from speakerlab.utils import runtime_io
    scp, ids = [], ['spk1/utt1', 'spk0/utt2', 'spk2/utt0']
    for i, u in enumerate(ids):
        p = tmp_path / f'w{i}.wav'
        write_wav(str(p), synthetic.synth_wav(int((1.2 + i) * 16000), seed=70 + i) / 32768.0)
        scp.append(f'{u} {p}')
    (tmp_path / 'wav.scp').write_text('\n'.join(scp) + '\n')
    cfg = tmp_path / 'fbank_config.json'
    cfg.write_text(json.dumps({'FrameExtractionOptions': {'sample_freq': 16000, 'frame_shift_ms': 10.0,
                                                          'frame_length_ms': 25.0, 'dither': 0.0},
                               'MelBanksOptions': {'num_bins': 80}, 'use_power': True}))
    out = tmp_path / 'emb'
    assert ese.main([str(cfg), MODEL_ID, str(tmp_path / 'wav.scp'), str(tmp_path / 'emb.scp'), str(out)]) == 0
    got_scp = runtime_io.read_wav_scp(str(tmp_path / 'emb.scp'))
    assert list(got_scp) == sorted(ids)

    class A:
        synthetic_weights = True
    sd = isb.build_model(isb.supports[MODEL_ID], A, None).state_dict()
    for i, u in enumerate(ids):
        path = out / (runtime_io.normalize_for_path(u) + '.embedding')
        assert got_scp[u] == str(path)
        wav = runtime_io.read_runtime_wav(str(tmp_path / f'w{i}.wav')).samples
        feats = torch.from_numpy(fbank_ref.fbank_batch(wav[None]))
        ref = models_ref.forward('campplus_192', sd, feats).numpy()
        got = runtime_io.read_runtime_embedding(str(path))[None]
        assert helpers.rel_err(got, ref).max() < 1e-4, u       # text %g keeps 6 significant digits
