"""GPU parity of the Fbank kernel vs the numpy oracle, and wav -> embedding end to end."""
import numpy as np
import pytest
import torch

import helpers
from oracle import fbank_ref, models_ref
from speakerlab import _hip
from speakerlab.utils import synthetic

pytestmark = pytest.mark.gpu


def _check(feat, ref):
    err = np.abs(feat - ref)
    # the kernel computes in fp64 like the oracle: what is left is the fp32 rounding of the
    # stored log-mel (half an ulp of |x| <= 16 is 9.5e-7) plus, with mean_nor, the rounding
    # of the normalised value
    assert err.max() < 5e-6, err.max()
    assert np.median(err) < 1e-6, np.median(err)


@pytest.mark.parametrize('mean_nor', [False, True])
@pytest.mark.parametrize('n_samples', [400, 16000, 32000, 32123])
def test_fbank_uniform_batch(mean_nor, n_samples):
    wavs = synthetic.pcm16_batch(3, n_samples, seed=n_samples)
    feats = _hip.fbank(torch.from_numpy(wavs).cuda(), 80, mean_nor=mean_nor).cpu().numpy()
    ref = np.stack([fbank_ref.fbank(w, 80, mean_nor) for w in wavs])
    assert feats.shape == ref.shape == (3, fbank_ref.num_frames(n_samples), 80)
    _check(feats, ref)


def test_fbank_ragged():
    lens = [16000, 24000, 400, 32000, 1000]
    L = max(lens)
    wavs = np.zeros((len(lens), L), np.float32)
    for i, n in enumerate(lens):
        wavs[i, :n] = synthetic.synth_wav(n, seed=100 + i)
    outs = _hip.fbank(torch.from_numpy(wavs).cuda(), 80, mean_nor=True, lengths=lens)
    for i, n in enumerate(lens):
        _check(outs[i].cpu().numpy(), fbank_ref.fbank(wavs[i, :n], 80, True))


def test_fbank_silence_floor():
    """all-zero input hits log(FLT_EPSILON) exactly like the reference."""
    feats = _hip.fbank(torch.zeros(1, 16000, device='cuda'), 80).cpu().numpy()
    np.testing.assert_allclose(feats, np.log(np.float32(np.finfo(np.float32).eps)), rtol=1e-6)


def test_processor_fbank_dropin():
    from speakerlab.process.processor import FBank
    wav = torch.from_numpy(synthetic.synth_wav(32000, 9))
    fb = FBank(80, 16000, mean_nor=True)
    out = fb(wav.cuda())
    assert out.shape == (198, 80) and out.is_cuda
    _check(out.cpu().numpy(), fbank_ref.fbank(wav.numpy(), 80, True))
    out_cpu_in = fb(wav)               # CPU tensor in: computed on the GPU, returned on CPU
    assert out_cpu_in.device.type == 'cpu'
    np.testing.assert_allclose(out_cpu_in.numpy(), out.cpu().numpy())


def test_processor_fbank_under_vmap():
    """The reference's diarization call site, unchanged: torch.vmap(FBank)(wavs[:, None, :])
    (infer_diarization.py:634)."""
    from speakerlab.process.processor import FBank
    wavs = synthetic.pcm16_batch(6, 24000, seed=11)
    fb = FBank(80, 16000, mean_nor=True)
    out = torch.vmap(fb)(torch.from_numpy(wavs).cuda()[:, None, :])
    assert out.shape == (6, fbank_ref.num_frames(24000), 80) and out.is_cuda
    _check(out.cpu().numpy(), np.stack([fbank_ref.fbank(w, 80, True) for w in wavs]))


def test_wav_to_embedding_end_to_end():
    wavs = synthetic.pcm16_batch(4, 32000, seed=77)
    m = helpers.loaded_module('eres2netv2')
    ref = models_ref.forward('eres2netv2', m.state_dict(), torch.from_numpy(fbank_ref.fbank_batch(wavs))).numpy()
    m = m.to('cuda')
    with torch.no_grad():
        emb = m(_hip.fbank(torch.from_numpy(wavs).cuda(), 80, mean_nor=True)).cpu().numpy()
    err = helpers.rel_err(emb, ref).max()
    assert err < 1e-4, err
