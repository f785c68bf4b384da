"""Pin the numpy Fbank oracle (oracle/fbank_ref.py).

* FFT step vs the reference's own radix-2 FFT (runtime/onnxruntime/feature/
  feature_functions.cpp:37-60) compiled from source into oracle/_ref by oracle/Makefile.
* Whole pipeline with that FFT substituted (= the C++ runtime's FbankComputer order,
  feature_fbank.cpp:47-86) vs the oracle.
* Known answers of the published torchaudio/Kaldi recipe: frame count, window, mel bank.
"""
import ctypes
import os

import numpy as np
import pytest

from oracle import fbank_ref
from speakerlab.utils import synthetic

REF_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle', '_ref', 'libref_fft.so')


def _ref_fft():
    if not os.path.exists(REF_SO):
        pytest.skip('oracle/_ref/libref_fft.so not built (reference sources absent)')
    lib = ctypes.CDLL(REF_SO)
    lib.ref_custom_fft.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] + [ctypes.c_void_p] * 2

    def fft(x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        re = np.zeros_like(x)
        im = np.zeros_like(x)
        assert lib.ref_custom_fft(x.ctypes.data, None, x.size, re.ctypes.data, im.ctypes.data) == 0
        return re.astype(np.float64) + 1j * im.astype(np.float64)
    return fft


def test_fft_step_matches_reference_fft():
    fft = _ref_fft()
    wav = synthetic.synth_wav(16000, seed=21)
    frames = fbank_ref.windowed_frames(wav)
    for fr in frames[::7]:
        ours = np.fft.fft(fr)
        ref = fft(fr)
        scale = np.abs(ours).max()
        assert np.abs(ours - ref).max() / scale < 2e-6


def test_pipeline_with_reference_fft():
    fft = _ref_fft()
    wav = synthetic.synth_wav(24000, seed=22)
    frames = fbank_ref.windowed_frames(wav).astype(np.float32)
    power = np.stack([np.abs(fft(f)[:257]) ** 2 for f in frames])
    banks = fbank_ref.mel_banks(80)
    feat = np.log(np.maximum(power @ banks.T, fbank_ref.FLT_EPS))
    ours = fbank_ref.fbank(wav)
    err = np.abs(feat - ours)
    # an fp32 FFT carries ~1e-7 x (frame energy) absolute noise, which is visible in the log
    # of near-silent mel bands (E ~ 1e-7): bound the worst case loosely, the typical tightly
    assert err.max() < 5e-4
    assert np.median(err) < 1e-6


def test_known_answers():
    assert fbank_ref.num_frames(32000) == 198
    assert fbank_ref.num_frames(24000) == 148
    assert fbank_ref.num_frames(399) == 0
    w = fbank_ref.povey_window()
    assert w[0] == 0.0 and abs(w[199] - w[200]) < 1e-12 and w.max() <= 1.0
    banks = fbank_ref.mel_banks(80)
    assert banks.shape == (80, 257)
    assert np.all(banks[:, 256] == 0) and np.all(banks >= 0) and np.all(banks.max(axis=1) > 0.4) and np.all((banks > 0).sum(axis=1) >= 1)
    feat = fbank_ref.fbank(synthetic.synth_wav(32000, 3), mean_nor=True)
    assert feat.shape == (198, 80)
    assert np.abs(feat.mean(axis=0)).max() < 1e-9


def test_multichannel_uses_channel0():
    a = synthetic.synth_wav(16000, 5)
    b = synthetic.synth_wav(16000, 6)
    np.testing.assert_array_equal(fbank_ref.fbank(np.stack([a, b])), fbank_ref.fbank(a))
