"""ORACLE (test infrastructure only) — Kaldi Fbank restated in numpy.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker.  The product path (``speakerlab.process.
processor.FBank`` in ``3d-speaker_amd/``) runs the HIP kernel and never calls this.

What it restates
----------------
``speakerlab/process/processor.py:133-158`` (``FBank.__call__``) calls
``torchaudio.compliance.kaldi.fbank(wav, num_mel_bins=n_mels, sample_frequency=16000,
dither=0)`` then optionally subtracts the per-utterance mean (``processor.py:156-157``).
torchaudio (``requirements.txt:2``, ``>=0.10.1``, version otherwise unpinned) is absent
from this image, so its published algorithm is restated step by step with the defaults
that call uses (SURVEY.md §8(a) note a1):

1. frames of 400 samples, hop 160, ``snip_edges=True``: m = 1 + (L-400)//160;
2. per-frame DC removal (``remove_dc_offset``);
3. pre-emphasis 0.97 with a replicate-padded first sample;
4. Povey window = hann(400, periodic=False) ** 0.85;
5. zero-pad to 512 and take |rfft|^2 (``use_power``);
6. 80 triangular mel filters on 1127 ln(1 + f/700), 20 Hz .. 8 kHz, 256 bins plus a
   zero Nyquist column;
7. log(max(E, FLT_EPSILON)).

Parity pinning: the FFT step is pinned against the reference's own
radix-2 FFT (``runtime/onnxruntime/feature/feature_functions.cpp:37-60``) compiled from
source into ``oracle/_ref`` by ``oracle/Makefile``; the rest of the reference's C++
Fbank (``feature_fbank.cpp:22-91``) needs nlohmann/json, which the image lacks, so it is
unbuildable here and torchaudio parity of steps 1-4 and 6-7 is *unpinned* (restated
from the published algorithm, cross-checked against the C++ runtime's restatement of
the same Kaldi recipe in ``tests/test_fbank_oracle.py``).
"""
from __future__ import annotations

import math

import numpy as np

FRAME_LEN = 400
FRAME_SHIFT = 160
PADDED = 512
N_FFT_BINS = PADDED // 2
FLT_EPS = float(np.finfo(np.float32).eps)


def num_frames(n_samples: int) -> int:
    """``snip_edges=True`` frame count (torchaudio ``_get_strided``)."""
    if n_samples < FRAME_LEN:
        return 0
    return 1 + (n_samples - FRAME_LEN) // FRAME_SHIFT


def povey_window(dtype=np.float64) -> np.ndarray:
    n = np.arange(FRAME_LEN, dtype=np.float64)
    hann = 0.5 - 0.5 * np.cos(2.0 * math.pi * n / (FRAME_LEN - 1))
    return (hann ** 0.85).astype(dtype)


def _mel(f):
    return 1127.0 * np.log(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_banks(n_mels: int = 80, sample_rate: float = 16000.0, low_freq: float = 20.0,
              high_freq: float = 0.0) -> np.ndarray:
    """[n_mels, 257] triangular filters (torchaudio ``get_mel_banks`` + zero Nyquist pad).

    torchaudio builds the bank in float32 tensors; the values here are computed in float64
    and rounded once (difference <= 1 ulp of the weights).
    """
    nyquist = 0.5 * sample_rate
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = sample_rate / PADDED
    mel_low = 1127.0 * math.log(1.0 + low_freq / 700.0)
    mel_high = 1127.0 * math.log(1.0 + high_freq / 700.0)
    delta = (mel_high - mel_low) / (n_mels + 1)
    b = np.arange(n_mels, dtype=np.float64)[:, None]
    left = mel_low + b * delta
    center = mel_low + (b + 1.0) * delta
    right = mel_low + (b + 2.0) * delta
    mel = _mel(fft_bin_width * np.arange(N_FFT_BINS, dtype=np.float64))[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    banks = np.maximum(0.0, np.minimum(up, down))
    return np.pad(banks, ((0, 0), (0, 1)))


def frames_of(wav: np.ndarray) -> np.ndarray:
    m = num_frames(wav.shape[-1])
    idx = np.arange(m)[:, None] * FRAME_SHIFT + np.arange(FRAME_LEN)[None, :]
    return wav[idx]


def windowed_frames(wav: np.ndarray, dtype=np.float64) -> np.ndarray:
    """Steps 1-4 + zero pad: [m, 512]."""
    fr = frames_of(np.asarray(wav, dtype=dtype))
    fr = fr - fr.mean(axis=1, keepdims=True)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    fr = fr - 0.97 * prev
    fr = fr * povey_window(dtype)[None, :]
    return np.pad(fr, ((0, 0), (0, PADDED - FRAME_LEN)))


def fbank(wav, n_mels: int = 80, mean_nor: bool = False, dtype=np.float64) -> np.ndarray:
    """Kaldi log-mel fbank of a 1-D waveform (float in [-1, 1)), [m, n_mels].

    ``dtype=np.float64`` is the high-precision oracle; ``np.float32`` emulates an fp32 run.
    Multi-channel input follows ``processor.py:146-151`` (channel 0 is used).
    """
    wav = np.asarray(wav)
    if wav.ndim == 2:
        wav = wav[0]
    fr = windowed_frames(wav, dtype)
    spec = np.fft.rfft(fr, axis=1)
    power = (spec.real ** 2 + spec.imag ** 2).astype(dtype)
    banks = mel_banks(n_mels).astype(dtype)
    energies = power @ banks.T
    feat = np.log(np.maximum(energies, FLT_EPS)).astype(dtype)
    if mean_nor:
        feat = feat - feat.mean(axis=0, keepdims=True)
    return feat


def fbank_batch(wavs: np.ndarray, n_mels: int = 80, mean_nor: bool = True) -> np.ndarray:
    """[B, L] equal-length waveforms -> [B, m, n_mels] float32 (fp64 internally)."""
    return np.stack([fbank(w, n_mels, mean_nor) for w in wavs]).astype(np.float32)
