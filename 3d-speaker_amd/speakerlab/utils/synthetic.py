"""Deterministic synthetic inputs and weights (SURVEY.md §8(c) golden-vector plan, §8(d)).

There is no network in this environment: no modelscope checkpoints and no datasets.
Benchmarks and parity tests therefore run on

* synthetic 16 kHz speech-like audio, PCM16-quantised and scaled by 1/32768 exactly
  like ``torchaudio.load`` / ``speakerlab/utils/fileio.py:117-119`` do;
* deterministic random weights whose value depends only on the ``state_dict`` key,
  so the same weights can be rebuilt for the reference modules (fixture generation)
  and for this package's modules (tests, bench) without shipping 70 MB checkpoints.

This module is self-contained (numpy + torch only) so that the fixture script can load
it by file path next to the reference package without a ``speakerlab`` name clash.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Mapping, Tuple

import numpy as np

SAMPLE_RATE = 16000


def synth_wav(n_samples: int, seed: int, speaker: int | None = None) -> np.ndarray:
    """Speech-like float32 waveform in [-1, 1), PCM16-quantised.

    Harmonic "voiced" bursts (f0 80-300 Hz, 12 harmonics shaped by two formant bumps)
    plus low-level noise and short silences.  ``speaker`` pins f0/formants so that
    different utterances of one synthetic speaker are similar (used by clustering tests).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    sp_rng = np.random.Generator(np.random.PCG64(10_007 * (speaker + 1))) if speaker is not None else rng
    f0 = sp_rng.uniform(80.0, 300.0)
    formants = sp_rng.uniform([300.0, 900.0], [900.0, 2600.0])
    t = np.arange(n_samples, dtype=np.float64) / SAMPLE_RATE
    # slow f0 wobble
    f0_t = f0 * (1.0 + 0.05 * np.sin(2 * np.pi * rng.uniform(0.5, 3.0) * t + rng.uniform(0, 6.28)))
    phase = 2 * np.pi * np.cumsum(f0_t) / SAMPLE_RATE
    sig = np.zeros(n_samples)
    for h in range(1, 13):
        fh = h * f0
        amp = sum(np.exp(-0.5 * ((fh - f) / 150.0) ** 2) for f in formants) + 0.05 / h
        sig += amp * np.sin(h * phase + rng.uniform(0, 6.28))
    # syllable envelope with silences
    env = np.zeros(n_samples)
    pos = 0
    while pos < n_samples:
        seg = int(rng.uniform(0.08, 0.35) * SAMPLE_RATE)
        if rng.uniform() < 0.8:
            w = np.hanning(max(seg, 2))
            env[pos:pos + seg] = w[: max(0, min(seg, n_samples - pos))]
        pos += seg + int(rng.uniform(0.0, 0.08) * SAMPLE_RATE)
    sig = sig * env / (np.abs(sig).max() + 1e-9)
    sig = 0.5 * sig + 0.01 * rng.standard_normal(n_samples)
    pcm = np.clip(np.round(sig * 32767.0), -32768, 32767).astype(np.int16)
    return (pcm.astype(np.float32) / 32768.0).astype(np.float32)


def _key_rng(key: str, seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(zlib.crc32(key.encode()) + 1_000_003 * seed))


def synth_state_dict(shapes: Mapping[str, Tuple[Tuple[int, ...], str]], seed: int = 0) -> Dict[str, np.ndarray]:
    """Deterministic weights for a ``state_dict`` layout.

    ``shapes`` maps key -> (shape, dtype-string).  Rules (per key, independent of order):
      * BatchNorm (a sibling ``running_mean`` exists): weight ~ U(0.8, 1.2),
        bias ~ N(0, 0.1), running_mean 0, running_var 1 (fixtures overwrite the running
        stats with a calibration pass), num_batches_tracked 0;
      * conv / linear weight: N(0, 1/fan_in);
      * any other bias / 1-D parameter: N(0, 0.05).
    """
    keys = set(shapes)
    out: Dict[str, np.ndarray] = {}
    for key, (shape, dtype) in shapes.items():
        prefix, _, leaf = key.rpartition('.')
        is_bn = (prefix + '.running_mean') in keys
        if leaf == 'num_batches_tracked':
            out[key] = np.zeros(shape, dtype=np.int64)
            continue
        rng = _key_rng(key, seed)
        if is_bn and leaf == 'weight':
            v = rng.uniform(0.8, 1.2, size=shape)
        elif is_bn and leaf == 'bias':
            v = rng.normal(0.0, 0.1, size=shape)
        elif leaf == 'running_mean':
            v = np.zeros(shape)
        elif leaf == 'running_var':
            v = np.ones(shape)
        elif leaf == 'weight' and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            v = rng.standard_normal(size=shape) / np.sqrt(fan_in)
        else:
            v = rng.normal(0.0, 0.05, size=shape)
        out[key] = np.asarray(v, dtype=np.float32)
    return out


def shapes_of(state_dict) -> Dict[str, Tuple[Tuple[int, ...], str]]:
    """``{key: (shape, dtype)}`` from a torch state_dict."""
    return {k: (tuple(v.shape), str(v.dtype)) for k, v in state_dict.items()}


def load_synthetic_weights(module, seed: int = 0, bn_stats: Mapping[str, np.ndarray] | None = None):
    """Fill ``module`` (any nn.Module) with :func:`synth_state_dict` weights in place.

    ``bn_stats`` (e.g. a committed calibration fixture) overrides running statistics.
    Uses strict ``load_state_dict`` like ``infer_sv_batch.py:249-252``.
    """
    import torch
    sd = module.state_dict()
    vals = synth_state_dict(shapes_of(sd), seed)
    if bn_stats is not None:
        for k in bn_stats:
            if k in vals:
                vals[k] = np.asarray(bn_stats[k]).astype(vals[k].dtype)
    module.load_state_dict({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in vals.items()}, strict=True)
    return module


def pcm16_batch(n_utts: int, n_samples: int, seed: int) -> np.ndarray:
    """[n_utts, n_samples] float32 batch; utterance i uses seed ``seed * 1_000_000 + i``."""
    return np.stack([synth_wav(n_samples, seed * 1_000_000 + i) for i in range(n_utts)])


def synth_meeting(seconds: float, n_speakers: int, seed: int, turn=(1.0, 8.0), silence=0.1):
    """Synthetic meeting: random speaker turns of ``turn`` seconds from
    ``n_speakers`` fixed-timbre synthetic speakers, ~``silence`` fraction of pauses.
    Returns (wav float32 [L], turns [[st, ed, speaker], ...])."""
    rng = np.random.Generator(np.random.PCG64(seed))
    total = int(seconds * SAMPLE_RATE)
    wav = np.zeros(total, dtype=np.float32)
    turns, pos, k, prev = [], 0, 0, -1
    while pos < total:
        if rng.uniform() < silence:
            pos += int(rng.uniform(0.2, 1.0) * SAMPLE_RATE)
            continue
        spk = int(rng.integers(n_speakers))
        if spk == prev:
            spk = (spk + 1) % n_speakers
        n = min(int(rng.uniform(*turn) * SAMPLE_RATE), total - pos)
        if n <= 0:
            break
        wav[pos:pos + n] = synth_wav(n, seed * 100_003 + k, speaker=spk)
        turns.append([pos / SAMPLE_RATE, (pos + n) / SAMPLE_RATE, spk])
        pos += n
        k += 1
        prev = spk
    return wav, turns
