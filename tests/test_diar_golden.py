"""Diarization host stages vs fixtures produced by the REFERENCE
``speakerlab/bin/infer_diarization.py`` methods (``tests/golden/make_cluster_golden.py``):
``_post_process_speech_flags`` (:347-384), ``postprocess_vad`` = flags -> mask ->
``_refine_vad_boundaries_with_energy`` -> ``_mask_to_intervals`` (:322-482), ``chunk``
(:606-619) and ``compressed_seg`` (:780-797).  The product methods run on an instance built the
same way the fixture script built the reference's (``object.__new__`` + the ``__init__``
defaults), so these tests read like calls into the reference."""
import json
import os

import numpy as np
import pytest

from speakerlab.bin import infer_diarization as D
from speakerlab.utils import vad_post

GJ = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'diar_host_golden.json')))


def inst(**over):
    o = object.__new__(D.Diarization3Dspeaker)
    o.fs = 16000
    o.chunk_dur, o.chunk_step = 1.5, 0.75
    o.vad_frame_size_ms = 16.0
    o.vad_min_speech_ms, o.vad_max_silence_ms = 200.0, 300.0
    o.vad_energy_threshold = 0.05
    o.vad_boundary_expansion_ms, o.vad_boundary_energy_percentile = 10.0, 10.0
    for k, v in over.items():
        setattr(o, k, v)
    return o


def from_runs(runs, n):
    m = np.zeros(n, dtype=np.int64)
    for a, b in runs:
        m[a:b] = 1
    return m


def runs(mask):
    d = np.diff(np.concatenate(([0], (np.asarray(mask) != 0).astype(np.int8), [0])))
    return np.stack([np.where(d > 0)[0], np.where(d < 0)[0]], axis=1).tolist()


def synth_audio(n, seed):
    """Same generator as the fixture script (tests/golden/make_cluster_golden.py)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 16000.0
    env = np.zeros(n)
    pos = 0
    while pos < n:
        ln = int(rng.integers(1600, 24000))
        if rng.random() < 0.6:
            env[pos:pos + ln] = rng.uniform(0.1, 0.8)
        pos += ln + int(rng.integers(0, 8000))
    f0 = rng.uniform(90, 250)
    sig = sum(np.sin(2 * np.pi * f0 * k * t + rng.uniform(0, 6)) / k for k in range(1, 6))
    x = env * sig + 0.003 * rng.standard_normal(n)
    return np.clip(x, -1, 1).astype(np.float32)


@pytest.mark.parametrize('i', range(len(GJ['flags'])))
def test_post_process_speech_flags(i):
    c = GJ['flags'][i]
    flags = from_runs(c['flags_runs'], c['n'])
    out = vad_post.post_process_speech_flags(flags.tolist(), c['min_speech_ms'], c['max_silence_ms'], 16.0)
    assert runs(out) == c['out_runs']


@pytest.mark.parametrize('i', range(len(GJ['vad'])))
def test_postprocess_vad(i):
    c = GJ['vad'][i]
    audio = synth_audio(c['n'], c['seed'])
    flags = from_runs(c['flags_runs'], (c['n'] + 255) // 256)
    o = inst(vad_energy_threshold=c['energy_threshold'], vad_boundary_expansion_ms=c['expansion_ms'],
             vad_boundary_energy_percentile=c['percentile'])
    processed, refined, vad_time = o.postprocess_vad(flags.tolist(), audio)
    assert runs(processed) == c['processed_runs']
    assert runs(refined) == c['refined_runs']
    assert vad_time == c['intervals']


@pytest.mark.parametrize('i', range(len(GJ['chunk'])))
def test_chunk(i):
    c = GJ['chunk'][i]
    assert inst(chunk_dur=c['dur'], chunk_step=c['step']).chunk(c['st'], c['ed']) == c['out']


@pytest.mark.parametrize('i', range(len(GJ['compressed'])))
def test_compressed_seg(i):
    c = GJ['compressed'][i]
    assert vad_post.compressed_seg([list(s) for s in c['in']]) == c['out']
