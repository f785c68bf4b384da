"""Vectorised diarization host pipeline (speakerlab.utils.vad_post) == the reference's loops
(oracle/diar_ref.py, restated from speakerlab/bin/infer_diarization.py)."""
import numpy as np
import pytest

from oracle import diar_ref
from speakerlab.utils import synthetic, vad_post


def _markov_flags(n, seed, p_on=0.08, p_off=0.05):
    rng = np.random.default_rng(seed)
    out, state = np.zeros(n, dtype=np.int64), 0
    u = rng.random(n)
    for i in range(n):
        state = (u[i] < p_on) if state == 0 else (u[i] >= p_off)
        out[i] = state
    return out.tolist()


@pytest.mark.parametrize('seed', range(6))
@pytest.mark.parametrize('params', [(200.0, 300.0), (16.0, 16.0), (1000.0, 50.0)])
def test_post_process_flags(seed, params):
    flags = _markov_flags(3000, seed, p_on=0.05 + 0.1 * (seed % 3), p_off=0.02 + 0.2 * (seed % 2))
    np.testing.assert_array_equal(vad_post.post_process_speech_flags(flags, *params),
                                  diar_ref.post_process_speech_flags(flags, *params))


def test_post_process_edges():
    for flags in ([1], [0], [0, 1, 1, 1], [1, 1, 0, 0, 1], [1] * 50, [0] * 50 + [1] * 3):
        np.testing.assert_array_equal(vad_post.post_process_speech_flags(flags),
                                      diar_ref.post_process_speech_flags(flags))


def _audio(n, seed):
    return np.clip(synthetic.synth_wav(n, seed) / 32768.0, -1, 1).astype(np.float32)


@pytest.mark.parametrize('n', [100, 320, 321, 480, 16000, 16160, 16161, 160000 + 37])
def test_frame_energy_prefix_max(n):
    a = _audio(n, n)
    fe, k = vad_post.frame_energy(a)
    ref, kr = diar_ref.frame_energy(a)
    assert k == kr
    np.testing.assert_array_equal(fe, ref)


@pytest.mark.parametrize('seed', range(5))
@pytest.mark.parametrize('exp_ms,pct,floor', [(10.0, 10.0, 0.05), (0.0, 30.0, 1e-4), (50.0, 5.0, 0.0)])
def test_refine_boundaries(seed, exp_ms, pct, floor):
    n = 16000 * 20 + 123 * seed
    a = _audio(n, 10 + seed)
    flags = _markov_flags(n // 256 + 1, seed)
    proc = diar_ref.post_process_speech_flags(flags)
    mask = diar_ref.flags_to_mask(proc, n, 256)
    np.testing.assert_array_equal(vad_post.flags_to_mask(proc, n, 256), mask)
    got = vad_post.refine_boundaries(a, mask, 16000, floor, exp_ms, pct)
    ref = diar_ref.refine_boundaries(a, mask, 16000, floor, exp_ms, pct)
    np.testing.assert_array_equal(got, ref)
    assert vad_post.mask_to_intervals(got) == diar_ref.mask_to_intervals(ref)


def test_chunk_and_compress_exact():
    rng = np.random.default_rng(0)
    for _ in range(300):
        st = float(rng.uniform(0, 100))
        ed = st + float(rng.choice([0.0, 0.01, 0.75, 1.5, 1.51, 2.25, rng.uniform(0, 30)]))
        assert vad_post.chunk(st, ed) == diar_ref.chunk(st, ed)
        assert vad_post.chunk(st, ed, 3.0, 1.0) == diar_ref.chunk(st, ed, 3.0, 1.0)
    chunks = [c for s in np.cumsum(rng.uniform(0.5, 6, 40)) for c in diar_ref.chunk(float(s), float(s) + 4.0)]
    segs = [[a, b, int(rng.integers(0, 3))] for a, b in chunks]
    assert vad_post.compressed_seg([list(s) for s in segs]) == diar_ref.compressed_seg([list(s) for s in segs])


def test_flags_to_intervals():
    flags = _markov_flags(500, 3)
    got = vad_post.flags_to_intervals(flags, 500 * 256 - 100, 256)
    ref, i = [], 0
    while i < len(flags):                       # infer_diarization.py:500-514
        if flags[i]:
            j = i + 1
            while j < len(flags) and flags[j]:
                j += 1
            st, ed = i * 256 / 16000, min(j * 256, 500 * 256 - 100) / 16000
            if ed > st:
                ref.append([st, ed])
            i = j
        else:
            i += 1
    assert got == ref


def test_energy_vad_and_writers(tmp_path):
    from speakerlab.bin import infer_diarization as idz
    wav, turns = synthetic.synth_meeting(10.0, 2, seed=1)
    flags, x = idz.EnergyVad()(wav)
    assert len(flags) == len(wav) // 256 and x.dtype == np.float32
    assert 0.3 < np.mean(flags) < 1.0
    d = idz.Diarization3Dspeaker.__new__(idz.Diarization3Dspeaker)
    d.output_field_labels = [[0.5, 2.25, 0], [2.25, 4.0, 1]]
    d.save_diar_output(str(tmp_path / 'a.rttm'), 'utt')
    assert (tmp_path / 'a.rttm').read_text() == ('SPEAKER utt 0 0.500 1.750 <NA> <NA> 0 <NA> <NA>\n'
                                                'SPEAKER utt 0 2.250 1.750 <NA> <NA> 1 <NA> <NA>\n')
    d.save_diar_output(str(tmp_path / 'a.json'))
    import json
    js = json.loads((tmp_path / 'a.json').read_text())
    assert js['default_0.5_2.25'] == {'start': 0.5, 'stop': 2.25, 'speaker': 0}
    with pytest.raises(ValueError):
        d.save_diar_output(str(tmp_path / 'a.txt'))
