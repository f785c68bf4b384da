"""VAD post-processing and segment bookkeeping of the diarization pipeline, vectorised.

Restates the per-frame / per-sample Python loops of the reference
``speakerlab/bin/infer_diarization.py`` with run-length numpy so that an hour of audio
(225 k VAD frames, 57.6 M samples) costs milliseconds instead of seconds.  Results are
identical to the loops (``tests/test_diar_host.py`` checks them against ``oracle/diar_ref.py``):

* ``post_process_speech_flags`` — 3-frame majority smoothing, fill silence gaps of
  <= max_silence frames that are followed by speech, then drop speech runs shorter than
  min_speech that are followed by silence (``infer_diarization.py:355-393``);
* ``frame_energy`` — the 20 ms / 10 ms energy track.  The reference writes
  ``max(track[s:e].max(), en)`` over half-overlapping windows, which makes the track the
  running (prefix) maximum of the frame energies, held per 10 ms hop
  (``infer_diarization.py:403-413``);
* ``refine_boundaries`` — per-segment percentile threshold, forward / backward contraction
  inside a 100 ms look-ahead and re-expansion (``infer_diarization.py:415-461``); note the
  re-expansion at the end starts at ``i + 1``, so a contracted end leaves a one-sample hole;
* ``mask_to_intervals`` / ``flags_to_intervals`` (``:463-516``), ``chunk`` (``:606-619``)
  and ``compressed_seg`` (``:780-797``), the last two with the reference's float
  accumulation order.
"""
import numpy as np
from numpy.lib.stride_tricks import sliding_window_view


def _runs(x: np.ndarray):
    """Run-length encoding: (starts, ends_exclusive, values)."""
    n = len(x)
    if n == 0:
        e = np.zeros(0, dtype=np.int64)
        return e, e, x[:0]
    change = np.flatnonzero(x[1:] != x[:-1]) + 1
    starts = np.concatenate(([0], change))
    ends = np.concatenate((change, [n]))
    return starts, ends, x[starts]


def _set_runs(res, starts, ends, value):
    if len(starts) == 0:
        return
    delta = np.zeros(len(res) + 1, dtype=np.int64)
    np.add.at(delta, starts, 1)
    np.add.at(delta, ends, -1)
    res[np.cumsum(delta[:-1]) > 0] = value


def post_process_speech_flags(flags, min_speech_ms=200.0, max_silence_ms=300.0, frame_ms=16.0):
    f = np.asarray(flags, dtype=np.float32)
    if f.size == 0:
        return f.copy()
    p = np.pad(f, (1, 1), mode='edge')
    res = (np.convolve(p, np.ones(3) / 3, mode='valid') > 0.5).astype(np.float32)
    min_speech = max(1, int(min_speech_ms / frame_ms))
    max_sil = max(1, int(max_silence_ms / frame_ms))
    n = len(res)
    s, e, v = _runs(res)
    gap = (v == 0) & (e < n) & (e - s <= max_sil)          # a zero run closed by speech
    _set_runs(res, s[gap], e[gap], 1.0)
    s, e, v = _runs(res)
    short = (v == 1) & (e < n) & (e - s < min_speech)      # a speech run closed by silence
    _set_runs(res, s[short], e[short], 0.0)
    return res


def flags_to_mask(flags, n_samples: int, hop: int) -> np.ndarray:
    """Frame flags -> per-sample mask (the last frame clipped to the audio)."""
    f = np.asarray(flags, dtype=np.float32)
    mask = np.zeros(n_samples, dtype=np.float32)
    m = min(len(f) * hop, n_samples)
    mask[:m] = np.repeat(f, hop)[:m]
    return mask


def frame_energy(audio: np.ndarray, fs: int = 16000):
    win, hop = int(0.02 * fs), int(0.01 * fs)
    if win != 2 * hop:
        raise ValueError('energy track assumes 50% window overlap (16 kHz)')
    L = len(audio)
    n = (L - win) // hop + 1
    fe = np.zeros(L, dtype=np.float32)
    if n <= 0:
        return fe, n
    frames = sliding_window_view(audio, win)[::hop][:n]
    en = np.mean(frames ** 2, axis=1).astype(np.float32)
    c = np.maximum.accumulate(en)
    fe[:n * hop] = np.repeat(c, hop)
    fe[n * hop:(n - 1) * hop + win] = c[-1]
    return fe, n


def refine_boundaries(audio, vad_mask, fs=16000, energy_threshold=0.05, expansion_ms=10.0, percentile=10.0):
    refined = vad_mask.copy()
    fe, n = frame_energy(audio, fs)
    if n <= 0:
        return refined
    d = np.diff(np.concatenate(([0], vad_mask, [0])))
    starts, ends = np.where(d > 0)[0], np.where(d < 0)[0]
    if len(starts) == 0 or len(ends) == 0:
        return refined
    look = 10 * int(0.01 * fs)
    expand = int(expansion_ms * fs / 1000.0)
    floor = float(energy_threshold)
    for start, end in zip(starts.tolist(), ends.tolist()):
        if end <= start:
            continue
        th = max(np.percentile(fe[start:end], percentile), floor)
        new_start = start
        hit = np.flatnonzero(fe[start:min(end, start + look)] < th)
        if hit.size:
            new_start = start + int(hit[0])
            refined[start:new_start] = 0
        new_end = end
        lo = max(new_start, end - look) + 1
        if lo < end:
            hit = np.flatnonzero(fe[lo:end] < th)
            if hit.size:
                i = lo + int(hit[-1])
                refined[i:end] = 0
                new_end = i + 1
        if expand > 0:
            refined[max(start, new_start - expand):new_start] = 1
            refined[new_end:end] = 1
    return refined.astype(np.float32)


def mask_to_intervals(mask, fs=16000):
    if len(mask) == 0:
        return []
    d = np.diff(np.concatenate(([0], mask, [0])))
    starts, ends = np.where(d > 0)[0], np.where(d < 0)[0]
    return [[s / fs, e / fs] for s, e in zip(starts.tolist(), ends.tolist()) if e / fs > s / fs]


def flags_to_intervals(flags, n_samples, hop, fs=16000):
    """Raw flags -> [[st, ed]] seconds (``_flags_to_intervals``, infer_diarization.py:487-516)."""
    f = np.asarray(flags)
    if f.size == 0:
        return []
    s, e, v = _runs((f != 0).astype(np.int8))
    out = []
    for a, b in zip(s[v == 1].tolist(), e[v == 1].tolist()):
        st, ed = float(a * hop) / fs, float(min(b * hop, n_samples)) / fs
        if ed > st:
            out.append([st, ed])
    return out


def chunk(st, ed, dur=1.5, step=0.75):
    """Sliding sub-segments of one VAD segment; the last one clipped to ``ed``."""
    if ed - st <= 0:
        return []
    out = []
    s = st
    while s + dur < ed + step:
        out.append([s, min(s + dur, ed)])
        s += step
    return out or [[st, ed]]


def compressed_seg(seg_list):
    """Merge consecutive same-speaker segments; split overlaps between speakers at the midpoint."""
    out = []
    for st, ed, spk in seg_list:
        if not out:
            out.append([st, ed, spk])
        elif spk == out[-1][2]:
            if st > out[-1][1]:
                out.append([st, ed, spk])
            else:
                out[-1][1] = ed
        else:
            if st < out[-1][1]:
                mid = (out[-1][1] + st) / 2
                out[-1][1] = mid
                st = mid
            out.append([st, ed, spk])
    return out


def apply_mask(wav, mask):
    """Zero the non-speech samples (``_apply_vad_mask_from_mask``, infer_diarization.py:560-601)."""
    x = wav.detach().cpu().numpy() if hasattr(wav, 'detach') else np.asarray(wav)
    a = x[0] if x.ndim == 2 else x
    m = np.zeros(len(a), dtype=np.float32)
    k = min(len(mask), len(a))
    m[:k] = mask[:k]
    out = a * m
    return out.reshape(1, -1) if x.ndim == 2 else out
