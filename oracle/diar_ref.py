"""TEST INFRASTRUCTURE ONLY — scalar restatement of the diarization host pipeline.

Only ``tests/`` may import this module, as the checker for the vectorised product code in
``speakerlab/bin/infer_diarization.py``.  Every function follows the per-frame / per-sample
loops of the reference ``speakerlab/bin/infer_diarization.py`` literally (line numbers
cited) so that the product's numpy formulation can be checked for exact equality.

Parity pinned by construction (the reference module imports modelscope, which is absent
here, so it cannot be imported; the loops are restated from its source).
"""
import numpy as np


def post_process_speech_flags(flags, min_speech_ms=200.0, max_silence_ms=300.0, frame_ms=16.0):
    """``_post_process_speech_flags`` (infer_diarization.py:355-393)."""
    f = np.array(flags, dtype=np.float32)
    padded = np.pad(f, (1, 1), mode='edge')
    smooth = (np.convolve(padded, np.ones(3) / 3, mode='valid') > 0.5).astype(np.float32)
    min_speech = max(1, int(min_speech_ms / frame_ms))
    max_sil = max(1, int(max_silence_ms / frame_ms))
    res = smooth.copy()
    zeros = 0
    for i in range(len(res)):                     # fill short gaps (:377-384)
        if res[i] == 0:
            zeros += 1
        else:
            if 0 < zeros <= max_sil:
                res[i - zeros:i] = 1
            zeros = 0
    ones = 0
    for i in range(len(res)):                     # drop short speech (:386-393)
        if res[i] == 1:
            ones += 1
        else:
            if 0 < ones < min_speech:
                res[i - ones:i] = 0
            ones = 0
    return res


def flags_to_mask(flags, n_samples, hop):
    """processed_mask construction (infer_diarization.py:340-346)."""
    mask = np.zeros(n_samples, dtype=np.float32)
    for i, fl in enumerate(flags):
        mask[i * hop:min((i + 1) * hop, n_samples)] = fl
    return mask


def frame_energy(audio, fs=16000):
    """The energy track of ``_refine_vad_boundaries_with_energy`` (:403-413)."""
    win, hop = int(0.02 * fs), int(0.01 * fs)
    n = (len(audio) - win) // hop + 1
    fe = np.zeros(len(audio), dtype=np.float32)
    for i in range(max(n, 0)):
        s = i * hop
        e = min(s + win, len(audio))
        en = float(np.mean(audio[s:e] ** 2))
        fe[s:e] = max(fe[s:e].max(), en)
    return fe, n


def refine_boundaries(audio, vad_mask, fs=16000, energy_threshold=0.05, expansion_ms=10.0, percentile=10.0):
    """``_refine_vad_boundaries_with_energy`` (infer_diarization.py:395-461)."""
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
    for start, end in zip(starts, ends):
        seg = fe[start:end]
        if len(seg) == 0:
            continue
        th = max(np.percentile(seg, percentile), float(energy_threshold))
        new_start = start
        for i in range(start, min(end, start + look)):
            if fe[i] < th:
                refined[start:i] = 0
                new_start = i
                break
        new_end = end
        for i in range(end - 1, max(new_start, end - look), -1):
            if fe[i] < th:
                refined[i:end] = 0
                new_end = i + 1
                break
        if expand > 0:
            refined[max(start, new_start - expand):new_start] = 1
            refined[new_end:end] = 1
    return refined.astype(np.float32)


def mask_to_intervals(mask, fs=16000):
    """``_mask_to_intervals`` (infer_diarization.py:463-485)."""
    if len(mask) == 0:
        return []
    d = np.diff(np.concatenate(([0], mask, [0])))
    out = []
    for s, e in zip(np.where(d > 0)[0], np.where(d < 0)[0]):
        if float(e) / fs > float(s) / fs:
            out.append([float(s) / fs, float(e) / fs])
    return out


def chunk(st, ed, dur=1.5, step=0.75):
    """``Diarization3Dspeaker.chunk`` (infer_diarization.py:606-619)."""
    out = []
    if ed - st <= 0:
        return out
    s = st
    made = False
    while s + dur < ed + step:
        out.append([s, min(s + dur, ed)])
        s += step
        made = True
    if not made:
        out.append([st, ed])
    return out


def compressed_seg(segs):
    """``compressed_seg`` (infer_diarization.py:780-797)."""
    out = []
    for i, (st, ed, c) in enumerate(segs):
        if i == 0:
            out.append([st, ed, c])
        elif c == out[-1][2]:
            if st > out[-1][1]:
                out.append([st, ed, c])
            else:
                out[-1][1] = ed
        else:
            if st < out[-1][1]:
                p = (out[-1][1] + st) / 2
                out[-1][1] = p
                st = p
            out.append([st, ed, c])
    return out
