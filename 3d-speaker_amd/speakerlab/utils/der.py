"""Diarization error rate exactly as the reference recipe scores it (config C5's "DER vs ref").

The reference computes DER with ``egs/3dspeaker/speaker-diarization/local/DER.py:38-153``,
which runs NIST ``md-eval.pl`` (``-af -r REF -s SYS -c 0``, overlap scored) and parses its
overall SCORED / MISSED / FALARM SPEAKER TIME and SPEAKER ERROR TIME (printed ``%f``,
``md-eval.pl:2437-2440``).  This is a restatement of that scoring path for SPEAKER-type
RTTMs (what ``infer_diarization`` writes):

* evaluation span per file = [earliest, latest] reference SPEAKER token
  (``uem_from_rttm``, ``md-eval.pl:2277-2289``);
* the time line is cut at every reference / system segment boundary
  (``create_speaker_segs``, ``md-eval.pl:2293-2345``; zero-length segments dropped,
  END before BEG at equal times);
* reference speakers are mapped one-to-one onto system speakers so that the summed
  co-speaking time is maximal (``map_speakers`` / ``weighted_bipartite_graph_match``,
  ``md-eval.pl:2494-2507, 2708-``; any maximum matching gives the same totals);
* per segment of duration d with n_ref / n_sys active speakers and n_map mapped pairs
  both active: scored += d*n_ref, missed += d*max(n_ref-n_sys, 0),
  falarm += d*max(n_sys-n_ref, 0), error += d*(min(n_ref, n_sys) - n_map)
  (``score_speaker_segments``, ``md-eval.pl:1995-2036``);
* percentages = 100 x time / scored, NaN -> 0, inf -> 100 (``DER.py:23-33``).

Pinned against the reference's own md-eval.pl + DER.py on committed RTTM fixtures
(``tests/golden/der_golden.json``, ``tests/test_der.py``).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, Iterable, List, Sequence, Tuple

import numpy as np
from scipy.optimize import linear_sum_assignment

Seg = Tuple[float, float, str]          # (tbeg, tend, speaker)


def parse_rttm(lines: Iterable[str]) -> Dict[Tuple[str, str], List[Seg]]:
    """SPEAKER lines -> {(file, channel): [(tbeg, tend, speaker)]}."""
    out: Dict[Tuple[str, str], List[Seg]] = defaultdict(list)
    for ln in lines:
        f = ln.split()
        if len(f) < 8 or f[0] != 'SPEAKER':
            continue
        tbeg, tdur = float(f[3]), float(f[4])
        out[(f[1], f[2])].append((tbeg, tbeg + tdur, f[7]))
    return out


def _segments(uem: Tuple[float, float], ref: Sequence[Seg], sys: Sequence[Seg]):
    events = [(uem[0], 1, 'U', None), (uem[1], 0, 'U', None)]
    for kind, segs in (('R', ref), ('S', sys)):
        for b, e, s in segs:
            if e - b > 0:
                events.append((b, 1, kind, s))
                events.append((e, 0, kind, s))
    events.sort(key=lambda ev: (ev[0], ev[1]))      # END (0) before BEG (1) at equal times
    cnt = {'R': defaultdict(int), 'S': defaultdict(int)}
    evaluating, tbeg, out = False, 0.0, []
    for t, beg, kind, spk in events:
        if evaluating and tbeg < t:
            out.append((t - tbeg, frozenset(cnt['R']), frozenset(cnt['S'])))
            tbeg = t
        if kind == 'U':
            evaluating = bool(beg)
            if evaluating:
                tbeg = t
        else:
            c = cnt[kind]
            c[spk] += 1 if beg else -1
            if not c[spk]:
                del c[spk]
    return out


def score_file(ref: Sequence[Seg], sys: Sequence[Seg]) -> Dict[str, float]:
    uem = (min(b for b, _, _ in ref), max(e for _, e, _ in ref))
    segs = _segments(uem, ref, sys)
    rspk = sorted({s for _, r, _ in segs for s in r})
    sspk = sorted({s for _, _, q in segs for s in q})
    ri = {s: i for i, s in enumerate(rspk)}
    si = {s: i for i, s in enumerate(sspk)}
    ov = np.zeros((len(rspk), len(sspk)))
    for d, r, q in segs:
        if r:
            for a in r:
                for b in q:
                    ov[ri[a], si[b]] += d
    mapping = {}
    if ov.size:
        rows, cols = linear_sum_assignment(ov, maximize=True)
        mapping = {rspk[i]: sspk[j] for i, j in zip(rows, cols)}
    st = dict(scored=0.0, missed=0.0, falarm=0.0, error=0.0)
    for d, r, q in segs:
        nr, ns = len(r), len(q)
        nmap = sum(1 for a in r if mapping.get(a) in q)
        st['scored'] += d * nr
        st['missed'] += d * max(nr - ns, 0)
        st['falarm'] += d * max(ns - nr, 0)
        st['error'] += d * (min(nr, ns) - nmap)
    return st


def der(ref_lines: Iterable[str], sys_lines: Iterable[str]) -> Dict[str, float]:
    """Overall MS / FA / SER / DER in percent of scored speaker time, like the reference's
    ``DER(ref_rttm, sys_rttm)`` with its defaults (collar 0, overlap scored)."""
    ref, sys = parse_rttm(ref_lines), parse_rttm(sys_lines)
    tot = dict(scored=0.0, missed=0.0, falarm=0.0, error=0.0)
    for key in sorted(ref):
        st = score_file(ref[key], sys.get(key, []))
        for k in tot:
            tot[k] += st[k]
    tot = {k: float(f'{v:f}') for k, v in tot.items()}          # md-eval prints %f

    def pct(x):
        with np.errstate(invalid='ignore', divide='ignore'):
            v = np.float64(x) / np.float64(tot['scored'])
        return 0.0 if np.isnan(v) else (100.0 if np.isinf(v) else float(v * 100.0))
    return {'MS': pct(tot['missed']), 'FA': pct(tot['falarm']), 'SER': pct(tot['error']),
            'DER': pct(tot['missed'] + tot['falarm'] + tot['error']), 'scored_speaker_time': tot['scored']}
