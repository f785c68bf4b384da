"""Generate tests/golden/der_golden.json by scoring synthetic RTTM pairs with the
REFERENCE DER tool (``egs/3dspeaker/speaker-diarization/local/DER.py`` driving its
``md-eval.pl`` under /usr/bin/perl), read-only from /root/reference.  Build container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_der_golden.py

Cases: several recordings with overlapping reference speech, system outputs with
boundary jitter, speaker confusions, an extra system speaker, missed and false-alarm
stretches (inside and outside the reference span), and an empty system file.  The
fixture holds the RTTM text of every case and the reference's (MS, FA, SER, DER).
"""
import importlib.util
import json
import os
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LOCAL = '/root/reference/egs/3dspeaker/speaker-diarization/local'


def rttm(file, segs):
    return [f'SPEAKER {file} 0 {b:.3f} {e - b:.3f} <NA> <NA> {s} <NA> <NA>' for b, e, s in segs if e > b]


def synth_ref(rng, n_spk, dur, overlap):
    segs, t = [], float(rng.uniform(0, 2))
    while t < dur:
        d = float(rng.uniform(0.5, 6))
        s = int(rng.integers(n_spk))
        segs.append((round(t, 3), round(min(dur, t + d), 3), f'r{s}'))
        if rng.random() < overlap:     # overlapping second speaker
            o = (s + 1 + int(rng.integers(n_spk - 1))) % n_spk
            a = t + float(rng.uniform(0, d))
            segs.append((round(a, 3), round(min(dur, a + float(rng.uniform(0.2, 2))), 3), f'r{o}'))
        t += d + float(rng.uniform(0, 1.5))
    return segs


def synth_sys(rng, ref, n_spk, confuse, extra):
    perm = rng.permutation(n_spk + 1)
    out = []
    for b, e, s in ref:
        if rng.random() < 0.05:
            continue                                            # missed segment
        k = int(s[1:])
        lab = perm[k] if rng.random() > confuse else perm[(k + 1) % n_spk]
        jb, je = rng.normal(0, 0.15, 2)
        out.append((round(max(0.0, b + jb), 3), round(e + je, 3), f's{lab}'))
    for _ in range(extra):                                      # false alarms / extra speaker
        a = float(rng.uniform(0, ref[-1][1] + 5))
        out.append((round(a, 3), round(a + float(rng.uniform(0.3, 3)), 3), f's{perm[n_spk]}'))
    return out


def main():
    spec = importlib.util.spec_from_file_location('ref_DER', os.path.join(LOCAL, 'DER.py'))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.Generator(np.random.PCG64(7))
    cases = []
    for c in range(8):
        ref_lines, sys_lines = [], []
        for f in range(1 + c % 3):
            n_spk = int(rng.integers(2, 6))
            ref = synth_ref(rng, n_spk, float(rng.uniform(60, 240)), overlap=0.3 if c % 2 else 0.0)
            fid = f'rec{c}_{f}'
            ref_lines += rttm(fid, ref)
            if c == 5 and f == 0:
                continue                                         # no system output for this file
            sys_lines += rttm(fid, synth_sys(rng, ref, n_spk, confuse=0.1 * (c % 4), extra=c % 3))
        with tempfile.TemporaryDirectory() as d:
            rp, sp = os.path.join(d, 'ref.rttm'), os.path.join(d, 'sys.rttm')
            open(rp, 'w').write('\n'.join(ref_lines) + '\n')
            open(sp, 'w').write('\n'.join(sys_lines) + '\n')
            ms, fa, ser, der = mod.DER(rp, sp)
        cases.append({'ref': ref_lines, 'sys': sys_lines,
                      'MS': float(ms), 'FA': float(fa), 'SER': float(ser), 'DER': float(der)})
        print(c, len(ref_lines), len(sys_lines), f'DER {float(der):.4f}')
    with open(os.path.join(HERE, 'der_golden.json'), 'w') as f:
        json.dump({'source': 'reference DER.py + md-eval.pl (collar 0, overlap scored)', 'cases': cases}, f)


if __name__ == '__main__':
    main()
