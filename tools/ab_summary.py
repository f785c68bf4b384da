"""Summarise tools/gpu_run.sh PHASE=ab output: per build, per rep, the forward and the per-kernel-family totals.
    python tools/ab_summary.py TAG lib1 lib2 ... [--archs a,b] [--top 8]"""
import argparse
import collections
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument('tag')
ap.add_argument('libs', nargs='+')
ap.add_argument('--archs', default='eres2netv2')
ap.add_argument('--top', type=int, default=8)
ap.add_argument('--reps', type=int, default=2)
a = ap.parse_args()
for arch in a.archs.split(','):
    for lib in a.libs:
        for rep in range(1, a.reps + 1):
            f = f'gpurun_out/{a.tag}_ab_libspk_{lib}_{arch}_{rep}.json'
            if not os.path.exists(f):
                print('missing', f)
                continue
            steps = json.load(open(f))
            fam = collections.defaultdict(float)
            for x in steps:
                fam[x['kernel'].split('<')[0]] += x['ms']
            top = sorted(fam.items(), key=lambda kv: -kv[1])[:a.top]
            print(f'{arch:12s} {lib:10s} rep{rep}: {sum(x["ms"] for x in steps):7.3f} ms |',
                  ' '.join(f'{k}={v:.3f}' for k, v in top))
