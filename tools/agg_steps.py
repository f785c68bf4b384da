"""Aggregate a profile_steps.py JSON by layer type (layerN.*.name)."""
import collections
import json
import re
import sys

rows = json.load(open(sys.argv[1]))
cat = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in rows:
    key = re.sub(r'\.\d+\.', '.*.', r['step'])
    c = cat[key]
    c[0] += 1
    c[1] += r['ms']
    c[2] += r['tflops'] * r['ms']
tot = sum(r['ms'] for r in rows)
for k, (n, ms, tfms) in sorted(cat.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f"{ms:7.2f} ms {100 * ms / tot:5.1f}%  n={n:2d}  {tfms / ms if ms else 0:6.1f} TF  {k}")
