"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (sums over dispatches).

Usage: python tools/pmc_sq.py <pmc_dir> [kernel-substring ...]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r'([A-Za-z_0-9]+<[^()]*>)\s*\(', name)
    return m.group(1) if m else name.split('(')[0]


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    agg = defaultdict(lambda: defaultdict(float))
    nd = defaultdict(set)
    for p in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(p)):
            k = short(row['Kernel_Name'])
            agg[k][row['Counter_Name']] += float(row['Counter_Value'])
            nd[k].add(row.get('Dispatch_Id'))
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_WAVE_CYCLES', 0)):
        if keys and not any(s in k for s in keys):
            continue
        wc = c.get('SQ_WAVE_CYCLES', 0) or 1
        parts = ', '.join(f'{n}={v / wc:.3f}' for n, v in sorted(c.items()) if n != 'SQ_WAVE_CYCLES')
        print(f'{k}  [{len(nd[k])} disp]  wave_cycles={wc:.3e}  {parts}')


if __name__ == '__main__':
    main()
