"""Per-launch HBM bytes per kernel from two rocprofv3 ``--pmc`` passes (FETCH_SIZE, WRITE_SIZE).

Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> [-o profiles/pmc_traffic.json]

Pricing follows MI355X_MICROARCH.md §HBM: both counters are in KiB; on gfx950 FETCH_SIZE
reports half of the bytes of a wide coalesced read, so read bytes = 2 x FETCH_SIZE x 1024;
write bytes = WRITE_SIZE x 1024.  Kernel names are reduced to the template id the
executor reports (``conv_gemm_kernel<...>``) so bench.py can look them up.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short_name(name: str) -> str:
    m = re.search(r'([A-Za-z_0-9]+<[^()]*>)\s*\(', name)
    if m:
        return m.group(1)
    m = re.search(r'([A-Za-z_0-9]+)\s*\(', name)
    return m.group(1) if m else name


def per_dispatch(d, counter):
    vals = defaultdict(list)
    for path in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get('Counter_Name') != counter:
                    continue
                vals[short_name(row['Kernel_Name'])].append(float(row['Counter_Value']))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('-o', '--out', default='profiles/pmc_traffic.json')
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_dir, 'FETCH_SIZE')
    write = per_dispatch(a.write_dir, 'WRITE_SIZE')
    out = {}
    for k in sorted(set(fetch) & set(write)):
        rd = 2 * 1024 * sum(fetch[k]) / len(fetch[k])
        wr = 1024 * sum(write[k]) / len(write[k])
        out[k] = {'bytes_per_launch': rd + wr, 'read_bytes': rd, 'write_bytes': wr,
                  'dispatches': [len(fetch[k]), len(write[k])]}
    os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]['bytes_per_launch'])[:12]:
        print(f"{v['bytes_per_launch'] / 1e6:10.2f} MB/launch  {k}")


if __name__ == '__main__':
    main()
