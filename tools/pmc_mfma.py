"""MFMA utilisation per kernel from one rocprofv3 --pmc pass (SQ + GRBM counters).

Usage: python tools/pmc_mfma.py <pmc_dir> [-o out.json]

Per dispatch: cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs, MI355X_MICROARCH.md
'DVFS give-back'); MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs) (the
MFMA pipe's busy cycles summed over every SIMD; 32 per v_mfma_f32_32x32x16_f16).  Wave-state
fractions are SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (the
three are disjoint and cover the wave's life).  Aggregated per kernel over its dispatches
(cycle-weighted)."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r'([A-Za-z_0-9]+<[^()]*>)\s*\(', name)
    if m:
        return m.group(1)
    name = name.replace('(anonymous namespace)::', '')
    return name.split('(')[0].split('::')[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('pmc_dir')
    ap.add_argument('-o', '--out')
    a = ap.parse_args()
    disp = defaultdict(dict)
    names = {}
    for p in glob.glob(os.path.join(a.pmc_dir, '**', '*counter_collection.csv'), recursive=True):
        for row in csv.DictReader(open(p)):
            key = (p, row.get('Dispatch_Id'))
            names[key] = short(row['Kernel_Name'])
            disp[key][row['Counter_Name']] = disp[key].get(row['Counter_Name'], 0.0) + float(row['Counter_Value'])
    agg = defaultdict(lambda: defaultdict(float))
    for key, c in disp.items():
        k = names[key]
        for n, v in c.items():
            agg[k][n] += v
        agg[k]['dispatches'] += 1
    out = {}
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get('GRBM_GUI_ACTIVE', 0)):
        cyc = c.get('GRBM_GUI_ACTIVE', 0) / 8.0
        wc = c.get('SQ_WAVE_CYCLES', 0) or 1.0
        r = {'dispatches': int(c['dispatches']), 'gpu_cycles': cyc,
             'mfma_util': c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024) if cyc else None,
             'mfma_insts': c.get('SQ_INSTS_MFMA', 0), 'valu_insts': c.get('SQ_INSTS_VALU', 0),
             'valu_per_mfma': c.get('SQ_INSTS_VALU', 0) / c['SQ_INSTS_MFMA'] if c.get('SQ_INSTS_MFMA') else None,
             'wait_any_frac': c.get('SQ_WAIT_ANY', 0) / wc, 'wait_inst_any_frac': c.get('SQ_WAIT_INST_ANY', 0) / wc,
             'active_inst_any_frac': c.get('SQ_ACTIVE_INST_ANY', 0) / wc,
             'sq_busy_cycles': c.get('SQ_BUSY_CYCLES', 0)}
        out[k] = r
        mu = r['mfma_util']
        print(f"{k[:70]:70s} n={r['dispatches']:4d} cyc={cyc:.3e} mfma_util={mu if mu is None else round(mu, 3)} "
              f"valu/mfma={r['valu_per_mfma'] if r['valu_per_mfma'] is None else round(r['valu_per_mfma'], 2)} "
              f"wait={r['wait_any_frac']:.2f} stall={r['wait_inst_any_frac']:.2f} active={r['active_inst_any_frac']:.2f}")
    if a.out:
        json.dump({'counters': 'SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, SQ_INSTS_VALU, SQ_WAVE_CYCLES, SQ_WAIT_ANY, '
                               'SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE (one pass)',
                   'mfma_util_formula': 'SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)',
                   'kernels': out}, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
