"""Instruction mix per basic block of one kernel in a hipcc -S listing (dev tool).

    python tools/isa_stats.py file.s <mangled-substring> [min_block_len]
"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(key) + r'\S*:', l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith('.Lfunc_end'))
    blocks, cur = [], None
    for l in lines[start:end]:
        if re.match(r'^(\.LBB\d+_\d+|_Z\S+):', l):
            cur = [l.split(':')[0], []]
            blocks.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith(';') or s.startswith('.') or cur is None:
            continue
        cur[1].append(s.split()[0])
    tot = collections.Counter()
    for lab, ins in blocks:
        c = collections.Counter()
        for op in ins:
            k = ('mfma' if 'mfma' in op else 'wait' if op.startswith('s_waitcnt') else 'valu' if op.startswith('v_')
                 else 'salu' if op.startswith('s_') else 'ds' if op.startswith('ds_')
                 else 'vmem' if op.startswith(('global_', 'buffer_')) else 'other')
            c[k] += 1
        tot += c
        if len(ins) >= minlen:
            print(f'{lab:12s} {len(ins):5d} {dict(c)}')
    print('total', dict(tot))


if __name__ == '__main__':
    main()
