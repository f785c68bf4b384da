"""Diagnostic: the captured guarded forward's nodes and dependency edges.

Run once per word-reset arm (the env is read once per process):
    SPK_WORD_RESET=memset SPK_GRAPH_DOT=gpurun_out/g_memset.dot python tools/graph_dot_probe.py
    SPK_GRAPH_DOT=gpurun_out/g_kernel.dot python tools/graph_dot_probe.py
    python tools/graph_dot_probe.py --parse gpurun_out/g_memset.dot gpurun_out/g_kernel.dot

The first two capture one ERes2NetV2 forward (the runtime writes the graph with
hipGraphDebugDotPrint before instantiating it, runtime.cpp run_graph); --parse reads the DOT
files and reports, per graph: the root nodes, the word-reset node (the memset node, or the
first kernel node), its successors, and whether every other node is reachable from it -- i.e.
whether the reset precedes the first kernel node of its own plan in the graph's edges.
"""
import os
import re
import sys
from collections import defaultdict, deque

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def capture(arch='eres2netv2'):
    for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
        sys.path.insert(0, p)
    import torch
    import helpers
    g = helpers.golden(arch)
    dev = torch.device('cuda', 0)
    m = helpers.loaded_module(arch).to(dev).eval()
    with torch.no_grad():
        out = m(torch.from_numpy(g['feats2']).to(dev))
    torch.cuda.synchronize()
    print(f'captured {arch} forward {tuple(out.shape)} -> {os.environ.get("SPK_GRAPH_DOT")}')


def parse(path):
    txt = open(path).read()
    labels, edges = {}, []
    for m in re.finditer(r'^\s*"?([\w]+)"?\s*\[(.*?)\];?\s*$', txt, re.M | re.S):
        name, attrs = m.group(1), m.group(2)
        if name in ('graph', 'node', 'edge'):
            continue
        lab = re.search(r'label\s*=\s*"(.*?)"', attrs, re.S) or re.search(r'label\s*=\s*<(.*?)>\s*(,|$)', attrs, re.S)
        labels[name] = (lab.group(1) if lab else attrs)[:400]
    for m in re.finditer(r'"?([\w]+)"?\s*->\s*"?([\w]+)"?', txt):
        edges.append((m.group(1), m.group(2)))
    nodes = set(labels) | {a for a, _ in edges} | {b for _, b in edges}
    succ, npred = defaultdict(list), defaultdict(int)
    for a, b in edges:
        succ[a].append(b)
        npred[b] += 1
    roots = sorted(n for n in nodes if npred[n] == 0)

    def kind(n):
        lab = labels.get(n, '').lower()
        if 'memset' in lab:
            return 'memset'
        if 'kernel' in lab or 'func' in lab or '_z' in lab:
            return 'kernel'
        if 'memcpy' in lab:
            return 'memcpy'
        return 'other'

    def short(n):
        lab = labels.get(n, '')
        k = re.search(r'(_Z\w+|word_reset\w*|range_check\w*|stem_conv\w*)', lab)
        return f'{n} [{kind(n)}{": " + k.group(1)[:60] if k else ""}]'

    print(f'== {path}: {len(nodes)} nodes, {len(edges)} edges, roots: {[short(r) for r in roots]}')
    reset = next((n for n in nodes if kind(n) == 'memset'), None)
    if reset is None:   # the kernel-node reset: the root kernel whose label names the reset kernel
        reset = next((r for r in roots if 'reset' in labels.get(r, '').lower()), roots[0] if roots else None)
    print(f'   word-reset node: {short(reset)}; successors: {[short(s) for s in succ[reset]]}')
    seen, q = {reset}, deque([reset])
    while q:
        for s in succ[q.popleft()]:
            if s not in seen:
                seen.add(s)
                q.append(s)
    print(f'   nodes reachable from the reset: {len(seen) - 1} of {len(nodes) - 1} others; '
          f'single root: {len(roots) == 1}; reset precedes every node: {len(seen) == len(nodes)}')
    return len(seen) == len(nodes)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == '--parse':
        ok = [parse(p) for p in sys.argv[2:]]
        print('all resets precede their plans:', all(ok))
    else:
        capture(sys.argv[1] if len(sys.argv) > 1 else 'eres2netv2')
