"""Per-step timing of one launch plan (HIP events around every step), printed as a table.

    python tools/profile_steps.py [--arch eres2netv2] [--batch 256] [--frames 198]

Columns: step, kernel, ms, algorithmic TFLOP/s, share of the forward.  Used to pick the
next kernel to optimise; bench.py reports the roofline of the dominant kernel.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arch', default='eres2netv2')
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--frames', type=int, default=198)
    ap.add_argument('--json', default='')
    args = ap.parse_args()
    import helpers
    dev = torch.device('cuda', 0)
    m = helpers.loaded_module(args.arch).to(dev)
    h = m._hip_handle(dev)
    x = torch.randn(args.batch, args.frames, 80, device=dev)
    out = torch.empty(args.batch, h.embed_dim, device=dev)
    plan = h.plan(args.batch, args.frames)
    for _ in range(3):
        ms = h.forward_timed(x, out)
    tot = sum(ms)
    rows = []
    for (name, kern, fl), t in zip(plan, ms):
        rows.append({'step': name, 'kernel': kern, 'ms': t, 'tflops': fl / (t * 1e-3) / 1e12 if t > 0 else 0.0,
                     'share': t / tot})
    print(f'{args.arch} B={args.batch} T={args.frames}: {tot:.3f} ms/forward, {len(rows)} steps, '
          f'{args.batch / tot * 1e3:.1f} utt/s')
    for r in sorted(rows, key=lambda r: -r['ms'])[:40]:
        print(f"{r['ms']:8.3f} ms {100 * r['share']:5.1f}% {r['tflops']:7.1f} TF  {r['step']:<34} {r['kernel']}")
    if args.json:
        with open(args.json, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
