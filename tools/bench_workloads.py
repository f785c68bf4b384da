"""Secondary workloads of BASELINE.json (reported next to the headline, not the bench line).

  c3   CAM++ (7.2 M) batch=1024 variable-length 1-5 s segments (lengths ~U{16000..80000},
       seed 2), GPU Fbank + embedding.  Utterances are sorted by length and
       cut into sub-batches padded to their own longest member (per-utterance lengths mask
       the rest, spk_model_forward_lengths): every embedding is that of the utterance alone.
  c1   ECAPA-TDNN batch=32 2 s (the reference's CPU config, here on the GPU).
  models  every architecture at B=256, 2 s.

    python tools/bench_workloads.py c3 [--steps K] [--warmup W] [--buckets 4] [--precision fp32|fp16]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, '3d-speaker_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(step, steps, warmup):
    with torch.no_grad():
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = step()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def load(arch, device):
    sys.path.insert(0, os.path.join(REPO, 'tests'))
    import helpers
    return helpers.loaded_module(arch).to(device).eval()


def c3_setup(device, precision='fp32', nbuckets=4, n=1024):
    """The C3 batch and its bucketed forward (also driven by tests/test_gpu_c3_full.py):
    returns (step, lens, order, host, model); step() gives the embeddings of the utterances in
    length order, row i = utterance order[i] (waveform host[i, :lens[order[i]]])."""
    from speakerlab import _hip
    from speakerlab.utils import synthetic
    rng = np.random.Generator(np.random.PCG64(2))
    lens = rng.integers(16000, 80001, size=n)
    order = np.argsort(lens, kind='stable')
    lens_sorted = lens[order]
    L = int(lens.max())
    host = np.zeros((n, L), np.float32)
    for i, j in enumerate(order):
        host[i, :lens_sorted[i]] = synthetic.synth_wav(int(lens_sorted[i]), seed=2_000_000 + int(j))
    wavs = torch.from_numpy(host).to(device)
    model = load('campplus', device).set_hip_precision(precision)
    bounds = np.linspace(0, n, nbuckets + 1).astype(int)
    buckets = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        lmax = int(lens_sorted[b - 1])
        buckets.append((a, b, lmax, [int(v) for v in lens_sorted[a:b]]))

    def step():
        outs = []
        for a, b, lmax, ls in buckets:
            feats, frames = _hip.fbank_padded(wavs[a:b, :lmax], ls, 80, mean_nor=True)
            outs.append(model(feats, lengths=frames))
        return torch.cat(outs)

    return step, lens, order, host, model


def c3(args, device):
    step, lens, order, host, model = c3_setup(device, args.precision, args.buckets)
    n = len(lens)
    dt, emb = timed(step, args.steps, args.warmup)
    assert torch.isfinite(emb).all()
    audio_s = float(lens.sum()) / 16000
    frames = sum(1 + (int(v) - 400) // 160 for v in lens)
    flops = model._hip_handle(device).flops(198) / 198 * frames   # ~linear in frames
    return {'workload': 'c3', 'model': 'CAM++(512)', 'utterances': n, 'buckets': args.buckets,
            'lengths': '1-5 s ~U{16000..80000} samples, seed 2', 'ms_per_step': round(dt * 1e3, 3),
            'value': round(n / dt, 1), 'unit': 'utt/s (variable length)',
            'two_s_equivalent_per_s': round(audio_s / 2 / dt, 1), 'approx_tflops': round(flops / dt / 1e12, 2),
            'dtype': 'f32 (fp16x3 MFMA)' if args.precision == 'fp32' else
            'fp16 single-product MFMA, fp32 accumulate (C3 reduced-precision mode)', 'data': 'synthetic'}


def c1(args, device):
    from speakerlab import _hip
    from speakerlab.utils import synthetic
    wavs = torch.from_numpy(synthetic.pcm16_batch(32, 32000, seed=0)).to(device)
    model = load('ecapa', device)
    dt, _ = timed(lambda: model(_hip.fbank(wavs, 80, mean_nor=True)), args.steps, args.warmup)
    return {'workload': 'c1', 'model': 'ECAPA-TDNN', 'batch': 32, 'ms_per_step': round(dt * 1e3, 3),
            'value': round(32 / dt, 1), 'unit': 'utt/s (2 s)', 'data': 'synthetic'}


def models(args, device):
    from speakerlab import _hip
    from speakerlab.utils import synthetic
    wavs = torch.from_numpy(synthetic.pcm16_batch(256, 32000, seed=1)).to(device)
    out = []
    for arch in ('eres2netv2', 'eres2net_large', 'ecapa', 'campplus'):
        model = load(arch, device)
        dt, _ = timed(lambda: model(_hip.fbank(wavs, 80, mean_nor=True)), args.steps, args.warmup)
        out.append({'workload': 'b256_2s', 'model': arch, 'ms_per_step': round(dt * 1e3, 3),
                    'value': round(256 / dt, 1), 'unit': 'utt/s (2 s, GPU Fbank + embedding)'})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('workload', choices=['c3', 'c1', 'models'])
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--buckets', type=int, default=4)
    ap.add_argument('--precision', choices=['fp32', 'fp16'], default='fp32',
                    help="c3: 'fp16' = the single-product mode (set_hip_precision)")
    args = ap.parse_args()
    device = torch.device('cuda', 0)
    torch.cuda.set_device(device)
    res = {'c3': c3, 'c1': c1, 'models': models}[args.workload](args, device)
    for r in res if isinstance(res, list) else [res]:
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
