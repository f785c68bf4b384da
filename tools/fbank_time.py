"""Time the GPU Fbank front end alone (bench.fbank_roofline) at B = 256 x 2 s and a ragged
C3-like batch; prints one JSON line per case."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-speaker_amd')]
import torch  # noqa: E402

import bench  # noqa: E402
from speakerlab.utils import synthetic  # noqa: E402

dev = torch.device('cuda', 0)
for B, L in [(256, 32000), (1024, 32000), (64, 80000)]:
    wavs = torch.from_numpy(synthetic.pcm16_batch(B, L, seed=1)).to(dev)
    r = bench.fbank_roofline(wavs, dev)
    print(json.dumps(dict(B=B, samples=L, **r)), flush=True)
