"""Diagnostic: one B = 256 forward on one stream vs the same 256 utterances as S concurrent
sub-batches on S streams (own workspaces), wall time over N back-to-back forwards
(torch.cuda.synchronize on both sides).  Prints ms per 256 utterances per arm."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402

import helpers  # noqa: E402
from speakerlab import _hip  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else 'eres2netv2'
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
dev = torch.device('cuda', 0)
m = helpers.loaded_module(arch).to(dev).eval()
h = m._hip_handle(dev)
lib = _hip.lib()
B, T = 256, 198
x = torch.randn(B, T, 80, device=dev)
out = torch.empty(B, h.embed_dim, device=dev)


def arm(S):
    b = B // S
    streams = [torch.cuda.Stream(dev) for _ in range(S)]
    ws = [torch.empty(h.workspace_bytes(b, T), dtype=torch.uint8, device=dev) for _ in range(S)]
    xs = [x[i * b:(i + 1) * b].contiguous() for i in range(S)]

    def once():
        for i in range(S):
            _hip._check(lib.spk_model_forward(h.handle, xs[i].data_ptr(), b, T, ws[i].data_ptr(), ws[i].numel(),
                                              out[i * b:].data_ptr(), streams[i].cuda_stream), 'fwd')
    for _ in range(3):
        once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        once()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / N * 1e3


with torch.no_grad():
    res = {}
    for rep in range(2):
        for S in (1, 2, 4):
            res.setdefault(S, []).append(round(arm(S), 3))
    for S, v in res.items():
        print(f'{arch} streams={S} sub-batch={B // S}: ms per 256 utts {v}')
