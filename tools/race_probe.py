"""Diagnostic: forwards of one handle on two streams at once vs the same forwards run alone.
Reports, per stream, whether the concurrent result equals the isolated fp16x3 result and/or
the exact-fp32 result, the range words, and the max |diff|."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import helpers  # noqa: E402
from speakerlab import _hip  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else 'eres2netv2'
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = helpers.golden(arch)
dev = torch.device('cuda', 0)
m = helpers.loaded_module(arch).to(dev).eval()
h = m._hip_handle(dev)
xs = [torch.from_numpy(g[f'feats{i}']).to(dev).contiguous() for i in range(2)]
lib = _hip.lib()


def fwd(x, ws, out, stream, exact=False):
    B, T, _ = x.shape
    f = lib.spk_model_forward_exact if exact else None
    if exact:
        _hip._check(f(h.handle, x.data_ptr(), B, T, None, ws.data_ptr(), ws.numel(), out.data_ptr(), stream), 'ex')
    else:
        _hip._check(lib.spk_model_forward(h.handle, x.data_ptr(), B, T, ws.data_ptr(), ws.numel(), out.data_ptr(),
                                          stream), 'fwd')


def word(x, ws, stream):
    B, T, _ = x.shape
    v = ctypes.c_int32(-1)
    _hip._check(lib.spk_model_range_check(h.handle, B, T, 0, ws.data_ptr(), stream, ctypes.byref(v)), 'rc')
    return v.value


with torch.no_grad():
    S = [torch.cuda.Stream(dev) for _ in range(2)]
    W = [torch.empty(h.workspace_bytes(*x.shape[:2]), dtype=torch.uint8, device=dev) for x in xs]
    alone = [torch.empty(x.shape[0], h.embed_dim, device=dev) for x in xs]
    exact = [torch.empty(x.shape[0], h.embed_dim, device=dev) for x in xs]
    for i in range(2):
        fwd(xs[i], W[i], alone[i], S[i].cuda_stream)
        torch.cuda.synchronize()
        print(f'stream {i} alone: range word {word(xs[i], W[i], S[i].cuda_stream)}')
        fwd(xs[i], W[i], exact[i], S[i].cuda_stream, exact=True)
        torch.cuda.synchronize()
    print('alone vs exact max|d|', [float((alone[i] - exact[i]).abs().max()) for i in range(2)])
    bad = 0
    for r in range(reps):
        outs = [torch.empty_like(a) for a in alone]
        for i in range(2):
            fwd(xs[i], W[i], outs[i], S[i].cuda_stream)
        torch.cuda.synchronize()
        for i in range(2):
            d = float((outs[i] - alone[i]).abs().max())
            de = float((outs[i] - exact[i]).abs().max())
            w = word(xs[i], W[i], S[i].cuda_stream)
            if d != 0:
                bad += 1
            print(f'rep {r} stream {i}: |d alone| {d:.3e} |d exact| {de:.3e} word {w}')
    print('MISMATCHES', bad)
