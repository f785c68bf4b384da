"""Diagnostic: which sequence raises the range word of a workspace (graph replays, exact-only
forwards in between), and which plan step raises it first."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402

import helpers  # noqa: E402
from speakerlab import _hip  # noqa: E402

arch = sys.argv[1] if len(sys.argv) > 1 else 'eres2netv2'
g = helpers.golden(arch)
dev = torch.device('cuda', 0)
m = helpers.loaded_module(arch).to(dev).eval()
h = m._hip_handle(dev)
x = torch.from_numpy(g['feats0']).to(dev).contiguous()
B, T, _ = x.shape
lib = _hip.lib()
S = torch.cuda.Stream(dev)
st = S.cuda_stream
W = torch.zeros(h.workspace_bytes(B, T), dtype=torch.uint8, device=dev)
out = torch.empty(B, h.embed_dim, device=dev)


def fwd(exact=False):
    f = lib.spk_model_forward_exact if exact else None
    if exact:
        _hip._check(lib.spk_model_forward_exact(h.handle, x.data_ptr(), B, T, None, W.data_ptr(), W.numel(),
                                                out.data_ptr(), st), 'ex')
    else:
        _hip._check(lib.spk_model_forward(h.handle, x.data_ptr(), B, T, W.data_ptr(), W.numel(), out.data_ptr(), st),
                    'fwd')
    torch.cuda.synchronize()


def word():
    v = ctypes.c_int32(-1)
    _hip._check(lib.spk_model_range_check(h.handle, B, T, 0, W.data_ptr(), st, ctypes.byref(v)), 'rc')
    return v.value


with torch.no_grad():
    fwd(); print('fresh ws, fwd 1: word', word())
    fwd(); print('fwd 2: word', word())
    fwd(exact=True); print('exact-only fwd: word', word())
    fwd(); print('fwd 3 after exact: word', word())
    fwd(); print('fwd 4: word', word())
    W.zero_()
    fwd(); print('ws zeroed, fwd 5: word', word())
    fwd(exact=True)
    # per step: the fp16x3 plan's steps one by one (timed forward: x3 plan only, flag in ws)
    plan = h.plan(B, T)
    n = len(plan)
    ms = (ctypes.c_float * n)()
    _hip._check(lib.spk_model_forward_timed(h.handle, x.data_ptr(), B, T, W.data_ptr(), W.numel(), out.data_ptr(),
                                            st, ms, n), 'timed')
    torch.cuda.synchronize()
    print('timed x3 plan after exact-only: word', word(), 'nan', bool(torch.isnan(out).any()))
    print('steps:', [p[0] for p in plan][:5], '...', n)
