"""Diagnostic: graph replays of one shape with DIFFERENT inputs in sequence vs direct launches
of the same plan (spk_diag_run_prefix over all steps)."""
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
lib = _hip.lib()
lib.spk_diag_run_prefix.restype = ctypes.c_int
lib.spk_diag_run_prefix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                    ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
xa = torch.from_numpy(g['feats0']).to(dev).contiguous()
xb = (xa.flip(1) * 0.9 + 0.1).contiguous()
B, T, _ = xa.shape
st = torch.cuda.current_stream(dev).cuda_stream
W = torch.zeros(h.workspace_bytes(B, T), dtype=torch.uint8, device=dev)
W2 = torch.zeros_like(W)
n = len(h.plan(B, T))


def graph(x):
    out = torch.empty(B, h.embed_dim, device=dev)
    _hip._check(lib.spk_model_forward(h.handle, x.data_ptr(), B, T, W.data_ptr(), W.numel(), out.data_ptr(), st), 'f')
    torch.cuda.synchronize()
    return out


def direct(x):
    out = torch.empty(B, h.embed_dim, device=dev)
    W2.zero_()
    assert lib.spk_diag_run_prefix(h.handle, x.data_ptr(), B, T, W2.data_ptr(), W2.numel(), out.data_ptr(), st, 100000,
                                   0) == 0
    torch.cuda.synchronize()
    return out


with torch.no_grad():
    da, db = direct(xa), direct(xb)
    print('direct a vs b max|d|', float((da - db).abs().max()))
    seq = [('a', xa, da), ('b', xb, db), ('a', xa, da), ('b', xb, db), ('b', xb, db), ('a', xa, da)]
    for name, x, ref in seq:
        o = graph(x)
        print(f'graph {name}: max|d| vs direct {float((o - ref).abs().max()):.3e}', flush=True)
    W.zero_()
    o = graph(xa)
    print(f'graph a after W.zero_: max|d| vs direct {float((o - da).abs().max()):.3e}', flush=True)
