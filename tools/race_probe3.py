"""Diagnostic: (1) each plan run sequentially after a LDS-poisoning kernel stream (NaN and
1e30 fill of all LDS), (2) concurrent replay with the poisoner on a second stream; compare
with the clean result and report the range word."""
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
pz = ctypes.CDLL(os.path.join(REPO, 'tools', 'diag', 'liblds_poison.so'))
pz.lds_poison.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int]
x = torch.from_numpy(g['feats0']).to(dev).contiguous()
B, T, _ = x.shape
S0, S1 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
W = torch.zeros(h.workspace_bytes(B, T), dtype=torch.uint8, device=dev)


def fwd(out, st):
    _hip._check(lib.spk_model_forward(h.handle, x.data_ptr(), B, T, W.data_ptr(), W.numel(), out.data_ptr(), st), 'f')


def word(st):
    v = ctypes.c_int32(-1)
    _hip._check(lib.spk_model_range_check(h.handle, B, T, 0, W.data_ptr(), st, ctypes.byref(v)), 'rc')
    return v.value


with torch.no_grad():
    ref = torch.empty(B, h.embed_dim, device=dev)
    fwd(ref, S0.cuda_stream)
    torch.cuda.synchronize()
    print('clean word', word(S0.cuda_stream))
    for val in (float('nan'), 1e30, -7.0):
        out = torch.empty_like(ref)
        pz.lds_poison(S0.cuda_stream, val, 2048, 4)
        fwd(out, S0.cuda_stream)
        torch.cuda.synchronize()
        print(f'sequential after poison {val}: word {word(S0.cuda_stream)} max|d| {float((out - ref).abs().max()):.3e}')
        out = torch.empty_like(ref)
        pz.lds_poison(S1.cuda_stream, val, 4096, 400)
        fwd(out, S0.cuda_stream)
        torch.cuda.synchronize()
        print(f'concurrent with poison {val}: word {word(S0.cuda_stream)} max|d| {float((out - ref).abs().max()):.3e}',
              flush=True)

    # where is the stuck state?
    f = W.view(torch.float32)
    nan = torch.isnan(f).nonzero().flatten()
    big = (f.abs() >= 16384).nonzero().flatten()
    print('NaN floats in ws:', int(nan.numel()), 'first/last byte offsets',
          (int(nan[0]) * 4, int(nan[-1]) * 4) if nan.numel() else None)
    print('|x|>=16384 floats in ws:', int(big.numel()),
          (int(big[0]) * 4, int(big[-1]) * 4) if big.numel() else None, 'ws bytes', W.numel())
    if nan.numel():
        # contiguous runs of NaN (byte ranges)
        idx = nan.cpu()
        starts = [int(idx[0])]
        ends = []
        for a, b in zip(idx[:-1].tolist(), idx[1:].tolist()):
            if b != a + 1:
                ends.append(a); starts.append(b)
        ends.append(int(idx[-1]))
        print('NaN runs (first 20, byte ranges):', [(s * 4, (e + 1) * 4) for s, e in list(zip(starts, ends))[:20]],
              'n runs', len(starts))
    out = torch.empty_like(ref)
    fwd(out, S0.cuda_stream); torch.cuda.synchronize()
    print('again: word', word(S0.cuda_stream))
    W.zero_()
    fwd(out, S0.cuda_stream); torch.cuda.synchronize()
    print('after W.zero_(): word', word(S0.cuda_stream), 'max|d|', float((out - ref).abs().max()))

    # bisect the first fp16x3 step that raises the word (prefix runs, word zeroed before each)
    lib.spk_diag_run_prefix.restype = ctypes.c_int
    lib.spk_diag_run_prefix.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
                                        ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    plan = h.plan(B, T)
    names = [p[0] for p in plan]
    first = None
    for k in range(1, len(plan) + 1):
        fwd(out, S0.cuda_stream)     # make sure the word slot exists / plan built
        torch.cuda.synchronize()
        # zero the word: it is the only int32 the range check reads
        v = ctypes.c_int32(0)
        wb = W.view(torch.int32)
        # find the word offset: run a guarded forward on zeros? simpler: zero all, then prefix
        W.zero_()
        rc = lib.spk_diag_run_prefix(h.handle, x.data_ptr(), B, T, W.data_ptr(), W.numel(), out.data_ptr(),
                                     S0.cuda_stream, k, 0)
        torch.cuda.synchronize()
        assert rc == 0, lib.spk_last_error()
        w = word(S0.cuda_stream)
        if w:
            first = k
            break
    print('first flagging prefix:', first, names[first - 1] if first else None, plan[first - 1][1] if first else None)
    if first:
        o = torch.empty_like(ref)
        f = W.view(torch.float32)
        print('ws max |x| after that prefix:', float(f.abs().max()), 'nan', int(torch.isnan(f).sum()))
