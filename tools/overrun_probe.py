"""Diagnostic: does a forward write outside its workspace / output?  The workspace and the
output are carved out of larger buffers filled with a canary byte pattern; after the
forward every canary byte must be intact."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')):
    sys.path.insert(0, p)
import torch  # noqa: E402

import helpers  # noqa: E402
from speakerlab import _hip  # noqa: E402

G = 8 << 20   # guard bytes on each side
dev = torch.device('cuda', 0)
lib = _hip.lib()
archs = sys.argv[1:] or ['eres2netv2']
for arch in archs:
    g = helpers.golden(arch)
    m = helpers.loaded_module(arch).to(dev).eval()
    h = m._hip_handle(dev)
    for i in range(3):
        x = torch.from_numpy(g[f'feats{i}']).to(dev).contiguous()
        B, T, _ = x.shape
        need = h.workspace_bytes(B, T)
        big = torch.full((need + 2 * G,), 0x5A, dtype=torch.uint8, device=dev)
        obig = torch.full((B * h.embed_dim + 2 * 4096,), 12345.0, dtype=torch.float32, device=dev)
        ws = big[G:G + need]
        out = obig[4096:4096 + B * h.embed_dim]
        for exact in (False, True):
            fn = lib.spk_model_forward_exact if exact else None
            if exact:
                rc = lib.spk_model_forward_exact(h.handle, x.data_ptr(), B, T, None, ws.data_ptr(), need,
                                                 out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            else:
                rc = lib.spk_model_forward(h.handle, x.data_ptr(), B, T, ws.data_ptr(), need, out.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert rc == 0, lib.spk_last_error()
            pre = (big[:G] != 0x5A).nonzero()
            post = (big[G + need:] != 0x5A).nonzero()
            opre = (obig[:4096] != 12345.0).nonzero()
            opost = (obig[4096 + B * h.embed_dim:] != 12345.0).nonzero()
            print(f'{arch} B={B} T={T} exact={exact} ws={need}: before-ws {len(pre)} after-ws {len(post)} '
                  f'(first {int(post[0]) if len(post) else -1}) out-before {len(opre)} out-after {len(opost)}',
                  flush=True)
