"""TEST INFRASTRUCTURE: run the real executor (plan building, BN folding, weight packing,
channel layouts, workspace aliasing) on the host through tests/emu/libspk_emu.so, whose
kernels are plain-loop emulations of the launch contracts in csrc/common.h.  Lets the
plan logic be checked against the oracle without a GPU; the kernels themselves are
checked by the -m gpu tests."""
import ctypes
import os
import subprocess

import torch

from speakerlab import _hip

EMU_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'emu')
_lib = None


def lib():
    global _lib
    if _lib is None:
        os.environ['SPK_GRAPH'] = '0'   # launches are emulated one by one (no graph replay)
        subprocess.run(['make', '-s', '-C', EMU_DIR], check=True)
        h = ctypes.CDLL(os.path.join(EMU_DIR, 'libspk_emu.so'))
        for name, (res, args) in _hip.SYMBOLS.items():
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, args
        _lib = h
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f'{what}: {lib().spk_last_error().decode()}')


class EmuModel:
    def __init__(self, module):
        cfg = module._hip_config()
        c = _hip.spk_model_config_t()
        c.arch = module._hip_arch
        for k in ('feat_dim', 'embed_dim', 'm_channels', 'base_width', 'scale', 'expansion', 'two_emb_layer',
                  'pooling'):
            setattr(c, k, int(cfg.get(k, 0)))
        for k in ('channels', 'kernel_sizes', 'dilations'):
            vals = list(cfg.get(k, []))[:5]
            getattr(c, k)[:len(vals)] = vals
        sd = module.state_dict()
        self.embed_dim = int(cfg['embed_dim'])
        host = []
        ws = (_hip.spk_weight_t * len(sd))()
        for i, (name, t) in enumerate(sd.items()):
            ws[i].name = name.encode()
            ws[i].ndim = t.dim()
            for d in range(t.dim()):
                ws[i].shape[d] = t.shape[d]
            if t.is_floating_point():
                h = t.detach().float().contiguous()
                host.append(h)
                ws[i].data = h.data_ptr()
        self.handle = ctypes.c_void_p()
        _check(lib().spk_model_create(ctypes.byref(c), ws, len(sd), ctypes.byref(self.handle)), 'create')

    def __call__(self, feats, lengths=None, ws=None):
        feats = feats.float().contiguous()
        B, T, _ = feats.shape
        n = ctypes.c_size_t()
        _check(lib().spk_model_workspace_bytes_lengths(self.handle, B, T, int(lengths is not None), ctypes.byref(n)),
               'workspace')
        if ws is None:
            ws = torch.zeros(max(n.value, 256), dtype=torch.uint8)
        self.last = (B, T, int(lengths is not None), ws)
        out = torch.empty(B, self.embed_dim)
        lens = None if lengths is None else torch.as_tensor(lengths, dtype=torch.int32).contiguous()
        _check(lib().spk_model_forward_lengths(self.handle, feats.data_ptr(), B, T,
                                               None if lens is None else lens.data_ptr(), ws.data_ptr(), ws.numel(),
                                               out.data_ptr(), None), 'forward')
        return out

    def range_word(self, last=None):
        """spk_model_range_check of the last forward (or of `last` = (B, T, ragged, ws))."""
        B, T, rg, ws = last or self.last
        v = ctypes.c_int32(-1)
        _check(lib().spk_model_range_check(self.handle, B, T, rg, ws.data_ptr(), None, ctypes.byref(v)), 'range_check')
        return v.value

    def plan(self, B, T):
        n = ctypes.c_int32()
        _check(lib().spk_model_plan_size(self.handle, B, T, ctypes.byref(n)), 'plan_size')
        steps = []
        for i in range(n.value):
            name = ctypes.create_string_buffer(256)
            kern = ctypes.create_string_buffer(256)
            fl = ctypes.c_double()
            _check(lib().spk_model_plan_step(self.handle, B, T, i, name, 256, kern, 256, ctypes.byref(fl)), 'step')
            steps.append((name.value.decode(), fl.value, kern.value.decode()))
        return steps

    def plan_bytes(self, B, T):
        out = []
        for i in range(len(self.plan(B, T))):
            b = ctypes.c_double()
            _check(lib().spk_model_plan_step_bytes(self.handle, B, T, i, ctypes.byref(b)), 'step_bytes')
            out.append(b.value)
        return out

    def flops(self, T):
        f = ctypes.c_double()
        _check(lib().spk_model_flops(self.handle, T, ctypes.byref(f)), 'flops')
        return f.value
