"""ctypes binding of ``libspk_hip.so`` (declared in ``include/spk_hip.h``).

This is the only bridge between the drop-in Python surface and the HIP kernels.  There is
no CPU fallback: if the shared library is missing, or a tensor is not on a ROCm device,
the call raises.  (The CPU restatement used to *check* results lives in ``oracle/`` and
is imported by tests only.)
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Dict, Optional

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # .../3d-speaker_amd
LIB_PATH = os.environ.get('SPK_HIP_LIB', os.path.join(_PKG_ROOT, 'lib', 'libspk_hip.so'))

ARCH_ERES2NETV2 = 1
ARCH_ERES2NET = 2
ARCH_ECAPA = 3
ARCH_CAMPPLUS = 4
ARCH_RESNET = 5
ARCH_RES2NET = 6


class spk_weight_t(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char_p), ('data', ctypes.c_void_p), ('ndim', ctypes.c_int32),
                ('shape', ctypes.c_int64 * 4)]


class spk_model_config_t(ctypes.Structure):
    _fields_ = [('arch', ctypes.c_int32), ('feat_dim', ctypes.c_int32), ('embed_dim', ctypes.c_int32),
                ('m_channels', ctypes.c_int32), ('base_width', ctypes.c_int32), ('scale', ctypes.c_int32),
                ('expansion', ctypes.c_int32), ('two_emb_layer', ctypes.c_int32),
                ('channels', ctypes.c_int32 * 5), ('kernel_sizes', ctypes.c_int32 * 5),
                ('dilations', ctypes.c_int32 * 5), ('precision', ctypes.c_int32), ('pooling', ctypes.c_int32), ('reserved', ctypes.c_int32 * 6)]


# spk_model_config_t.precision (include/spk_hip.h)
PRECISIONS = {'fp32': 0, 'fp16': 1}


SPK_CONSUME_TOPK = 1


class spk_affinity_consumer_t(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('k', ctypes.c_int32), ('exclude_self', ctypes.c_int32),
                ('self_offset', ctypes.c_int64), ('threshold', ctypes.c_float), ('top_scores', ctypes.c_void_p),
                ('top_index', ctypes.c_void_p), ('count_ge', ctypes.c_void_p), ('workspace', ctypes.c_void_p),
                ('workspace_bytes', ctypes.c_size_t)]


# every entry point of include/spk_hip.h: name -> (restype, argtypes)
_P = ctypes.c_void_p
SYMBOLS = {
    'spk_version': (ctypes.c_int, []),
    'spk_last_error': (ctypes.c_char_p, []),
    'spk_fbank_f32': (ctypes.c_int, [_P, _P, ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_int32, _P]),
    'spk_fbank_f32_padded': (ctypes.c_int, [_P, _P, ctypes.c_int32, _P, _P, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, _P]),
    'spk_model_create': (ctypes.c_int, [ctypes.POINTER(spk_model_config_t), ctypes.POINTER(spk_weight_t),
                                        ctypes.c_int32, ctypes.POINTER(_P)]),
    'spk_model_destroy': (ctypes.c_int, [_P]),
    'spk_model_workspace_bytes': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_size_t)]),
    'spk_model_forward': (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_size_t, _P, _P]),
    'spk_model_workspace_bytes_lengths': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                         ctypes.POINTER(ctypes.c_size_t)]),
    'spk_model_forward_lengths': (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_size_t, _P,
                                                 _P]),
    'spk_model_flops': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.POINTER(ctypes.c_double)]),
    'spk_model_range_check': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P,
                                             ctypes.POINTER(ctypes.c_int32)]),
    'spk_model_forward_exact': (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_size_t, _P,
                                               _P]),
    'spk_model_guard_plan': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                            ctypes.POINTER(ctypes.c_int32)]),
    'spk_model_plan_size': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    'spk_model_plan_step': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                           ctypes.c_int32, ctypes.c_char_p, ctypes.c_int32,
                                           ctypes.POINTER(ctypes.c_double)]),
    'spk_model_plan_step_bytes': (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.POINTER(ctypes.c_double)]),
    'spk_model_forward_timed': (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_size_t, _P, _P,
                                               _P, ctypes.c_int32]),
    'spk_cosine_affinity': (ctypes.c_int, [_P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int32, _P,
                                           ctypes.c_int64, _P]),
    'spk_spectral_laplacian': (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, _P, ctypes.c_int64,
                                              _P, ctypes.c_size_t, _P]),
    'spk_symmetric_eig': (ctypes.c_int, [_P, ctypes.c_int64, ctypes.c_int64, _P, _P]),
    'spk_cosine_topk_workspace_bytes': (ctypes.c_int, [ctypes.c_int64, ctypes.c_int64,
                                                       ctypes.POINTER(ctypes.c_size_t)]),
    'spk_cosine_topk': (ctypes.c_int, [_P, ctypes.c_int64, _P, ctypes.c_int64, ctypes.c_int32,
                                       ctypes.POINTER(spk_affinity_consumer_t), _P]),
    'spk_cosine_trials': (ctypes.c_int, [_P, _P, ctypes.c_int32, _P, _P, ctypes.c_int64, _P, _P]),
}

_lib = None
_lock = threading.Lock()


class HipError(RuntimeError):
    pass


def lib():
    """Load libspk_hip.so once (after torch, so it shares torch's HIP runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipError(f'libspk_hip.so not found at {LIB_PATH}: build it with '
                               f'`python -c "import __graft_entry__ as g; g.build()"` (or make -C 3d-speaker_amd/csrc)')
            handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            for name, (res, args) in SYMBOLS.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().spk_last_error()
        raise HipError(f'{what} failed ({rc}): {msg.decode() if msg else ""}')


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device_tensor(x: torch.Tensor, what: str):
    if not isinstance(x, torch.Tensor) or x.device.type != 'cuda':
        raise HipError(f'{what}: the MI355X path needs a ROCm device tensor (got '
                       f'{getattr(x, "device", type(x))}); move the input with .to("cuda")')


# ----------------------------------------------------------------------------- Fbank
_frame_offsets_cache: Dict = {}


def num_frames(n_samples: int) -> int:
    return 0 if n_samples < 400 else 1 + (n_samples - 400) // 160


def fbank(wavs: torch.Tensor, n_mels: int = 80, mean_nor: bool = False, lengths=None) -> torch.Tensor:
    """Batched Kaldi Fbank on the GPU.

    ``wavs``: [B, L] float32 device tensor (or [L]).  With ``lengths`` (list of ints) the
    rows are ragged (samples beyond each length are ignored) and the result is a list of
    [T_i, n_mels] views into one buffer; otherwise [B, T, n_mels].
    """
    require_device_tensor(wavs, 'fbank')
    squeeze = wavs.dim() == 1
    if squeeze:
        wavs = wavs.unsqueeze(0)
    wavs = wavs.to(torch.float32).contiguous()
    B, L = wavs.shape
    dev = wavs.device
    if lengths is None:
        lens = [L] * B
    else:
        lens = [int(v) for v in lengths]
    frames = [num_frames(n) for n in lens]
    frame_off = [0]
    for f in frames:
        frame_off.append(frame_off[-1] + f)
    wav_off = [i * L for i in range(B + 1)]
    offs = torch.tensor([wav_off, frame_off], dtype=torch.int64).to(dev, non_blocking=True)
    feats = torch.empty((frame_off[-1], n_mels), dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _check(lib().spk_fbank_f32(wavs.data_ptr(), offs[0].data_ptr(), B, feats.data_ptr(), offs[1].data_ptr(),
                                   n_mels, int(bool(mean_nor)), _stream(dev)), 'spk_fbank_f32')
    if lengths is not None:
        return [feats[frame_off[i]:frame_off[i + 1]] for i in range(B)]
    out = feats.view(B, frames[0], n_mels)
    return out[0] if squeeze else out


def fbank_padded(wavs: torch.Tensor, lengths, n_mels: int = 80, mean_nor: bool = False):
    """Ragged Fbank written straight into a zero-padded [B, T_max, n_mels] batch: returns
    (feats, frames) with ``frames`` a device int32 [B] tensor of valid frames per row, the
    input of the models' ``forward(x, lengths=frames)`` (spk_fbank_f32_padded)."""
    require_device_tensor(wavs, 'fbank_padded')
    wavs = wavs.to(torch.float32).contiguous()
    B, L = wavs.shape
    dev = wavs.device
    lens = [int(v) for v in lengths]
    if len(lens) != B or max(lens) > L or min(lens) < 400:
        raise HipError('fbank_padded: need B lengths in [400, padded length]')
    frames = [num_frames(n) for n in lens]
    tmax = max(frames)
    frame_off = [0]
    for f in frames:
        frame_off.append(frame_off[-1] + f)
    wav_off = [i * L for i in range(B + 1)]
    offs = torch.tensor([wav_off, frame_off], dtype=torch.int64).to(dev, non_blocking=True)
    feats = torch.empty((B, tmax, n_mels), dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _check(lib().spk_fbank_f32_padded(wavs.data_ptr(), offs[0].data_ptr(), B, feats.data_ptr(),
                                          offs[1].data_ptr(), tmax, n_mels, int(bool(mean_nor)), _stream(dev)),
               'spk_fbank_f32_padded')
    return feats, torch.tensor(frames, dtype=torch.int32).to(dev, non_blocking=True)


# ----------------------------------------------------------------------------- models
class NativeModel:
    """One ``spk_model_t`` handle (folded + packed weights on one device)."""

    def __init__(self, arch: int, cfg: dict, state_dict, device: torch.device, precision: str = 'fp32'):
        if precision not in PRECISIONS:
            raise HipError(f'precision must be one of {sorted(PRECISIONS)}, got {precision!r}')
        c = spk_model_config_t()
        c.arch = arch
        c.precision = PRECISIONS[precision]
        self.precision = precision
        for k in ('feat_dim', 'embed_dim', 'm_channels', 'base_width', 'scale', 'expansion', 'two_emb_layer',
                  'pooling'):
            setattr(c, k, int(cfg.get(k, 0)))
        for k in ('channels', 'kernel_sizes', 'dilations'):
            vals = list(cfg.get(k, []))[:5]
            getattr(c, k)[:len(vals)] = vals
        self.embed_dim = int(cfg['embed_dim'])
        self.arch = arch
        self.device = device
        host = []
        ws = (spk_weight_t * len(state_dict))()
        for i, (name, t) in enumerate(state_dict.items()):
            ws[i].name = name.encode()
            ws[i].ndim = t.dim()
            for d in range(min(t.dim(), 4)):
                ws[i].shape[d] = t.shape[d]
            if t.is_floating_point():
                h = t.detach().to('cpu', torch.float32).contiguous()
                host.append(h)
                ws[i].data = h.data_ptr()
            else:
                ws[i].data = None
        handle = ctypes.c_void_p()
        with torch.cuda.device(device):
            _check(lib().spk_model_create(ctypes.byref(c), ws, len(state_dict), ctypes.byref(handle)),
                   'spk_model_create')
        self.handle = handle
        self._ws: Optional[torch.Tensor] = None          # workspace of the last forward
        self._ws_by_stream = {}                           # stream handle -> workspace
        self._last = None                                 # (B, T, ragged, workspace, stream) of the last forward

    def __del__(self):
        h = getattr(self, 'handle', None)
        if h is not None and _lib is not None:
            try:
                _lib.spk_model_destroy(h)
            except Exception:
                pass

    def workspace_bytes(self, B: int, T: int) -> int:
        n = ctypes.c_size_t()
        _check(lib().spk_model_workspace_bytes(self.handle, B, T, ctypes.byref(n)), 'spk_model_workspace_bytes')
        return n.value

    def flops(self, T: int) -> float:
        f = ctypes.c_double()
        _check(lib().spk_model_flops(self.handle, T, ctypes.byref(f)), 'spk_model_flops')
        return f.value

    def plan(self, B: int, T: int):
        """[(step name, kernel name, algorithmic FLOPs)] of the launch plan for [B, T]."""
        n = ctypes.c_int32()
        _check(lib().spk_model_plan_size(self.handle, B, T, ctypes.byref(n)), 'spk_model_plan_size')
        out = []
        for i in range(n.value):
            name = ctypes.create_string_buffer(256)
            kern = ctypes.create_string_buffer(256)
            fl = ctypes.c_double()
            _check(lib().spk_model_plan_step(self.handle, B, T, i, name, 256, kern, 256, ctypes.byref(fl)),
                   'spk_model_plan_step')
            out.append((name.value.decode(), kern.value.decode(), fl.value))
        return out

    def plan_bytes(self, B: int, T: int):
        """Algorithmic HBM bytes of every plan step (0 where a step is not priced)."""
        out = []
        for i in range(len(self.plan(B, T))):
            b = ctypes.c_double()
            _check(lib().spk_model_plan_step_bytes(self.handle, B, T, i, ctypes.byref(b)), 'spk_model_plan_step_bytes')
            out.append(b.value)
        return out

    def _workspace(self, need: int) -> torch.Tensor:
        """The calling stream's workspace (grown on demand).  run_graph stages the inputs
        into the workspace and replays the graph captured for its address, so two forwards
        in flight on different streams must not share one: each stream gets its own.  A
        handle is still not safe for concurrent forwards on ONE stream from several threads
        (they would be serialised on the stream but share the staging space)."""
        key = _stream(self.device)
        ws = self._ws_by_stream.get(key)
        if ws is None or ws.numel() < need:
            if ws is not None and self._ws is ws:
                self._ws = None                 # free the old block before the larger one
            self._ws_by_stream.pop(key, None)
            ws = torch.empty(max(need, 256), dtype=torch.uint8, device=self.device)
            self._ws_by_stream[key] = ws
        return ws

    def forward_timed(self, feats: torch.Tensor, out: torch.Tensor):
        """forward() with a HIP event around every plan step; returns per-step ms."""
        B, T, _ = feats.shape
        n = len(self.plan(B, T))
        ms = (ctypes.c_float * n)()
        with torch.cuda.device(self.device):
            self._ws = self._workspace(self.workspace_bytes(B, T))
            _check(lib().spk_model_forward_timed(self.handle, feats.data_ptr(), B, T, self._ws.data_ptr(),
                                                 self._ws.numel(), out.data_ptr(), _stream(self.device), ms, n),
                   'spk_model_forward_timed')
        return list(ms)

    def workspace_bytes_lengths(self, B: int, T: int, ragged: bool) -> int:
        n = ctypes.c_size_t()
        _check(lib().spk_model_workspace_bytes_lengths(self.handle, B, T, int(ragged), ctypes.byref(n)),
               'spk_model_workspace_bytes_lengths')
        return n.value

    def forward(self, feats: torch.Tensor, out: Optional[torch.Tensor] = None, lengths=None) -> torch.Tensor:
        """``lengths`` (optional): valid frames per row (variable-length batch, CAM++)."""
        require_device_tensor(feats, 'embedding forward')
        if feats.device != self.device:
            raise HipError(f'model handle lives on {self.device}, input on {feats.device}')
        if feats.dim() != 3:
            raise HipError(f'expected feats [B, T, F], got {tuple(feats.shape)}')
        feats = feats.to(torch.float32).contiguous()
        B, T, _ = feats.shape
        if lengths is not None:
            lengths = torch.as_tensor(lengths, dtype=torch.int32).to(self.device).contiguous()
            if lengths.numel() != B:
                raise HipError(f'lengths has {lengths.numel()} entries for a batch of {B}')
            # a length past T would read the next utterance's rows (and past the workspace
            # for the last one); CAM++'s unbiased std needs >= 2 frames
            lo = 2 if self.arch == ARCH_CAMPPLUS else 1
            mn, mx = (int(v) for v in torch.aminmax(lengths))
            if mn < lo or mx > T:
                raise HipError(f'lengths must lie in [{lo}, T={T}] (got min {mn}, max {mx})')
        with torch.cuda.device(self.device):
            need = self.workspace_bytes(B, T) if lengths is None else self.workspace_bytes_lengths(B, T, True)
            self._ws = self._workspace(need)
            if out is None:
                out = torch.empty((B, self.embed_dim), dtype=torch.float32, device=self.device)
            if lengths is None:
                _check(lib().spk_model_forward(self.handle, feats.data_ptr(), B, T, self._ws.data_ptr(),
                                               self._ws.numel(), out.data_ptr(), _stream(self.device)),
                       'spk_model_forward')
            else:
                _check(lib().spk_model_forward_lengths(self.handle, feats.data_ptr(), B, T, lengths.data_ptr(),
                                                       self._ws.data_ptr(), self._ws.numel(), out.data_ptr(),
                                                       _stream(self.device)),
                       'spk_model_forward_lengths')
            # the fp16x3 range guard resolves on the device (include/spk_hip.h): no host sync
            self._last = (B, T, int(lengths is not None), self._ws, _stream(self.device))
        return out

    @property
    def last_forward_flagged(self) -> bool:
        """Whether an activation of the last forward reached the fp16x3 range limit (its range
        word is set; synchronises that forward's stream; diagnostics)."""
        if self._last is None:
            return False
        B, T, ragged, ws, stream = self._last
        flag = ctypes.c_int32(0)
        with torch.cuda.device(self.device):
            _check(lib().spk_model_range_check(self.handle, B, T, ragged, ws.data_ptr(), stream, ctypes.byref(flag)),
                   'spk_model_range_check')
        return bool(flag.value)

    @property
    def last_forward_exact(self) -> bool:
        """Whether the last forward was recomputed on the exact-fp32 kernels because an
        activation reached fp16's range: its word is set and its plan has an exact twin
        (ECAPA / CAM++ plans scale the split operands instead and have none)."""
        if not self.last_forward_flagged:
            return False
        B, T, ragged = self._last[:3]
        return self.guard_plan(B, T, bool(ragged))['twin_segments'] > 0

    def guard_plan(self, B: int, T: int, ragged: bool = False) -> dict:
        """How the guarded forward of shape (B, T) is cut into range-guard segments and how
        many exact-plan launches are enqueued behind it (include/spk_hip.h spk_model_guard_plan)."""
        vals = [ctypes.c_int32(0) for _ in range(3)]
        _check(lib().spk_model_guard_plan(self.handle, B, T, int(ragged), *[ctypes.byref(v) for v in vals]),
               'spk_model_guard_plan')
        return dict(zip(('segments', 'twin_segments', 'gated_steps'), (v.value for v in vals)))


class HipModuleMixin:
    """Mixin for the drop-in nn.Modules: lazily builds one native handle per device from
    the module's own state_dict and drops it whenever weights are reloaded or moved."""

    _hip_arch: int = 0

    def _hip_config(self) -> dict:  # pragma: no cover - overridden
        raise NotImplementedError

    def _hip_reset(self, *args, **kwargs):
        self.__dict__['_hip_handles'] = {}

    def set_hip_precision(self, precision: str):
        """'fp32' (default): fp32-accurate forward (fp16x3 split products), embeddings within
        1e-4 of the reference.  'fp16': one fp16 MFMA product per multiply with fp32
        accumulation -- the reduced-precision mode of BASELINE config C3 (cosine >= 0.9999 to
        the reference); layers without a single-product kernel stay fp16x3."""
        if precision not in PRECISIONS:
            raise HipError(f'precision must be one of {sorted(PRECISIONS)}, got {precision!r}')
        self.__dict__['_hip_precision'] = precision
        self._hip_reset()
        return self

    def _hip_handle(self, device: torch.device) -> NativeModel:
        handles = self.__dict__.setdefault('_hip_handles', {})
        key = (device.type, device.index)
        h = handles.get(key)
        if h is None:
            h = NativeModel(self._hip_arch, self._hip_config(), self.state_dict(), device,
                            self.__dict__.get('_hip_precision', 'fp32'))
            handles[key] = h
        return h

    def _hip_forward(self, x: torch.Tensor, lengths=None) -> torch.Tensor:
        require_device_tensor(x, type(self).__name__ + '.forward')
        if self.training:
            raise HipError(f'{type(self).__name__}: the MI355X path is inference-only; call .eval()')
        dev = x.device if x.device.index is not None else torch.device('cuda', torch.cuda.current_device())
        return self._hip_handle(dev).forward(x, lengths=lengths)

    def _apply(self, fn, *args, **kwargs):
        self._hip_reset()
        return super()._apply(fn, *args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self._hip_reset()
        return super()._load_from_state_dict(*args, **kwargs)


def cosine_affinity(a: torch.Tensor, b: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
    """[Na, E] x [Nb, E] -> [Na, Nb] cosine similarity on the GPU (sklearn semantics)."""
    require_device_tensor(a, 'cosine_affinity')
    b = a if b is None else b
    a = a.to(torch.float32).contiguous()
    b = b.to(torch.float32).contiguous()
    if out is None:
        out = torch.empty((a.shape[0], b.shape[0]), dtype=torch.float32, device=a.device)
    with torch.cuda.device(a.device):
        _check(lib().spk_cosine_affinity(a.data_ptr(), a.shape[0], b.data_ptr(), b.shape[0], a.shape[1],
                                         out.data_ptr(), out.stride(0), _stream(a.device)), 'spk_cosine_affinity')
    return out


def cosine_topk(a: torch.Tensor, b: torch.Tensor, k: int = 1, self_offset: Optional[int] = None,
                threshold: float = float('inf')):
    """Row-block consumer of the cosine affinity (the [Na, Nb] matrix is never written): for
    every row of ``a`` the ``k`` best (score, column) pairs over ``b`` -- score descending,
    column ascending on ties, column ``i + self_offset`` of row ``i`` excluded when
    ``self_offset`` is given -- and the number of columns scoring >= ``threshold``.
    Returns (scores [Na, k] float32, index [Na, k] int64, count [Na] int64)."""
    require_device_tensor(a, 'cosine_topk')
    b = a if b is None else b
    a = a.to(torch.float32).contiguous()
    b = b.to(torch.float32).contiguous()
    if not 1 <= k <= 8:
        raise HipError('cosine_topk: k must be in 1..8')
    Na, Nb, E = a.shape[0], b.shape[0], a.shape[1]
    dev = a.device
    scores = torch.empty((Na, k), dtype=torch.float32, device=dev)
    index = torch.empty((Na, k), dtype=torch.int64, device=dev)
    count = torch.empty(Na, dtype=torch.int64, device=dev)
    nbytes = ctypes.c_size_t(0)
    _check(lib().spk_cosine_topk_workspace_bytes(Na, Nb, ctypes.byref(nbytes)), 'spk_cosine_topk_workspace_bytes')
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
    c = spk_affinity_consumer_t(SPK_CONSUME_TOPK, k, 0 if self_offset is None else 1,
                                0 if self_offset is None else int(self_offset), float(threshold), scores.data_ptr(),
                                index.data_ptr(), count.data_ptr(), ws.data_ptr(), nbytes.value)
    with torch.cuda.device(dev):
        _check(lib().spk_cosine_topk(a.data_ptr(), Na, b.data_ptr(), Nb, E, ctypes.byref(c), _stream(dev)),
               'spk_cosine_topk')
    return scores, index, count


def cosine_trials(a: torch.Tensor, b: torch.Tensor, ia: torch.Tensor, ib: torch.Tensor) -> torch.Tensor:
    """scores[t] = cosine(a[ia[t]], b[ib[t]]) on the device (compute_score_metrics.py:102-118)."""
    require_device_tensor(a, 'cosine_trials')
    a = a.to(torch.float32).contiguous()
    b = b.to(torch.float32).contiguous()
    ia = ia.to(device=a.device, dtype=torch.int64).contiguous()
    ib = ib.to(device=a.device, dtype=torch.int64).contiguous()
    if ia.numel() and (int(ia.min()) < 0 or int(ia.max()) >= a.shape[0] or int(ib.min()) < 0
                       or int(ib.max()) >= b.shape[0]):
        raise HipError('cosine_trials: trial index out of range')
    out = torch.empty(ia.numel(), dtype=torch.float32, device=a.device)
    with torch.cuda.device(a.device):
        _check(lib().spk_cosine_trials(a.data_ptr(), b.data_ptr(), a.shape[1], ia.data_ptr(), ib.data_ptr(),
                                       ia.numel(), out.data_ptr(), _stream(a.device)), 'spk_cosine_trials')
    return out


def spectral_laplacian(S: torch.Tensor, n_elems: int) -> torch.Tensor:
    """p-pruned, symmetrised unnormalised Laplacian of an N x N affinity (device)."""
    require_device_tensor(S, 'spectral_laplacian')
    S = S.to(torch.float32).contiguous()
    N = S.shape[0]
    L = torch.empty_like(S)
    ws = torch.empty(N * N, dtype=torch.float32, device=S.device)
    with torch.cuda.device(S.device):
        _check(lib().spk_spectral_laplacian(S.data_ptr(), N, S.stride(0), max(0, int(n_elems)), L.data_ptr(),
                                            L.stride(0), ws.data_ptr(), ws.numel() * 4, _stream(S.device)),
               'spk_spectral_laplacian')
    return L


def symmetric_eig(A: torch.Tensor):
    """(eigenvalues ascending [N], eigenvectors as ROWS [N, N]) of a symmetric device matrix;
    A is overwritten."""
    require_device_tensor(A, 'symmetric_eig')
    if A.dtype != torch.float32 or not A.is_contiguous():
        raise HipError('symmetric_eig: float32 contiguous matrix expected')
    N = A.shape[0]
    w = torch.empty(N, dtype=torch.float32, device=A.device)
    with torch.cuda.device(A.device):
        _check(lib().spk_symmetric_eig(A.data_ptr(), N, A.stride(0), w.data_ptr(), _stream(A.device)),
               'spk_symmetric_eig')
    return w, A
