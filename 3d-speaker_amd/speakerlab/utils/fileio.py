"""Audio ingest — ``load_audio`` semantics of ``speakerlab/utils/fileio.py:105-129``
(float in [-1, 1), int PCM scaled by 1/32768, channels averaged, [1, L]).  torchaudio is
absent here; WAV files are read with scipy.io.wavfile (PCM16/32, float).  Other rates are
resampled by ``resample``, an op-for-op restatement of torchaudio.functional.resample's
default path (the call at fileio.py:110,126): Hann-windowed sinc, lowpass_filter_width 6,
rolloff 0.99, gcd-reduced rates, a strided conv1d (torchaudio >= 0.13 op order, computed in
the waveform's dtype).  torchaudio itself is not importable here, so parity with it is
**unpinned**: tests/test_resample.py holds known answers (lengths, DC / impulse / sine
responses, an fp64 loop restatement of the same formula)."""
import math

import numpy as np
import torch


def read_wav(path):
    from scipy.io import wavfile
    fs, data = wavfile.read(path)
    if data.dtype == np.int16:
        data = data.astype(np.float32) / 32768.0
    elif data.dtype == np.int32:
        data = data.astype(np.float32) / 2147483648.0
    elif data.dtype == np.uint8:
        data = (data.astype(np.float32) - 128.0) / 128.0
    data = data.astype(np.float32)
    if data.ndim == 2:
        data = data.T            # [C, L]
    else:
        data = data[None]
    return torch.from_numpy(np.ascontiguousarray(data)), fs


def write_wav(path, wav, fs=16000):
    from scipy.io import wavfile
    x = np.asarray(wav, dtype=np.float32).reshape(-1)
    wavfile.write(path, fs, np.clip(np.round(x * 32768.0), -32768, 32767).astype(np.int16))


def sinc_resample_kernel(orig_freq: int, new_freq: int, gcd: int, lowpass_filter_width: int = 6,
                         rolloff: float = 0.99, dtype=torch.float32, device=None):
    """[new, 1, 2*width + orig] polyphase kernel and `width` (torchaudio
    ``_get_sinc_resample_kernel``, method ``sinc_interp_hann``)."""
    if lowpass_filter_width <= 0:
        raise ValueError('Low pass filter width should be positive.')
    orig_freq = int(orig_freq) // gcd
    new_freq = int(new_freq) // gcd
    base_freq = min(orig_freq, new_freq) * rolloff
    width = math.ceil(lowpass_filter_width * orig_freq / base_freq)
    idx = torch.arange(-width, width + orig_freq, dtype=dtype, device=device)[None, None] / orig_freq
    t = torch.arange(0, -new_freq, -1, dtype=dtype, device=device)[:, None, None] / new_freq + idx
    t *= base_freq
    t = t.clamp_(-lowpass_filter_width, lowpass_filter_width)
    window = torch.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t *= math.pi
    scale = base_freq / orig_freq
    kernels = torch.where(t == 0, torch.tensor(1.0).to(t), t.sin() / t)
    kernels *= window * scale
    return kernels, width


def resample(waveform: torch.Tensor, orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
             rolloff: float = 0.99) -> torch.Tensor:
    """torchaudio.functional.resample(waveform, orig_freq, new_freq) with its defaults: any
    leading shape, time last; output length ceil(new * L / orig) in gcd-reduced rates."""
    if orig_freq <= 0 or new_freq <= 0:
        raise ValueError('Original frequency and desired frequecy should be positive')
    if orig_freq == new_freq:
        return waveform
    g = math.gcd(int(orig_freq), int(new_freq))
    kernel, width = sinc_resample_kernel(orig_freq, new_freq, g, lowpass_filter_width, rolloff,
                                         waveform.dtype, waveform.device)
    o, n = int(orig_freq) // g, int(new_freq) // g
    shape = waveform.size()
    x = waveform.reshape(-1, shape[-1])
    num, length = x.shape
    x = torch.nn.functional.pad(x, (width, width + o))
    y = torch.nn.functional.conv1d(x[:, None], kernel, stride=o)
    y = y.transpose(1, 2).reshape(num, -1)
    target = int(math.ceil(n * length / o))
    return y[..., :target].reshape(shape[:-1] + (min(target, y.shape[-1]),))


def _resample(wav: torch.Tensor, fs: int, obj_fs: int) -> torch.Tensor:
    return resample(wav, fs, obj_fs)


def load_audio(input, ori_fs=None, obj_fs=None):
    if isinstance(input, str):
        wav, fs = read_wav(input)
        wav = wav.mean(dim=0, keepdim=True)
        if obj_fs is not None and fs != obj_fs:
            wav = _resample(wav, fs, obj_fs)
        return wav
    if isinstance(input, (np.ndarray, torch.Tensor)):
        wav = torch.from_numpy(input) if isinstance(input, np.ndarray) else input
        if wav.dtype in (torch.int16, torch.int32, torch.int64):
            wav = wav.to(torch.float32) / 32768
        wav = wav.to(torch.float32)
        assert wav.ndim <= 2
        if wav.ndim == 2:
            if wav.shape[0] > wav.shape[1]:
                wav = wav.t()
            wav = wav.mean(dim=0, keepdim=True)
        if wav.ndim == 1:
            wav = wav.unsqueeze(0)
        if ori_fs is not None and obj_fs is not None and ori_fs != obj_fs:
            wav = _resample(wav, ori_fs, obj_fs)
        return wav
    return input
