"""Audio ingest — ``load_audio`` semantics of ``speakerlab/utils/fileio.py:105-129``
(float in [-1, 1), int PCM scaled by 1/32768, channels averaged, [1, L]).  torchaudio is
absent here; WAV files are read with scipy.io.wavfile (PCM16/32, float), other rates are
resampled with scipy's polyphase resampler."""
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


def _resample(wav: torch.Tensor, fs: int, obj_fs: int) -> torch.Tensor:
    from math import gcd

    from scipy.signal import resample_poly
    g = gcd(fs, obj_fs)
    return torch.from_numpy(resample_poly(wav.numpy(), obj_fs // g, fs // g, axis=-1).astype(np.float32))


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
