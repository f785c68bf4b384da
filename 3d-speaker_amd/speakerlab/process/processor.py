"""FBank front-end — drop-in for ``speakerlab.process.processor.FBank``
(reference ``speakerlab/process/processor.py:133-158``).

``FBank(n_mels, sample_rate, mean_nor)(wav, dither=0)`` returns the Kaldi log-mel fbank
[T, n_mels] computed by the HIP kernel (``csrc/fbank.hip``).  A device tensor stays on its
device; a CPU tensor is moved to the current ROCm device for the computation and the
result is returned on the CPU (same device-in/device-out contract as the reference).
``FBank.batch`` is the batched form used by the CLIs (the reference vmaps ``__call__``,
``infer_diarization.py:634``).
"""
import torch

from speakerlab import _hip


class FBank(object):
    def __init__(self, n_mels, sample_rate, mean_nor: bool = False):
        self.n_mels = n_mels
        self.sample_rate = sample_rate
        self.mean_nor = mean_nor

    def _on_device(self, wav: torch.Tensor):
        if wav.device.type == 'cuda':
            return wav, None
        if not torch.cuda.is_available():
            raise _hip.HipError('FBank: no ROCm device available (the MI355X path has no CPU implementation)')
        return wav.to('cuda'), wav.device

    def __call__(self, wav, dither=0):
        assert self.sample_rate == 16000, 'only 16 kHz is supported (processor.py:145)'
        if dither:
            raise NotImplementedError('dither != 0 is not supported on the MI355X path (inference uses 0)')
        if wav.dim() == 1:
            wav = wav.unsqueeze(0)
        if wav.shape[0] > 1:           # select channel 0 (processor.py:148-151)
            wav = wav[0:1]
        assert wav.dim() == 2 and wav.shape[0] == 1
        dev_wav, back = self._on_device(wav)
        feat = _hip.fbank(dev_wav[0], self.n_mels, self.mean_nor)
        return feat if back is None else feat.to(back)

    def batch(self, wavs: torch.Tensor, lengths=None):
        """[B, L] -> [B, T, n_mels] (or a list of [T_i, n_mels] with ``lengths``)."""
        dev_wavs, back = self._on_device(wavs)
        out = _hip.fbank(dev_wavs, self.n_mels, self.mean_nor, lengths=lengths)
        if back is None:
            return out
        return [o.to(back) for o in out] if isinstance(out, list) else out.to(back)
