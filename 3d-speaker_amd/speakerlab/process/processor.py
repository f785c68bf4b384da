"""FBank front-end — drop-in for ``speakerlab.process.processor.FBank``
(reference ``speakerlab/process/processor.py:133-158``).

``FBank(n_mels, sample_rate, mean_nor)(wav, dither=0)`` returns the Kaldi log-mel fbank
[T, n_mels] computed by the HIP kernel (``csrc/fbank.hip``).  A device tensor stays on its
device; a CPU tensor is moved to the current ROCm device for the computation and the
result is returned on the CPU (same device-in/device-out contract as the reference).

The computation is the custom operator ``spk::fbank`` (``torch.library``) so that the
reference's own batched call site, ``torch.vmap(self.feature_extractor)(wavs_batch)``
(``infer_diarization.py:634``), works unchanged: the operator's vmap rule hands the whole
[N, 1, L] batch to the batched kernel in one launch instead of looping.  ``FBank.batch``
is the same batched form for callers that do not vmap.
"""
import torch

from speakerlab import _hip


@torch.library.custom_op('spk::fbank', mutates_args=())
def _fbank_op(wav: torch.Tensor, n_mels: int, mean_nor: bool) -> torch.Tensor:
    """wav [1, L] (device) -> [T, n_mels]; the reference's per-call shape contract."""
    return _hip.fbank(wav[0], n_mels, mean_nor)


@_fbank_op.register_fake
def _(wav, n_mels, mean_nor):
    return wav.new_empty((_hip.num_frames(wav.shape[-1]), n_mels))


def _fbank_vmap(info, in_dims, wav, n_mels, mean_nor):
    """vmap rule: [N, 1, L] (batch dim anywhere) -> one batched kernel launch, [N, T, n_mels]."""
    bdim = in_dims[0]
    if bdim is None:
        return _fbank_op(wav, n_mels, mean_nor), None
    wav = wav.movedim(bdim, 0)
    if wav.dim() != 3 or wav.shape[1] != 1:
        raise _hip.HipError(f'FBank under vmap: expected per-sample [1, L], got {tuple(wav.shape[1:])}')
    return _hip.fbank(wav[:, 0].contiguous(), n_mels, mean_nor), 0


_fbank_op.register_vmap(_fbank_vmap)


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
        feat = _fbank_op(dev_wav.to(torch.float32), self.n_mels, bool(self.mean_nor))
        return feat if back is None else feat.to(back)

    def batch(self, wavs: torch.Tensor, lengths=None):
        """[B, L] -> [B, T, n_mels] (or a list of [T_i, n_mels] with ``lengths``)."""
        dev_wavs, back = self._on_device(wavs)
        out = _hip.fbank(dev_wavs, self.n_mels, self.mean_nor, lengths=lengths)
        if back is None:
            return out
        return [o.to(back) for o in out] if isinstance(out, list) else out.to(back)
