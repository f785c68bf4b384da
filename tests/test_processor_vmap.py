"""The drop-in FBank under torch.vmap, as the reference diarization calls it
(``infer_diarization.py:634``: ``torch.vmap(self.feature_extractor)(wavs_batch)`` with
wavs_batch [N, 1, L]).  CPU: the operator's vmap rule must route the whole batch to ONE
batched kernel call (the kernel is replaced by a recording stand-in, no GPU here)."""
import torch

from speakerlab import _hip
from speakerlab.process import processor


def _fake_kernel(calls):
    def fbank(w, n_mels=80, mean_nor=False, lengths=None):
        calls.append(tuple(w.shape))
        sq = w.dim() == 1
        w2 = w[None] if sq else w
        T = _hip.num_frames(w2.shape[-1])
        # distinct per row: row sum broadcast (a fresh tensor, no aliasing)
        out = w2.sum(-1)[:, None, None] + torch.arange(T * n_mels, dtype=w2.dtype).view(1, T, n_mels)
        return out[0] if sq else out
    return fbank


def test_vmap_routes_batch_to_one_kernel_call(monkeypatch):
    calls = []
    monkeypatch.setattr(_hip, 'fbank', _fake_kernel(calls))
    monkeypatch.setattr(processor.FBank, '_on_device', lambda self, w: (w, None))
    fb = processor.FBank(80, 16000, mean_nor=True)
    x = torch.randn(5, 1, 16000)
    y = torch.vmap(fb)(x)
    assert y.shape == (5, 98, 80)
    assert calls == [(5, 16000)]                 # one batched launch, not five
    for i in (0, 3):
        z = fb(x[i])                              # the plain per-utterance call
        assert torch.equal(y[i], z)
    # batch dimension not in front
    calls.clear()
    y2 = torch.vmap(fb, in_dims=2)(x.permute(1, 2, 0).contiguous())
    assert calls == [(5, 16000)] and torch.equal(y2, y)
