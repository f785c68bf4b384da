"""Diagnostic: per-phase cycle counts of fbank_frames_kernel (fbank.hip built with
-DSPK_FB_PROF=1 into exp_libs/libspk_fbprof.so, SPK_HIP_LIB=...).  B = 256 x 2 s."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-speaker_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PH = ['load+mean', 'window', 'fft', 'power', 'mel+log+store']


def main():
    from speakerlab import _hip
    from speakerlab.utils import synthetic
    dev = torch.device('cuda', 0)
    wavs = torch.from_numpy(synthetic.pcm16_batch(256, 32000, seed=1)).to(dev)
    for _ in range(3):
        _hip.fbank(wavs, 80, mean_nor=True)
    torch.cuda.synchronize()
    n = 8192 * 4 * 6
    buf = (ctypes.c_longlong * n)()
    assert ctypes.CDLL(_hip.LIB_PATH).spk_exp_fb_prof(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.int64).reshape(8192 * 4, 6)
    a = a[a[:, 5] > 0]
    pairs = a[:, 5].sum()
    per = a[:, :5].sum(axis=0) / pairs
    for p, v in zip(PH, per):
        print(f'{p:14s} {v:8.0f} cycles/pair {100 * v / per.sum():5.1f}%')
    print(f'total {per.sum():.0f} cycles per pair per wave; waves {len(a)}, pairs {pairs}')


if __name__ == '__main__':
    main()
