"""Diagnostic: per-phase cycle counts of the fused stage-2 Res2Net block kernel
(res2block_s2.hip built with -DSPK_S2_PROF=1 into a separate library, SPK_HIP_LIB=...).
Runs ERes2NetV2 forwards (B=256, T=198) and prints mean cycles per tile per phase over
waves (the last fused stage-2 block, layer2.3)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, '3d-speaker_amd'), os.path.join(REPO, 'tests')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

PH = ['bar-chunk', 'x-stage', 'conv1+epi', 'bar-end1', 'convs.0', 'sp/cat', 'convs.1', 'a3+bar', 'conv3',
      'bar-end']


def main():
    import helpers
    from speakerlab import _hip
    dev = torch.device('cuda', 0)
    m = helpers.loaded_module('eres2netv2').to(dev)
    x = torch.randn(256, 198, 80, device=dev)
    with torch.no_grad():
        for _ in range(3):
            m(x)
    torch.cuda.synchronize()
    n = 256 * 8 * 10 * 64
    buf = (ctypes.c_longlong * n)()
    assert _hip.lib()._name and ctypes.CDLL(_hip.LIB_PATH).spk_exp_s2_prof(buf, n) == 0
    a = np.frombuffer(buf, dtype=np.int64).reshape(256, 8, 10, 64)[:, :, :, 0]
    ntiles = 256 * 5 * 7
    per_tile = a.sum(axis=0).mean(axis=0) / ntiles   # summed over blocks, mean over waves
    tot = per_tile.sum()
    for i, p in enumerate(PH):
        print(f'{p:10s} {per_tile[i]:10.0f} cycles/tile  {100 * per_tile[i] / tot:5.1f}%')
    print(f'total {tot:.0f} cycles per tile (waves averaged)')


if __name__ == '__main__':
    main()
