"""AFF attentional feature fusion — parameter layout of ``speakerlab/models/eres2net/fusion.py:8-28``.

The forward runs fused inside the ERes2Net executor (two GEMMs, the second with the
``x*(1+tanh a) + y*(1-tanh a)`` epilogue; see ``3d-speaker_amd/csrc/eres2net.cpp``).
"""
import torch.nn as nn


class _FusedOnly(nn.Module):
    def forward(self, *args, **kwargs):
        raise RuntimeError(f'{type(self).__name__} executes inside the fused model forward on the MI355X path; '
                           'call the top-level embedding model instead')


class AFF(_FusedOnly):
    def __init__(self, channels=64, r=4):
        super().__init__()
        mid = int(channels // r)
        # local_att: conv(2C->C/r)+bias, BN, SiLU, conv(C/r->C)+bias, BN  (keys .0 .1 .3 .4)
        self.local_att = nn.Sequential(
            nn.Conv2d(2 * channels, mid, 1, 1, 0), nn.BatchNorm2d(mid), nn.SiLU(inplace=True),
            nn.Conv2d(mid, channels, 1, 1, 0), nn.BatchNorm2d(channels))
