"""Shared module tree of the ERes2Net family (parameter containers only).

Both ``ERes2NetV2`` (``ERes2NetV2.py:31-254``) and ``ERes2Net`` (``ERes2Net.py:30-231``)
are stacks of the same Res2Net-style basic block; they differ in base width, in whether
expansion is a ctor argument, and in the bottom-up fusion head.  This module builds the
identical ``state_dict`` layout (strict ``load_state_dict`` of reference checkpoints works)
while the computation itself is one native plan (``csrc/eres2net.cpp``).
"""
import math

import torch.nn as nn

from speakerlab.models.eres2net.fusion import AFF, _FusedOnly


class ReLU(nn.Hardtanh):
    """The reference's ``ReLU`` is Hardtanh(0, 20) (``ERes2NetV2.py:20-28``)."""

    def __init__(self, inplace=False):
        super().__init__(0, 20, inplace)

    def __repr__(self):
        return 'ReLU (' + ('inplace' if self.inplace else '') + ')'


class Res2Block(_FusedOnly):
    """conv1(1x1, stride) -> `scale` chained 3x3 convs (sum or AFF fusion) -> conv3 + shortcut."""

    def __init__(self, in_planes, planes, stride=1, baseWidth=26, scale=2, expansion=2, use_aff=False):
        super().__init__()
        width = int(math.floor(planes * (baseWidth / 64.0)))
        out_planes = planes * expansion
        self.width, self.scale, self.nums, self.stride, self.expansion = width, scale, scale, stride, expansion
        self.conv1 = nn.Conv2d(in_planes, width * scale, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(width * scale)
        self.convs = nn.ModuleList(nn.Conv2d(width, width, 3, padding=1, bias=False) for _ in range(scale))
        self.bns = nn.ModuleList(nn.BatchNorm2d(width) for _ in range(scale))
        if use_aff:
            self.fuse_models = nn.ModuleList(AFF(channels=width, r=4) for _ in range(scale - 1))
        self.relu = ReLU(inplace=True)
        self.conv3 = nn.Conv2d(width * scale, out_planes, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_planes)
        if stride != 1 or in_planes != out_planes:
            self.shortcut = nn.Sequential(nn.Conv2d(in_planes, out_planes, 1, stride=stride, bias=False),
                                          nn.BatchNorm2d(out_planes))
        else:
            self.shortcut = nn.Sequential()


def make_stage(block_cls, in_planes, planes, n_blocks, stride, **kw):
    """Returns (nn.Sequential of blocks, output channels)."""
    blocks = []
    for i in range(n_blocks):
        b = block_cls(in_planes, planes, stride if i == 0 else 1, **kw)
        blocks.append(b)
        in_planes = planes * b.expansion
    return nn.Sequential(*blocks), in_planes


def embedding_head(module, stats_dim, n_stats, embedding_size, two_emb_layer):
    module.seg_1 = nn.Linear(stats_dim * n_stats, embedding_size)
    if two_emb_layer:
        module.seg_bn_1 = nn.BatchNorm1d(embedding_size, affine=False)
        module.seg_2 = nn.Linear(embedding_size, embedding_size)
    else:
        module.seg_bn_1 = nn.Identity()
        module.seg_2 = nn.Identity()
