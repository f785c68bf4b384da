"""Res2Net — drop-in for ``speakerlab.models.res2net.Res2Net.Res2Net`` (reference
``speakerlab/models/res2net/Res2Net.py:17-147``).

Same constructor and ``state_dict`` keys; the forward (stem, four stages of
BasicBlockRes2Net -- conv1 1x1 -> scale-1 chained 3x3 convs, the last split passed through
to the concat -> conv3 + shortcut, Hardtanh(0, 20) activations -- TSTP, seg_1) is one
native plan (``csrc/resnet.cpp``, arch SPK_ARCH_RES2NET).
"""
import math

import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.eres2net import pooling_layers
from speakerlab.models.eres2net._resnet2d import ReLU, embedding_head
from speakerlab.models.eres2net.fusion import _FusedOnly

__all__ = ['ReLU', 'BasicBlockRes2Net', 'Res2Net']


class BasicBlockRes2Net(_FusedOnly):
    expansion = 2

    def __init__(self, in_planes, planes, stride=1, baseWidth=32, scale=2):
        super().__init__()
        width = int(math.floor(planes * (baseWidth / 64.0)))
        self.conv1 = nn.Conv2d(in_planes, width * scale, kernel_size=1, stride=stride, bias=False)
        self.bn1 = nn.BatchNorm2d(width * scale)
        self.nums = scale - 1
        self.convs = nn.ModuleList(nn.Conv2d(width, width, kernel_size=3, padding=1, bias=False)
                                   for _ in range(self.nums))
        self.bns = nn.ModuleList(nn.BatchNorm2d(width) for _ in range(self.nums))
        self.relu = ReLU(inplace=True)
        self.conv3 = nn.Conv2d(width * scale, planes * self.expansion, kernel_size=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes))
        self.stride, self.width, self.scale = stride, width, scale


class Res2Net(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_RES2NET

    def __init__(self, block=BasicBlockRes2Net, num_blocks=[3, 4, 6, 3], m_channels=32, feat_dim=80,
                 embedding_size=192, pooling_func='TSTP', two_emb_layer=False):
        super().__init__()
        if pooling_func != 'TSTP':
            raise NotImplementedError('the MI355X executor implements TSTP pooling')
        if block is not BasicBlockRes2Net:
            raise NotImplementedError('the MI355X executor implements BasicBlockRes2Net')
        self.in_planes = m_channels
        self.feat_dim, self.embedding_size, self.two_emb_layer = feat_dim, embedding_size, two_emb_layer
        self.m_channels = m_channels
        self.stats_dim = int(feat_dim / 8) * m_channels * 8
        self.conv1 = nn.Conv2d(1, m_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(m_channels)
        self.layer1 = self._make_layer(block, m_channels, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, m_channels * 2, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, m_channels * 4, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, m_channels * 8, num_blocks[3], 2)
        self.n_stats = 2
        self.pool = pooling_layers.TSTP(in_dim=self.stats_dim * block.expansion)
        embedding_head(self, self.stats_dim * block.expansion, self.n_stats, embedding_size, two_emb_layer)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def _hip_config(self):
        return dict(feat_dim=self.feat_dim, embed_dim=self.embedding_size, m_channels=self.m_channels,
                    base_width=32, scale=2, expansion=2, two_emb_layer=int(bool(self.two_emb_layer)))

    def forward(self, x):
        """x: [B, T, feat_dim] float32 on a ROCm device -> [B, embedding_size]."""
        return self._hip_forward(x)
