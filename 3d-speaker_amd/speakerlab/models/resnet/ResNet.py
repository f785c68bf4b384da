"""ResNet — drop-in for ``speakerlab.models.resnet.ResNet.ResNet`` (reference
``speakerlab/models/resnet/ResNet.py:15-113``; ResNet34 = num_blocks [3, 4, 6, 3]).

Same constructor and ``state_dict`` keys; the forward (stem, four stages of BasicBlocks,
TSTP, seg_1 [-> ReLU -> seg_bn_1 -> seg_2]) is one native plan (``csrc/resnet.cpp``, arch
SPK_ARCH_RESNET).  The blocks are parameter containers only.
"""
import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.eres2net import pooling_layers
from speakerlab.models.eres2net._resnet2d import embedding_head
from speakerlab.models.eres2net.fusion import _FusedOnly

__all__ = ['BasicBlock', 'ResNet']


class BasicBlock(_FusedOnly):
    """conv3x3(stride) + BN + ReLU -> conv3x3 + BN -> + shortcut -> ReLU (ResNet.py:15-35)."""
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(self.expansion * planes))


class ResNet(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_RESNET

    def __init__(self, block=BasicBlock, num_blocks=[3, 4, 6, 3], m_channels=32, feat_dim=40, embedding_size=128,
                 pooling_func='TSTP', two_emb_layer=True):
        super().__init__()
        if pooling_func != 'TSTP':
            raise NotImplementedError('the MI355X executor implements TSTP pooling')
        if block is not BasicBlock:
            raise NotImplementedError('the MI355X executor implements the BasicBlock ResNet')
        self.in_planes = m_channels
        self.feat_dim, self.embedding_size, self.two_emb_layer = feat_dim, embedding_size, two_emb_layer
        self.m_channels, self.num_blocks = m_channels, list(num_blocks)
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
                    base_width=0, scale=0, expansion=1, two_emb_layer=int(bool(self.two_emb_layer)))

    def forward(self, x):
        """x: [B, T, feat_dim] float32 on a ROCm device -> [B, embedding_size]."""
        return self._hip_forward(x)
