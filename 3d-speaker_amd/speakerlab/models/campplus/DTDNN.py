"""CAM++ — drop-in for ``speakerlab.models.campplus.DTDNN.CAMPPlus`` (reference
``speakerlab/models/campplus/DTDNN.py:13-115``).  CAMPPlus(embedding_size=512) is the
7.2 M model of BASELINE config 3; the 192-d "common" model uses the same plan.

Same constructor and ``state_dict`` keys (937 tensors); forward = one native plan
(``csrc/campplus.cpp``).
"""
from collections import OrderedDict

import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.campplus.layers import (BasicResBlock, CAMDenseTDNNBlock, DenseLayer, StatsPool, TDNNLayer,
                                               TransitLayer, get_nonlinear)
from speakerlab.models.eres2net.fusion import _FusedOnly


class FCM(_FusedOnly):
    """2-D front-end: conv3x3 -> 2x2 BasicResBlocks (stride 2 on frequency) -> conv3x3 (2,1)."""

    def __init__(self, block=BasicResBlock, num_blocks=[2, 2], m_channels=32, feat_dim=80):
        super().__init__()
        self.in_planes = m_channels
        self.conv1 = nn.Conv2d(1, m_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(m_channels)
        self.layer1 = self._stage(block, m_channels, num_blocks[0], 2)
        self.layer2 = self._stage(block, m_channels, num_blocks[1], 2)
        self.conv2 = nn.Conv2d(m_channels, m_channels, kernel_size=3, stride=(2, 1), padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(m_channels)
        self.out_channels = m_channels * (feat_dim // 8)

    def _stage(self, block, planes, n, stride):
        mods = []
        for s in [stride] + [1] * (n - 1):
            mods.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*mods)


class CAMPPlus(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_CAMPPLUS

    def __init__(self, feat_dim=80, embedding_size=512, growth_rate=32, bn_size=4, init_channels=128,
                 config_str='batchnorm-relu', memory_efficient=True):
        super().__init__()
        if config_str != 'batchnorm-relu':
            raise NotImplementedError('MI355X executor implements config_str="batchnorm-relu"')
        self.feat_dim, self.embedding_size = feat_dim, embedding_size
        self.head = FCM(feat_dim=feat_dim)
        ch = self.head.out_channels
        self.xvector = nn.Sequential(OrderedDict([
            ('tdnn', TDNNLayer(ch, init_channels, 5, stride=2, dilation=1, padding=-1, config_str=config_str))]))
        ch = init_channels
        for i, (n_layers, ksize, dil) in enumerate(zip((12, 24, 16), (3, 3, 3), (1, 2, 2))):
            self.xvector.add_module('block%d' % (i + 1), CAMDenseTDNNBlock(
                num_layers=n_layers, in_channels=ch, out_channels=growth_rate, bn_channels=bn_size * growth_rate,
                kernel_size=ksize, dilation=dil, config_str=config_str, memory_efficient=memory_efficient))
            ch += n_layers * growth_rate
            self.xvector.add_module('transit%d' % (i + 1),
                                    TransitLayer(ch, ch // 2, bias=False, config_str=config_str))
            ch //= 2
        self.xvector.add_module('out_nonlinear', get_nonlinear(config_str, ch))
        self.xvector.add_module('stats', StatsPool())
        self.xvector.add_module('dense', DenseLayer(ch * 2, embedding_size, config_str='batchnorm_'))
        for m in self.modules():
            if isinstance(m, (nn.Conv1d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight.data)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def _hip_config(self):
        return dict(feat_dim=self.feat_dim, embed_dim=self.embedding_size)

    def forward(self, x, lengths=None):
        """x: [B, T, feat_dim] on a ROCm device -> [B, embedding_size].

        ``lengths`` (extension, optional): valid frames of each row for a variable-length
        batch (e.g. from ``speakerlab._hip.fbank_padded``); row b then gets exactly the
        embedding of its first lengths[b] frames on their own."""
        return self._hip_forward(x, lengths=lengths)
