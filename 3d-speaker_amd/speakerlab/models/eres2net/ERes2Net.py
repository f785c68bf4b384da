"""ERes2Net — drop-in for ``speakerlab.models.eres2net.ERes2Net.ERes2Net``
(reference ``speakerlab/models/eres2net/ERes2Net.py:154-231``).  With ``m_channels=64``
it is the 22.46 M "ERes2Net-large" of BASELINE config 4.

Same constructor and ``state_dict`` keys; the forward (stem, 4 Res2Net stages, three
stride-2 3x3 downsamples + AFF bottom-up fusions, TSTP, seg_1) is one native plan
(``csrc/eres2net.cpp``, arch SPK_ARCH_ERES2NET).
"""
import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.eres2net import pooling_layers
from speakerlab.models.eres2net._resnet2d import ReLU, Res2Block, embedding_head, make_stage
from speakerlab.models.eres2net.fusion import AFF

__all__ = ['ReLU', 'BasicBlockERes2Net', 'BasicBlockERes2Net_diff_AFF', 'ERes2Net']


class BasicBlockERes2Net(Res2Block):
    expansion = 2

    def __init__(self, in_planes, planes, stride=1, baseWidth=32, scale=2):
        super().__init__(in_planes, planes, stride, baseWidth, scale, 2, use_aff=False)


class BasicBlockERes2Net_diff_AFF(Res2Block):
    expansion = 2

    def __init__(self, in_planes, planes, stride=1, baseWidth=32, scale=2):
        super().__init__(in_planes, planes, stride, baseWidth, scale, 2, use_aff=True)


class ERes2Net(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_ERES2NET
    _block_cfg = dict(baseWidth=32, scale=2, expansion=2)

    def __init__(self, block=BasicBlockERes2Net, block_fuse=BasicBlockERes2Net_diff_AFF, num_blocks=[3, 4, 6, 3],
                 m_channels=32, feat_dim=80, embedding_size=192, pooling_func='TSTP', two_emb_layer=False):
        super().__init__()
        self.pooling_func = pooling_func
        pooling_layers.pooling_code(pooling_func)   # TSTP / TAP / TSDP / ASTP
        self.feat_dim, self.embedding_size, self.two_emb_layer = feat_dim, embedding_size, two_emb_layer
        self.m_channels = m_channels
        self.stats_dim = int(feat_dim / 8) * m_channels * 8
        m, e = m_channels, block.expansion
        self.conv1 = nn.Conv2d(1, m, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(m)
        c = m
        self.layer1, c = make_stage(block, c, m, num_blocks[0], 1)
        self.layer2, c = make_stage(block, c, m * 2, num_blocks[1], 2)
        self.layer3, c = make_stage(block_fuse, c, m * 4, num_blocks[2], 2)
        self.layer4, c = make_stage(block_fuse, c, m * 8, num_blocks[3], 2)
        self.in_planes = c
        # three stride-2 3x3 downsamples + AFF bottom-up fusions (ERes2Net.py:178-186)
        ds = dict(kernel_size=3, stride=2, padding=1, bias=False)
        self.layer1_downsample = nn.Conv2d(m * e, m * e * 2, **ds)
        self.layer2_downsample = nn.Conv2d(m * e * 2, m * e * 4, **ds)
        self.layer3_downsample = nn.Conv2d(m * e * 4, m * e * 8, **ds)
        self.fuse_mode12 = AFF(channels=m * e * 2)
        self.fuse_mode123 = AFF(channels=m * e * 4)
        self.fuse_mode1234 = AFF(channels=m * e * 8)
        self.n_stats = pooling_layers.n_stats(pooling_func)
        self.pool = getattr(pooling_layers, pooling_func)(in_dim=self.stats_dim * e)
        embedding_head(self, self.stats_dim * e, self.n_stats, embedding_size, two_emb_layer)

    def _hip_config(self):
        b = self._block_cfg
        return dict(feat_dim=self.feat_dim, embed_dim=self.embedding_size, m_channels=self.m_channels,
                    base_width=b['baseWidth'], scale=b['scale'], expansion=b['expansion'],
                    two_emb_layer=int(bool(self.two_emb_layer)),
                    pooling=pooling_layers.pooling_code(self.pooling_func))

    def forward(self, x):
        """x: [B, T, feat_dim] float32 on a ROCm device -> [B, embedding_size]."""
        return self._hip_forward(x)
