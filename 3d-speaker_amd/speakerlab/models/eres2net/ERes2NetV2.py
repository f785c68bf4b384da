"""ERes2NetV2 — drop-in for ``speakerlab.models.eres2net.ERes2NetV2.ERes2NetV2``
(reference ``speakerlab/models/eres2net/ERes2NetV2.py:161-254``; registry config
``infer_sv_batch.py:70-76``: feat_dim 80, embedding 192, m 64, baseWidth 26, scale 2,
expansion 2).

Same constructor, same ``state_dict`` keys (557 tensors).  ``forward(x[B,T,F])`` on a ROCm
tensor runs the whole network as one native launch plan: Fbank-compatible input ->
stem -> 4 stages of Res2Net blocks (conv+BN+Hardtanh fused, split/cat as slices) ->
layer3_ds + AFF -> TSTP -> seg_1, all fp32 on MFMA (``csrc/eres2net.cpp``).
"""
import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.eres2net import pooling_layers
from speakerlab.models.eres2net._resnet2d import ReLU, Res2Block, embedding_head, make_stage
from speakerlab.models.eres2net.fusion import AFF

__all__ = ['ReLU', 'BasicBlockERes2NetV2', 'BasicBlockERes2NetV2AFF', 'ERes2NetV2']


class BasicBlockERes2NetV2(Res2Block):
    def __init__(self, in_planes, planes, stride=1, baseWidth=26, scale=2, expansion=2):
        super().__init__(in_planes, planes, stride, baseWidth, scale, expansion, use_aff=False)


class BasicBlockERes2NetV2AFF(Res2Block):
    def __init__(self, in_planes, planes, stride=1, baseWidth=26, scale=2, expansion=2):
        super().__init__(in_planes, planes, stride, baseWidth, scale, expansion, use_aff=True)


class ERes2NetV2(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_ERES2NETV2

    def __init__(self, block=BasicBlockERes2NetV2, block_fuse=BasicBlockERes2NetV2AFF, num_blocks=[3, 4, 6, 3],
                 m_channels=64, feat_dim=80, embedding_size=192, baseWidth=26, scale=2, expansion=2,
                 pooling_func='TSTP', two_emb_layer=False):
        super().__init__()
        self.pooling_func = pooling_func
        pooling_layers.pooling_code(pooling_func)   # TSTP / TAP / TSDP / ASTP
        self.feat_dim, self.embedding_size, self.two_emb_layer = feat_dim, embedding_size, two_emb_layer
        self.m_channels, self.baseWidth, self.scale, self.expansion = m_channels, baseWidth, scale, expansion
        self.stats_dim = int(feat_dim / 8) * m_channels * 8
        kw = dict(baseWidth=baseWidth, scale=scale, expansion=expansion)
        self.conv1 = nn.Conv2d(1, m_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(m_channels)
        c = m_channels
        self.layer1, c = make_stage(block, c, m_channels, num_blocks[0], 1, **kw)
        self.layer2, c = make_stage(block, c, m_channels * 2, num_blocks[1], 2, **kw)
        self.layer3, c = make_stage(block_fuse, c, m_channels * 4, num_blocks[2], 2, **kw)
        self.layer4, c = make_stage(block_fuse, c, m_channels * 8, num_blocks[3], 2, **kw)
        self.in_planes = c
        # bottom-up fusion of stage 3 (downsampled) into stage 4
        self.layer3_ds = nn.Conv2d(m_channels * 4 * expansion, m_channels * 8 * expansion, kernel_size=3, padding=1,
                                   stride=2, bias=False)
        self.fuse34 = AFF(channels=m_channels * 8 * expansion, r=4)
        self.n_stats = pooling_layers.n_stats(pooling_func)
        self.pool = getattr(pooling_layers, pooling_func)(in_dim=self.stats_dim * expansion)
        embedding_head(self, self.stats_dim * expansion, self.n_stats, embedding_size, two_emb_layer)

    def _hip_config(self):
        return dict(feat_dim=self.feat_dim, embed_dim=self.embedding_size, m_channels=self.m_channels,
                    base_width=self.baseWidth, scale=self.scale, expansion=self.expansion,
                    two_emb_layer=int(bool(self.two_emb_layer)),
                    pooling=pooling_layers.pooling_code(self.pooling_func))

    def forward(self, x):
        """x: [B, T, feat_dim] float32 on a ROCm device -> [B, embedding_size]."""
        return self._hip_forward(x)
