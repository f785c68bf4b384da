"""ERes2Net-huge — drop-in for ``speakerlab.models.eres2net.ERes2Net_huge.ERes2Net``
(reference ``speakerlab/models/eres2net/ERes2Net_huge.py:30-232``: blocks with expansion 4,
baseWidth 24, scale 3; m_channels 64).  Registry ``ERes2Net_COMMON`` (``infer_sv_batch.py:78-84``).

Same executor as ERes2Net (SPK_ARCH_ERES2NET) with the block hyper-parameters passed in the
config; same ``state_dict`` layout as the reference.
"""
from speakerlab.models.eres2net import ERes2Net as _e
from speakerlab.models.eres2net._resnet2d import ReLU, Res2Block

__all__ = ['ReLU', 'BasicBlockERes2Net', 'BasicBlockERes2Net_diff_AFF', 'ERes2Net']


class BasicBlockERes2Net(Res2Block):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, baseWidth=24, scale=3):
        super().__init__(in_planes, planes, stride, baseWidth, scale, 4, use_aff=False)


class BasicBlockERes2Net_diff_AFF(Res2Block):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, baseWidth=24, scale=3):
        super().__init__(in_planes, planes, stride, baseWidth, scale, 4, use_aff=True)


class ERes2Net(_e.ERes2Net):
    _block_cfg = dict(baseWidth=24, scale=3, expansion=4)

    def __init__(self, block=BasicBlockERes2Net, block_fuse=BasicBlockERes2Net_diff_AFF, num_blocks=[3, 4, 6, 3],
                 m_channels=64, feat_dim=80, embedding_size=192, pooling_func='TSTP', two_emb_layer=False):
        super().__init__(block, block_fuse, num_blocks, m_channels, feat_dim, embedding_size, pooling_func,
                         two_emb_layer)
