"""Pooling heads of ``speakerlab/models/eres2net/pooling_layers.py`` (parameter layout).

TSTP (``:38-55``) is what every registry model uses; it runs as the HIP ``tstp`` kernel
(mean and sqrt(unbiased var + 1e-8) over time).  TAP/TSDP/ASTP keep their constructor
and parameter layout for ``getattr(pooling_layers, name)`` compatibility.
"""
import torch.nn as nn

from speakerlab.models.eres2net.fusion import _FusedOnly


class TAP(_FusedOnly):
    def __init__(self, **kwargs):
        super().__init__()


class TSDP(_FusedOnly):
    def __init__(self, **kwargs):
        super().__init__()


class TSTP(_FusedOnly):
    def __init__(self, **kwargs):
        super().__init__()


class ASTP(_FusedOnly):
    def __init__(self, in_dim, bottleneck_dim=128, global_context_att=False):
        super().__init__()
        self.global_context_att = global_context_att
        self.linear1 = nn.Conv1d(in_dim * (3 if global_context_att else 1), bottleneck_dim, kernel_size=1)
        self.linear2 = nn.Conv1d(bottleneck_dim, in_dim, kernel_size=1)
