"""ECAPA-TDNN — drop-in for ``speakerlab.models.ecapa_tdnn.ECAPA_TDNN.ECAPA_TDNN``
(reference ``speakerlab/models/ecapa_tdnn/ECAPA_TDNN.py:350-463``; registry config
``infer_sv_batch.py:113-120``: input 80, lin_neurons 192, channels [1024]*4 + [3072]).

Same constructor and ``state_dict`` keys (231 tensors).  The forward is one native plan
(``csrc/ecapa.cpp``): reflect-'same' Conv1d folded into the operand loader, conv -> ReLU
-> BN as a GEMM epilogue (BN after the activation is a post-affine, not folded), the
Res2Net chain with the ``x_i + y_{i-1}`` add in the operand load, SE and attentive
statistics pooling as reductions + small GEMMs.
"""
import torch
import torch.nn as nn

from speakerlab import _hip
from speakerlab.models.eres2net.fusion import _FusedOnly

__all__ = ['Conv1d', 'BatchNorm1d', 'TDNNBlock', 'Res2NetBlock', 'SEBlock', 'AttentiveStatisticsPooling',
           'SERes2NetBlock', 'ECAPA_TDNN']


class Conv1d(_FusedOnly):
    """speechbrain-style wrapper: the actual nn.Conv1d lives at ``.conv`` (padding done by
    the wrapper: 'same' with reflect mode, ``ECAPA_TDNN.py:42-106``)."""

    def __init__(self, out_channels, kernel_size, in_channels, stride=1, dilation=1, padding='same', groups=1,
                 bias=True, padding_mode='reflect'):
        super().__init__()
        self.kernel_size, self.stride, self.dilation = kernel_size, stride, dilation
        self.padding, self.padding_mode = padding, padding_mode
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, stride=stride, dilation=dilation, padding=0,
                              groups=groups, bias=bias)


class BatchNorm1d(_FusedOnly):
    def __init__(self, input_size, eps=1e-05, momentum=0.1):
        super().__init__()
        self.norm = nn.BatchNorm1d(input_size, eps=eps, momentum=momentum)


class TDNNBlock(_FusedOnly):
    def __init__(self, in_channels, out_channels, kernel_size, dilation, activation=nn.ReLU, groups=1):
        super().__init__()
        self.conv = Conv1d(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                           dilation=dilation, groups=groups)
        self.activation = activation()
        self.norm = BatchNorm1d(input_size=out_channels)


class Res2NetBlock(_FusedOnly):
    def __init__(self, in_channels, out_channels, scale=8, kernel_size=3, dilation=1):
        super().__init__()
        assert in_channels % scale == 0 and out_channels % scale == 0
        self.scale = scale
        self.blocks = nn.ModuleList(
            TDNNBlock(in_channels // scale, out_channels // scale, kernel_size=kernel_size, dilation=dilation)
            for _ in range(scale - 1))


class SEBlock(_FusedOnly):
    def __init__(self, in_channels, se_channels, out_channels):
        super().__init__()
        self.conv1 = Conv1d(in_channels=in_channels, out_channels=se_channels, kernel_size=1)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = Conv1d(in_channels=se_channels, out_channels=out_channels, kernel_size=1)
        self.sigmoid = nn.Sigmoid()


class AttentiveStatisticsPooling(_FusedOnly):
    def __init__(self, channels, attention_channels=128, global_context=True):
        super().__init__()
        self.eps = 1e-12
        self.global_context = global_context
        self.tdnn = TDNNBlock(channels * (3 if global_context else 1), attention_channels, 1, 1)
        self.tanh = nn.Tanh()
        self.conv = Conv1d(in_channels=attention_channels, out_channels=channels, kernel_size=1)


class SERes2NetBlock(_FusedOnly):
    def __init__(self, in_channels, out_channels, res2net_scale=8, se_channels=128, kernel_size=1, dilation=1,
                 activation=nn.ReLU, groups=1):
        super().__init__()
        self.out_channels = out_channels
        self.tdnn1 = TDNNBlock(in_channels, out_channels, kernel_size=1, dilation=1, activation=activation,
                               groups=groups)
        self.res2net_block = Res2NetBlock(out_channels, out_channels, res2net_scale, kernel_size, dilation)
        self.tdnn2 = TDNNBlock(out_channels, out_channels, kernel_size=1, dilation=1, activation=activation,
                               groups=groups)
        self.se_block = SEBlock(out_channels, se_channels, out_channels)
        self.shortcut = None
        if in_channels != out_channels:
            self.shortcut = Conv1d(in_channels=in_channels, out_channels=out_channels, kernel_size=1)


class ECAPA_TDNN(_hip.HipModuleMixin, nn.Module):
    _hip_arch = _hip.ARCH_ECAPA

    def __init__(self, input_size, device='cpu', lin_neurons=192, activation=nn.ReLU,
                 channels=[512, 512, 512, 512, 1536], kernel_sizes=[5, 3, 3, 3, 1], dilations=[1, 2, 3, 4, 1],
                 attention_channels=128, res2net_scale=8, se_channels=128, global_context=True,
                 groups=[1, 1, 1, 1, 1]):
        super().__init__()
        assert len(channels) == len(kernel_sizes) == len(dilations)
        if any(g != 1 for g in groups) or not global_context or len(channels) != 5:
            raise NotImplementedError('MI355X executor: groups=1, global_context=True, 3 SE-Res2Net blocks')
        self.channels, self.kernel_sizes, self.dilations = list(channels), list(kernel_sizes), list(dilations)
        self.input_size, self.lin_neurons = input_size, lin_neurons
        self.blocks = nn.ModuleList([TDNNBlock(input_size, channels[0], kernel_sizes[0], dilations[0], activation,
                                               groups[0])])
        for i in range(1, len(channels) - 1):
            self.blocks.append(SERes2NetBlock(channels[i - 1], channels[i], res2net_scale=res2net_scale,
                                              se_channels=se_channels, kernel_size=kernel_sizes[i],
                                              dilation=dilations[i], activation=activation, groups=groups[i]))
        self.mfa = TDNNBlock(channels[-1], channels[-1], kernel_sizes[-1], dilations[-1], activation,
                             groups=groups[-1])
        self.asp = AttentiveStatisticsPooling(channels[-1], attention_channels=attention_channels,
                                              global_context=global_context)
        self.asp_bn = BatchNorm1d(input_size=channels[-1] * 2)
        self.fc = Conv1d(in_channels=channels[-1] * 2, out_channels=lin_neurons, kernel_size=1)

    def _hip_config(self):
        return dict(feat_dim=self.input_size, embed_dim=self.lin_neurons, channels=self.channels,
                    kernel_sizes=self.kernel_sizes, dilations=self.dilations)

    def forward(self, x, lengths=None):
        """x: [B, T, input_size] on a ROCm device -> [B, lin_neurons].

        ``lengths`` (reference semantics, ``ECAPA_TDNN.py:209-287, 430-454``): RELATIVE
        lengths in (0, 1]; the convolutions still see the whole padded input and only the SE
        squeeze means and the attentive-pooling statistics are masked to the frames
        ``t < lengths[b] * T`` (``length_to_mask``).  The mask is evaluated here exactly as
        the reference builds it (same dtype arithmetic), then passed to the kernels as
        valid-frame counts."""
        if lengths is None:
            return self._hip_forward(x)
        T = x.shape[1]
        rel = torch.as_tensor(lengths)
        if rel.dim() != 1 or rel.numel() != x.shape[0]:
            raise ValueError(f'lengths must be 1-D with {x.shape[0]} entries')
        if not rel.is_floating_point():
            rel = rel.float()
        rel = rel.detach().cpu()
        frames = (torch.arange(T, dtype=rel.dtype).expand(len(rel), T) < (rel * T).unsqueeze(1)).sum(1)
        if int(frames.min()) < 1:
            raise ValueError('ECAPA lengths: every utterance needs at least one valid frame '
                             '(the reference divides by the mask total)')
        return self._hip_forward(x, lengths=frames.to(torch.int32))
