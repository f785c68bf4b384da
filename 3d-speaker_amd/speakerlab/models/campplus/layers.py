"""CAM++ layers — parameter layout of ``speakerlab/models/campplus/layers.py:10-253``.

All computation happens in the fused CAM++ plan (``csrc/campplus.cpp``): BN-ReLU
pre-activations are folded into the consuming 1x1 GEMMs where possible, the dense
``torch.cat`` growth is a preallocated channel buffer written in place, and CAMLayer's
context (mean + 100-frame segment average) + gate run as a reduction, two tiny GEMMs and
a gated epilogue.
"""
import torch.nn as nn

from speakerlab.models.eres2net.fusion import _FusedOnly


def get_nonlinear(config_str, channels):
    seq = nn.Sequential()
    for name in config_str.split('-'):
        if name == 'relu':
            seq.add_module('relu', nn.ReLU(inplace=True))
        elif name == 'prelu':
            seq.add_module('prelu', nn.PReLU(channels))
        elif name == 'batchnorm':
            seq.add_module('batchnorm', nn.BatchNorm1d(channels))
        elif name == 'batchnorm_':
            seq.add_module('batchnorm', nn.BatchNorm1d(channels, affine=False))
        else:
            raise ValueError('Unexpected module ({}).'.format(name))
    return seq


class StatsPool(_FusedOnly):
    pass


class TDNNLayer(_FusedOnly):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, bias=False,
                 config_str='batchnorm-relu'):
        super().__init__()
        if padding < 0:
            assert kernel_size % 2 == 1
            padding = (kernel_size - 1) // 2 * dilation
        self.linear = nn.Conv1d(in_channels, out_channels, kernel_size, stride=stride, padding=padding,
                                dilation=dilation, bias=bias)
        self.nonlinear = get_nonlinear(config_str, out_channels)


class CAMLayer(_FusedOnly):
    def __init__(self, bn_channels, out_channels, kernel_size, stride, padding, dilation, bias, reduction=2):
        super().__init__()
        self.linear_local = nn.Conv1d(bn_channels, out_channels, kernel_size, stride=stride, padding=padding,
                                      dilation=dilation, bias=bias)
        self.linear1 = nn.Conv1d(bn_channels, bn_channels // reduction, 1)
        self.relu = nn.ReLU(inplace=True)
        self.linear2 = nn.Conv1d(bn_channels // reduction, out_channels, 1)
        self.sigmoid = nn.Sigmoid()


class CAMDenseTDNNLayer(_FusedOnly):
    def __init__(self, in_channels, out_channels, bn_channels, kernel_size, stride=1, dilation=1, bias=False,
                 config_str='batchnorm-relu', memory_efficient=False):
        super().__init__()
        assert kernel_size % 2 == 1
        self.memory_efficient = memory_efficient
        self.nonlinear1 = get_nonlinear(config_str, in_channels)
        self.linear1 = nn.Conv1d(in_channels, bn_channels, 1, bias=False)
        self.nonlinear2 = get_nonlinear(config_str, bn_channels)
        self.cam_layer = CAMLayer(bn_channels, out_channels, kernel_size, stride=stride,
                                  padding=(kernel_size - 1) // 2 * dilation, dilation=dilation, bias=bias)


class CAMDenseTDNNBlock(nn.ModuleList):
    def __init__(self, num_layers, in_channels, out_channels, bn_channels, kernel_size, stride=1, dilation=1,
                 bias=False, config_str='batchnorm-relu', memory_efficient=False):
        super().__init__()
        for i in range(num_layers):
            self.add_module('tdnnd%d' % (i + 1), CAMDenseTDNNLayer(
                in_channels=in_channels + i * out_channels, out_channels=out_channels, bn_channels=bn_channels,
                kernel_size=kernel_size, stride=stride, dilation=dilation, bias=bias, config_str=config_str,
                memory_efficient=memory_efficient))


class TransitLayer(_FusedOnly):
    def __init__(self, in_channels, out_channels, bias=True, config_str='batchnorm-relu'):
        super().__init__()
        self.nonlinear = get_nonlinear(config_str, in_channels)
        self.linear = nn.Conv1d(in_channels, out_channels, 1, bias=bias)


class DenseLayer(_FusedOnly):
    def __init__(self, in_channels, out_channels, bias=False, config_str='batchnorm-relu'):
        super().__init__()
        self.linear = nn.Conv1d(in_channels, out_channels, 1, bias=bias)
        self.nonlinear = get_nonlinear(config_str, out_channels)


class BasicResBlock(_FusedOnly):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, stride=(stride, 1), padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=(stride, 1), bias=False),
                nn.BatchNorm2d(self.expansion * planes))
