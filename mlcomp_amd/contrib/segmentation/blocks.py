"""Building blocks shared by the segmentation decoders
(`mlcomp/contrib/segmentation/common/blocks.py`)."""
from __future__ import annotations

import torch
import torch.nn as nn


class ConvBnRelu(nn.Sequential):
    """conv (no bias when followed by BN) -> [BN] -> ReLU."""

    def __init__(self, cin, cout, kernel_size=3, padding=None, stride=1, use_batchnorm=True, dilation=1):
        if padding is None:
            padding = (kernel_size // 2) * dilation if isinstance(kernel_size, int) else 0
        layers = [nn.Conv2d(cin, cout, kernel_size, stride=stride, padding=padding, dilation=dilation,
                            bias=not use_batchnorm)]
        if use_batchnorm:
            layers.append(nn.BatchNorm2d(cout))
        layers.append(nn.ReLU(inplace=True))
        super().__init__(*layers)


Conv2dReLU = ConvBnRelu   # the reference's name


class SCSE(nn.Module):
    """Concurrent spatial and channel squeeze-and-excitation (Roy et al. 2018):
    x * sigmoid(channel gate) + x * sigmoid(spatial gate)."""

    def __init__(self, channels, reduction=16):
        super().__init__()
        hidden = max(1, channels // reduction)
        self.cse = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(channels, hidden, 1), nn.ReLU(inplace=True),
                                 nn.Conv2d(hidden, channels, 1), nn.Sigmoid())
        self.sse = nn.Sequential(nn.Conv2d(channels, 1, 1), nn.Sigmoid())

    def forward(self, x):
        return x * self.cse(x) + x * self.sse(x)


def init_weights(module: nn.Module):
    for m in module.modules():
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)


def make_activation(activation):
    if activation is None or callable(activation):
        return activation
    if activation == 'softmax':
        return nn.Softmax(dim=1)
    if activation == 'sigmoid':
        return nn.Sigmoid()
    raise ValueError('Activation should be "sigmoid"/"softmax"/callable/None')


__all__ = ['ConvBnRelu', 'Conv2dReLU', 'SCSE', 'init_weights', 'make_activation']
