"""ResNet / ResNeXt family, written for NHWC (channels_last) bf16 training on MI355X.

The reference never defines these networks itself: it pulls them from torchvision /
pretrainedmodels (`mlcomp/contrib/model/pretrained.py:8-60`,
`mlcomp/contrib/segmentation/encoders/resnet.py:7-63`).  Neither package exists on
this image, so the architectures are re-implemented here from the published
definitions (He et al. 2015; Xie et al. 2016), with parameter names that match the
torchvision state-dict layout (``conv1``, ``bn1``, ``layer{1..4}.{i}.conv{1..3}``,
``downsample.0/1``, ``fc``) so checkpoints stay interchangeable.

Every conv is followed by a BatchNorm (and usually a ReLU); the blocks are built from
:class:`ConvBNAct` so the native engine (`mlcomp_amd.ops.fused`) can replace each
conv+BN(+ReLU)(+residual) group with a single fused HIP path instead of pattern
matching an arbitrary graph.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Type, Union

import torch
import torch.nn as nn
import torch.nn.functional as F


class ConvBNAct(nn.Module):
    """conv -> BN -> (ReLU).  Unit the native engine fuses.

    Parameter names are chosen so that a parent module can alias them to the
    torchvision names (``conv1``/``bn1`` ...) via the `_tv_names` map of the block.
    """

    def __init__(self, cin: int, cout: int, k: int, stride: int = 1,
                 padding: Optional[int] = None, groups: int = 1, act: bool = True,
                 dilation: int = 1, zero_init_gamma: bool = False):
        super().__init__()
        if padding is None:
            padding = ((k - 1) // 2) * dilation
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding,
                              groups=groups, bias=False, dilation=dilation)
        self.bn = nn.BatchNorm2d(cout)
        if zero_init_gamma:
            nn.init.zeros_(self.bn.weight)
        self.act = act

    def forward(self, x, residual=None):
        y = self.bn(self.conv(x))
        if residual is not None:
            y = y + residual
        if self.act:
            y = F.relu(y)
        return y


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, downsample=None, groups=1,
                 base_width=64, dilation=1):
        super().__init__()
        if groups != 1 or base_width != 64:
            raise ValueError('BasicBlock only supports groups=1 and base_width=64')
        self.cb1 = ConvBNAct(cin, planes, 3, stride, dilation=dilation)
        # the last BN of a block adds the residual before the ReLU
        self.cb2 = ConvBNAct(planes, planes, 3, 1, dilation=dilation, act=True)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        y = self.cb1(x)
        return self.cb2(y, residual=identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None, groups=1,
                 base_width=64, dilation=1):
        super().__init__()
        width = int(planes * (base_width / 64.0)) * groups
        # stride on the 3x3 (torchvision "ResNet v1.5")
        self.cb1 = ConvBNAct(cin, width, 1, 1)
        self.cb2 = ConvBNAct(width, width, 3, stride, groups=groups, dilation=dilation)
        self.cb3 = ConvBNAct(width, planes * self.expansion, 1, 1, act=True)
        self.downsample = downsample

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        y = self.cb1(x)
        y = self.cb2(y)
        return self.cb3(y, residual=identity)


class Downsample(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.cb = ConvBNAct(cin, cout, 1, stride, padding=0, act=False)

    def forward(self, x):
        return self.cb(x)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: Sequence[int],
                 num_classes: int = 1000, groups: int = 1, width_per_group: int = 64,
                 in_channels: int = 3, replace_stride_with_dilation=(False, False, False),
                 include_top: bool = True):
        super().__init__()
        self.inplanes = 64
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        self.stem = ConvBNAct(in_channels, 64, 7, 2, padding=3)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], 2, replace_stride_with_dilation[0])
        self.layer3 = self._make_layer(block, 256, layers[2], 2, replace_stride_with_dilation[1])
        self.layer4 = self._make_layer(block, 512, layers[3], 2, replace_stride_with_dilation[2])
        self.out_channels = 512 * block.expansion
        self.include_top = include_top
        if include_top:
            self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        # zero-init the last BN gamma of every residual branch (Goyal et al. 2017)
        for m in self.modules():
            if isinstance(m, Bottleneck):
                nn.init.zeros_(m.cb3.bn.weight)
            elif isinstance(m, BasicBlock):
                nn.init.zeros_(m.cb2.bn.weight)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = Downsample(self.inplanes, planes * block.expansion, stride)
        layers = [block(self.inplanes, planes, stride, downsample, self.groups,
                        self.base_width, previous_dilation)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups,
                                base_width=self.base_width, dilation=self.dilation))
        return nn.Sequential(*layers)

    def forward_features(self, x) -> List[torch.Tensor]:
        """Encoder outputs deepest-first, like the reference's ResNetEncoder
        (`mlcomp/contrib/segmentation/encoders/resnet.py:14-27`)."""
        x0 = self.stem(x)
        x1 = self.layer1(self.maxpool(x0))
        x2 = self.layer2(x1)
        x3 = self.layer3(x2)
        x4 = self.layer4(x3)
        return [x4, x3, x2, x1, x0]

    def forward(self, x):
        x = self.stem(x)
        x = self.maxpool(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        if not self.include_top:
            return x
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


_SPECS = {
    'resnet18': (BasicBlock, [2, 2, 2, 2], 1, 64),
    'resnet34': (BasicBlock, [3, 4, 6, 3], 1, 64),
    'resnet50': (Bottleneck, [3, 4, 6, 3], 1, 64),
    'resnet101': (Bottleneck, [3, 4, 23, 3], 1, 64),
    'resnet152': (Bottleneck, [3, 8, 36, 3], 1, 64),
    'resnext50_32x4d': (Bottleneck, [3, 4, 6, 3], 32, 4),
    'resnext101_32x4d': (Bottleneck, [3, 4, 23, 3], 32, 4),
    'resnext101_32x8d': (Bottleneck, [3, 4, 23, 3], 32, 8),
    'resnext101_64x4d': (Bottleneck, [3, 4, 23, 3], 64, 4),
    'wide_resnet50_2': (Bottleneck, [3, 4, 6, 3], 1, 128),
    'wide_resnet101_2': (Bottleneck, [3, 4, 23, 3], 1, 128),
}

# output channel shapes deepest-first, as in the reference encoder table
OUT_SHAPES = {
    'resnet18': (512, 256, 128, 64, 64),
    'resnet34': (512, 256, 128, 64, 64),
    'resnet50': (2048, 1024, 512, 256, 64),
    'resnet101': (2048, 1024, 512, 256, 64),
    'resnet152': (2048, 1024, 512, 256, 64),
    'resnext50_32x4d': (2048, 1024, 512, 256, 64),
    'resnext101_32x4d': (2048, 1024, 512, 256, 64),
    'resnext101_32x8d': (2048, 1024, 512, 256, 64),
    'resnext101_64x4d': (2048, 1024, 512, 256, 64),
    'wide_resnet50_2': (2048, 1024, 512, 256, 64),
    'wide_resnet101_2': (2048, 1024, 512, 256, 64),
}


def resnet(variant: str = 'resnet50', num_classes: int = 1000, **kw) -> ResNet:
    if variant not in _SPECS:
        raise KeyError(f'unknown resnet variant {variant!r}; known: {sorted(_SPECS)}')
    block, layers, groups, wpg = _SPECS[variant]
    return ResNet(block, layers, num_classes=num_classes, groups=groups,
                  width_per_group=wpg, **kw)


def resnet18(**kw):
    return resnet('resnet18', **kw)


def resnet34(**kw):
    return resnet('resnet34', **kw)


def resnet50(**kw):
    return resnet('resnet50', **kw)


def resnet101(**kw):
    return resnet('resnet101', **kw)


def resnet152(**kw):
    return resnet('resnet152', **kw)
