"""The remaining ImageNet classifiers of the reference's per-model presets
(`mlcomp/contrib/catalyst/configs/classify/*.yml`, variants resolved by ``Pretrained``
through the pretrainedmodels package, `mlcomp/contrib/model/pretrained.py:8-58`).
pretrainedmodels is not in this stack, so the architectures are defined here from their
papers, with the same layer widths (parameter counts are pinned by
``tests/test_models_cpu.py``):

* ``xception`` - Chollet 2017: entry / middle (8 x 728) / exit flows of depthwise-separable
  convolutions with residual shortcuts (22.9 M parameters);
* ``inceptionv3`` - Szegedy et al. 2016, Inception-A/B/C/D/E blocks, 299 x 299 input,
  optional auxiliary head (23.8 M without it, 27.2 M with it);
* ``inceptionv4`` - Szegedy et al. 2017, 4 x Inception-A, 7 x Inception-B, 3 x Inception-C
  (42.7 M);
* ``bninception`` - Ioffe & Szegedy 2015, GoogLeNet with batch normalisation and the 5x5
  branches replaced by two 3x3 convolutions (11.3 M);
* ``fbresnet152`` - ResNet-152 with biased convolutions (60.3 M);
* ``cafferesnet101`` - ResNet-101 with the stride on the first 1x1 convolution of each
  downsampling bottleneck, Caffe style (44.5 M);
* ``nasnetamobile`` / ``nasnetalarge`` / ``pnasnet5large`` / ``polynet``: see
  :mod:`mlcomp_amd.models.nas`.

All of them end in ``last_linear`` like the pretrainedmodels versions, take
``num_classes``, and train on the torch engine (autocast bf16, MIOpen convolutions).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register


def _cbr(cin, cout, k, stride=1, padding=0, eps=1e-3, bias=False):
    """conv -> BN -> ReLU (``k`` / ``padding`` may be (h, w) tuples)."""
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, padding, bias=bias), nn.BatchNorm2d(cout, eps=eps),
                         nn.ReLU(inplace=True))


class _Branches(nn.Module):
    """Parallel branches concatenated along channels."""

    def __init__(self, *branches):
        super().__init__()
        self.branches = nn.ModuleList(branches)

    def forward(self, x):
        return torch.cat([b(x) for b in self.branches], 1)


class _Split(nn.Module):
    """A stem followed by parallel heads whose outputs are concatenated (the 1x3 / 3x1
    fan-out of Inception-E / Inception-C)."""

    def __init__(self, stem, *heads):
        super().__init__()
        self.stem = stem
        self.heads = nn.ModuleList(heads)

    def forward(self, x):
        y = self.stem(x)
        return torch.cat([h(y) for h in self.heads], 1)


def _avg_proj(cin, cout, eps=1e-3, count_include_pad=True):
    return nn.Sequential(nn.AvgPool2d(3, 1, 1, count_include_pad=count_include_pad), _cbr(cin, cout, 1, eps=eps))


class _Classifier(nn.Module):
    """features -> global average pool -> (dropout) -> last_linear."""

    def __init__(self, features: nn.Module, width: int, num_classes: int, dropout: float = 0.0):
        super().__init__()
        self.features = features
        self.dropout = nn.Dropout(dropout) if dropout else nn.Identity()
        self.last_linear = nn.Linear(width, num_classes)

    def logits(self, f):
        return self.last_linear(self.dropout(torch.flatten(F.adaptive_avg_pool2d(f, 1), 1)))

    def forward(self, x):
        return self.logits(self.features(x))


# ---------------------------------------------------------------------------- xception
class _SepConv(nn.Sequential):
    def __init__(self, cin, cout, k=3, stride=1, padding=1):
        super().__init__(nn.Conv2d(cin, cin, k, stride, padding, groups=cin, bias=False),
                         nn.Conv2d(cin, cout, 1, bias=False))


class _XBlock(nn.Module):
    def __init__(self, cin, cout, reps, stride, start_with_relu=True, grow_first=True):
        super().__init__()
        self.skip = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
                     if cout != cin or stride != 1 else None)
        widths = ([(cin, cout)] + [(cout, cout)] * (reps - 1) if grow_first
                  else [(cin, cin)] * (reps - 1) + [(cin, cout)])
        layers = []
        for i, (a, b) in enumerate(widths):
            if i or start_with_relu:
                layers.append(nn.ReLU(inplace=False))
            layers += [_SepConv(a, b), nn.BatchNorm2d(b)]
        if stride != 1:
            layers.append(nn.MaxPool2d(3, stride, 1))
        self.rep = nn.Sequential(*layers)

    def forward(self, x):
        return self.rep(x) + (self.skip(x) if self.skip is not None else x)


def xception_features(in_channels=3) -> nn.Sequential:
    return nn.Sequential(
        _cbr(in_channels, 32, 3, 2, eps=1e-5), _cbr(32, 64, 3, eps=1e-5),
        _XBlock(64, 128, 2, 2, start_with_relu=False), _XBlock(128, 256, 2, 2), _XBlock(256, 728, 2, 2),
        *[_XBlock(728, 728, 3, 1) for _ in range(8)],
        _XBlock(728, 1024, 2, 2, grow_first=False),
        _SepConv(1024, 1536), nn.BatchNorm2d(1536), nn.ReLU(inplace=True),
        _SepConv(1536, 2048), nn.BatchNorm2d(2048), nn.ReLU(inplace=True))


@register('xception')
def xception(num_classes: int = 1000, in_channels: int = 3, **kw):
    return _Classifier(xception_features(in_channels), 2048, num_classes)


# ---------------------------------------------------------------------------- inception v3
def _inc_a(cin, pool):
    return _Branches(_cbr(cin, 64, 1),
                     nn.Sequential(_cbr(cin, 48, 1), _cbr(48, 64, 5, padding=2)),
                     nn.Sequential(_cbr(cin, 64, 1), _cbr(64, 96, 3, padding=1), _cbr(96, 96, 3, padding=1)),
                     _avg_proj(cin, pool))


def _inc_b(cin):
    return _Branches(_cbr(cin, 384, 3, 2),
                     nn.Sequential(_cbr(cin, 64, 1), _cbr(64, 96, 3, padding=1), _cbr(96, 96, 3, 2)),
                     nn.MaxPool2d(3, 2))


def _inc_c(cin, c7):
    return _Branches(_cbr(cin, 192, 1),
                     nn.Sequential(_cbr(cin, c7, 1), _cbr(c7, c7, (1, 7), padding=(0, 3)),
                                   _cbr(c7, 192, (7, 1), padding=(3, 0))),
                     nn.Sequential(_cbr(cin, c7, 1), _cbr(c7, c7, (7, 1), padding=(3, 0)),
                                   _cbr(c7, c7, (1, 7), padding=(0, 3)), _cbr(c7, c7, (7, 1), padding=(3, 0)),
                                   _cbr(c7, 192, (1, 7), padding=(0, 3))),
                     _avg_proj(cin, 192))


def _inc_d(cin):
    return _Branches(nn.Sequential(_cbr(cin, 192, 1), _cbr(192, 320, 3, 2)),
                     nn.Sequential(_cbr(cin, 192, 1), _cbr(192, 192, (1, 7), padding=(0, 3)),
                                   _cbr(192, 192, (7, 1), padding=(3, 0)), _cbr(192, 192, 3, 2)),
                     nn.MaxPool2d(3, 2))


def _fan13(c, out):
    return (_cbr(c, out, (1, 3), padding=(0, 1)), _cbr(c, out, (3, 1), padding=(1, 0)))


def _inc_e(cin):
    return _Branches(_cbr(cin, 320, 1),
                     _Split(_cbr(cin, 384, 1), *_fan13(384, 384)),
                     _Split(nn.Sequential(_cbr(cin, 448, 1), _cbr(448, 384, 3, padding=1)), *_fan13(384, 384)),
                     _avg_proj(cin, 192))


class InceptionV3(nn.Module):
    def __init__(self, num_classes=1000, in_channels=3, aux_logits=False, dropout=0.5):
        super().__init__()
        self.stem = nn.Sequential(_cbr(in_channels, 32, 3, 2), _cbr(32, 32, 3), _cbr(32, 64, 3, padding=1),
                                  nn.MaxPool2d(3, 2), _cbr(64, 80, 1), _cbr(80, 192, 3), nn.MaxPool2d(3, 2))
        self.mixed6 = nn.Sequential(_inc_a(192, 32), _inc_a(256, 64), _inc_a(288, 64), _inc_b(288),
                                    _inc_c(768, 128), _inc_c(768, 160), _inc_c(768, 160), _inc_c(768, 192))
        self.aux = (nn.Sequential(nn.AvgPool2d(5, 3), _cbr(768, 128, 1), _cbr(128, 768, 5),
                                  nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(768, num_classes))
                    if aux_logits else None)
        self.mixed7 = nn.Sequential(_inc_d(768), _inc_e(1280), _inc_e(2048))
        self.head = _Classifier(nn.Identity(), 2048, num_classes, dropout)
        self.last_linear = self.head.last_linear

    def forward(self, x):
        f = self.mixed6(self.stem(x))
        aux = self.aux(f) if (self.aux is not None and self.training) else None
        y = self.head(self.mixed7(f))
        return (y, aux) if aux is not None else y


@register('inceptionv3')
def inceptionv3(num_classes: int = 1000, **kw):
    return InceptionV3(num_classes, **kw)


# ---------------------------------------------------------------------------- inception v4
def _v4_a():
    return _Branches(_cbr(384, 96, 1),
                     nn.Sequential(_cbr(384, 64, 1), _cbr(64, 96, 3, padding=1)),
                     nn.Sequential(_cbr(384, 64, 1), _cbr(64, 96, 3, padding=1), _cbr(96, 96, 3, padding=1)),
                     _avg_proj(384, 96, count_include_pad=False))


def _v4_b():
    return _Branches(_cbr(1024, 384, 1),
                     nn.Sequential(_cbr(1024, 192, 1), _cbr(192, 224, (1, 7), padding=(0, 3)),
                                   _cbr(224, 256, (7, 1), padding=(3, 0))),
                     nn.Sequential(_cbr(1024, 192, 1), _cbr(192, 192, (7, 1), padding=(3, 0)),
                                   _cbr(192, 224, (1, 7), padding=(0, 3)), _cbr(224, 224, (7, 1), padding=(3, 0)),
                                   _cbr(224, 256, (1, 7), padding=(0, 3))),
                     _avg_proj(1024, 128, count_include_pad=False))


def _v4_c():
    return _Branches(_cbr(1536, 256, 1),
                     _Split(_cbr(1536, 384, 1), *_fan13(384, 256)),
                     _Split(nn.Sequential(_cbr(1536, 384, 1), _cbr(384, 448, (3, 1), padding=(1, 0)),
                                          _cbr(448, 512, (1, 3), padding=(0, 1))), *_fan13(512, 256)),
                     _avg_proj(1536, 256, count_include_pad=False))


def inceptionv4_features(in_channels=3) -> nn.Sequential:
    return nn.Sequential(
        _cbr(in_channels, 32, 3, 2), _cbr(32, 32, 3), _cbr(32, 64, 3, padding=1),
        _Branches(nn.MaxPool2d(3, 2), _cbr(64, 96, 3, 2)),                                   # 160
        _Branches(nn.Sequential(_cbr(160, 64, 1), _cbr(64, 96, 3)),
                  nn.Sequential(_cbr(160, 64, 1), _cbr(64, 64, (1, 7), padding=(0, 3)),
                                _cbr(64, 64, (7, 1), padding=(3, 0)), _cbr(64, 96, 3))),     # 192
        _Branches(_cbr(192, 192, 3, 2), nn.MaxPool2d(3, 2)),                                 # 384
        *[_v4_a() for _ in range(4)],
        _Branches(_cbr(384, 384, 3, 2),
                  nn.Sequential(_cbr(384, 192, 1), _cbr(192, 224, 3, padding=1), _cbr(224, 256, 3, 2)),
                  nn.MaxPool2d(3, 2)),                                                       # 1024
        *[_v4_b() for _ in range(7)],
        _Branches(nn.Sequential(_cbr(1024, 192, 1), _cbr(192, 192, 3, 2)),
                  nn.Sequential(_cbr(1024, 256, 1), _cbr(256, 256, (1, 7), padding=(0, 3)),
                                _cbr(256, 320, (7, 1), padding=(3, 0)), _cbr(320, 320, 3, 2)),
                  nn.MaxPool2d(3, 2)),                                                       # 1536
        *[_v4_c() for _ in range(3)])


@register('inceptionv4')
def inceptionv4(num_classes: int = 1000, in_channels: int = 3, **kw):
    return _Classifier(inceptionv4_features(in_channels), 1536, num_classes)


# ---------------------------------------------------------------------------- BN-Inception
def _bni(cin, c1, c3r, c3, d3r, d3, pool, proj, stride=1):
    """One BN-Inception module: [1x1] | 1x1 -> 3x3 | 1x1 -> 3x3 -> 3x3 | pool (-> 1x1).
    Stride-2 modules drop the 1x1 branch and pass the max-pooled input through."""
    cbr = lambda a, b, k, s=1: _cbr(a, b, k, s, k // 2, eps=1e-5, bias=True)  # noqa: E731
    br = [] if stride == 2 else [cbr(cin, c1, 1)]
    br.append(nn.Sequential(cbr(cin, c3r, 1), cbr(c3r, c3, 3, stride)))
    br.append(nn.Sequential(cbr(cin, d3r, 1), cbr(d3r, d3, 3), cbr(d3, d3, 3, stride)))
    if stride == 2:
        br.append(nn.MaxPool2d(3, 2, ceil_mode=True))
    else:
        p = nn.AvgPool2d(3, 1, 1, ceil_mode=True) if pool == 'avg' else nn.MaxPool2d(3, 1, 1, ceil_mode=True)
        br.append(nn.Sequential(p, cbr(cin, proj, 1)))
    return _Branches(*br)


def bninception_features(in_channels=3) -> nn.Sequential:
    cbr = lambda a, b, k, s=1: _cbr(a, b, k, s, k // 2, eps=1e-5, bias=True)  # noqa: E731
    return nn.Sequential(
        cbr(in_channels, 64, 7, 2), nn.MaxPool2d(3, 2, ceil_mode=True),
        cbr(64, 64, 1), cbr(64, 192, 3), nn.MaxPool2d(3, 2, ceil_mode=True),
        _bni(192, 64, 64, 64, 64, 96, 'avg', 32),          # 3a -> 256
        _bni(256, 64, 64, 96, 64, 96, 'avg', 64),          # 3b -> 320
        _bni(320, 0, 128, 160, 64, 96, None, 0, 2),        # 3c -> 576
        _bni(576, 224, 64, 96, 96, 128, 'avg', 128),       # 4a -> 576
        _bni(576, 192, 96, 128, 96, 128, 'avg', 128),      # 4b -> 576
        _bni(576, 160, 128, 160, 128, 160, 'avg', 128),    # 4c -> 608
        _bni(608, 96, 128, 192, 160, 192, 'avg', 128),     # 4d -> 608
        _bni(608, 0, 128, 192, 192, 256, None, 0, 2),      # 4e -> 1056
        _bni(1056, 352, 192, 320, 160, 224, 'avg', 128),   # 5a -> 1024
        _bni(1024, 352, 192, 320, 192, 224, 'max', 128))   # 5b -> 1024


@register('bninception')
def bninception(num_classes: int = 1000, in_channels: int = 3, **kw):
    return _Classifier(bninception_features(in_channels), 1024, num_classes)


# ---------------------------------------------------------------------------- fb / caffe ResNets
class _Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride, bias, stride_in_1x1):
        super().__init__()
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        out = planes * 4
        self.body = nn.Sequential(
            nn.Conv2d(cin, planes, 1, s1, bias=bias), nn.BatchNorm2d(planes), nn.ReLU(inplace=True),
            nn.Conv2d(planes, planes, 3, s3, 1, bias=bias), nn.BatchNorm2d(planes), nn.ReLU(inplace=True),
            nn.Conv2d(planes, out, 1, bias=bias), nn.BatchNorm2d(out))
        self.down = (nn.Sequential(nn.Conv2d(cin, out, 1, stride, bias=bias), nn.BatchNorm2d(out))
                     if stride != 1 or cin != out else None)

    def forward(self, x):
        return F.relu(self.body(x) + (self.down(x) if self.down is not None else x), inplace=True)


def variant_resnet_features(layers: Sequence[int], bias: bool, stride_in_1x1: bool, in_channels=3):
    mods = [nn.Conv2d(in_channels, 64, 7, 2, 3, bias=bias), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, 2, 1, ceil_mode=stride_in_1x1)]
    c = 64
    for i, n in enumerate(layers):
        planes = 64 * 2 ** i
        for j in range(n):
            mods.append(_Bottleneck(c, planes, 2 if (j == 0 and i > 0) else 1, bias, stride_in_1x1))
            c = planes * 4
    return nn.Sequential(*mods)


@register('fbresnet152')
def fbresnet152(num_classes: int = 1000, in_channels: int = 3, **kw):
    return _Classifier(variant_resnet_features((3, 8, 36, 3), True, False, in_channels), 2048, num_classes)


@register('cafferesnet101')
def cafferesnet101(num_classes: int = 1000, in_channels: int = 3, **kw):
    return _Classifier(variant_resnet_features((3, 4, 23, 3), False, True, in_channels), 2048, num_classes)


__all__ = ['xception', 'inceptionv3', 'inceptionv4', 'bninception', 'fbresnet152', 'cafferesnet101',
           'InceptionV3', 'xception_features', 'inceptionv4_features', 'bninception_features',
           'variant_resnet_features']
