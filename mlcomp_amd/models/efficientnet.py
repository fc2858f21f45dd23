"""EfficientNet B0-B7 (Tan & Le 2019) - classification model and feature encoder.

The reference wraps the external ``efficientnet_pytorch`` package
(`mlcomp/contrib/model/efficientnet.py:8-49`); it is not part of this stack, so the
architecture is implemented here: MBConv blocks (expand 1x1 -> depthwise kxk ->
squeeze-excitation -> project 1x1, stochastic depth on the residual), compound
width/depth scaling from the (width, depth, resolution, dropout) table.
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register

# (expand, kernel, stride, in, out, repeats) for B0
_B0 = [(1, 3, 1, 32, 16, 1), (6, 3, 2, 16, 24, 2), (6, 5, 2, 24, 40, 2), (6, 3, 2, 40, 80, 3),
       (6, 5, 1, 80, 112, 3), (6, 5, 2, 112, 192, 4), (6, 3, 1, 192, 320, 1)]
# width, depth, resolution, dropout
PARAMS = {'b0': (1.0, 1.0, 224, 0.2), 'b1': (1.0, 1.1, 240, 0.2), 'b2': (1.1, 1.2, 260, 0.3),
          'b3': (1.2, 1.4, 300, 0.3), 'b4': (1.4, 1.8, 380, 0.4), 'b5': (1.6, 2.2, 456, 0.4),
          'b6': (1.8, 2.6, 528, 0.5), 'b7': (2.0, 3.1, 600, 0.5)}


def _round_filters(c, width, divisor=8):
    c *= width
    new = max(divisor, int(c + divisor / 2) // divisor * divisor)
    if new < 0.9 * c:
        new += divisor
    return int(new)


def _round_repeats(r, depth):
    return int(math.ceil(depth * r))


class _ConvBnAct(nn.Sequential):
    def __init__(self, cin, cout, k, stride=1, groups=1, act=True):
        layers = [nn.Conv2d(cin, cout, k, stride, k // 2, groups=groups, bias=False),
                  nn.BatchNorm2d(cout, eps=1e-3, momentum=0.01)]
        if act:
            layers.append(nn.SiLU(inplace=True))
        super().__init__(*layers)


class MBConv(nn.Module):
    def __init__(self, cin, cout, expand, k, stride, se_ratio=0.25, drop_path=0.0):
        super().__init__()
        mid = cin * expand
        self.expand = _ConvBnAct(cin, mid, 1) if expand != 1 else nn.Identity()
        self.dw = _ConvBnAct(mid, mid, k, stride, groups=mid)
        sq = max(1, int(cin * se_ratio))
        self.se = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(mid, sq, 1), nn.SiLU(inplace=True),
                                nn.Conv2d(sq, mid, 1), nn.Sigmoid())
        self.project = _ConvBnAct(mid, cout, 1, act=False)
        self.residual = stride == 1 and cin == cout
        self.drop_path = drop_path

    def forward(self, x):
        y = self.dw(self.expand(x))
        y = y * self.se(y)
        y = self.project(y)
        if self.residual:
            if self.training and self.drop_path > 0:
                keep = 1 - self.drop_path
                # one draw per sample (rand_like of a [N, 1, 1, 1] slice: fx-traceable)
                mask = torch.rand_like(y[:, :1, :1, :1]) < keep
                y = y * mask / keep
            y = y + x
        return y


class EfficientNet(nn.Module):
    def __init__(self, variant: str = 'b0', num_classes: int = 1000, in_channels: int = 3,
                 drop_connect: float = 0.2, include_top: bool = True):
        super().__init__()
        width, depth, self.resolution, dropout = PARAMS[variant.replace('efficientnet-', '')]
        stem = _round_filters(32, width)
        self.stem = _ConvBnAct(in_channels, stem, 3, 2)
        blocks: List[nn.Module] = []
        self.stage_ends: List[int] = []   # block index ending each stride level (for encoders)
        total = sum(_round_repeats(r, depth) for *_, r in _B0)
        i = 0
        cin = stem
        for expand, k, stride, _, cout, reps in _B0:
            cout = _round_filters(cout, width)
            for j in range(_round_repeats(reps, depth)):
                blocks.append(MBConv(cin, cout, expand, k, stride if j == 0 else 1,
                                     drop_path=drop_connect * i / total))
                cin = cout
                i += 1
        self.blocks = nn.ModuleList(blocks)
        head = _round_filters(1280, width)
        self.head = _ConvBnAct(cin, head, 1)
        self.out_channels = head
        self.include_top = include_top
        if include_top:
            self.dropout = nn.Dropout(dropout)
            self.fc = nn.Linear(head, num_classes)

    def forward_features(self, x) -> List[torch.Tensor]:
        """Features at strides 2, 4, 8, 16, 32, deepest first."""
        feats = []
        x = self.stem(x)
        cur = x
        for b in self.blocks:
            if isinstance(b.dw[0], nn.Conv2d) and b.dw[0].stride[0] == 2:
                feats.append(cur)
            cur = b(cur)
        feats.append(self.head(cur))
        return feats[::-1][:5]

    def forward(self, x):
        x = self.stem(x)
        for b in self.blocks:
            x = b(x)
        x = self.head(x)
        if not self.include_top:
            return x
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(self.dropout(x))


for _v in PARAMS:
    register(f'efficientnet-{_v}')((lambda v: (lambda **kw: EfficientNet(v, **kw)))(_v))


@register('EfficientNet')
def efficientnet(variant: str = 'efficientnet-b0', num_classes: int = 1000, **kw):
    return EfficientNet(variant, num_classes=num_classes, **kw)


__all__ = ['EfficientNet', 'MBConv', 'PARAMS']
