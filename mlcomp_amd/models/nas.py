"""Searched-cell ImageNet classifiers of the reference's per-model presets
(`mlcomp/contrib/catalyst/configs/classify/{nasnetamobile,nasnetalarge,pnasnet5large,
polynet}.yml`, resolved by ``Pretrained`` through pretrainedmodels,
`mlcomp/contrib/model/pretrained.py:8-58`), defined here from their papers:

* NASNet-A (Zoph et al. 2018): ``nasnetamobile`` (4 @ 1056, 5.29 M parameters) and
  ``nasnetalarge`` (6 @ 4032, 88.75 M; the paper quotes 88.9 M).  Two stem cells, three stages of one "first" cell
  (factorised reduction of the skip input) plus N-1 normal cells, reduction cells between.
* PNASNet-5 (Liu et al. 2018): ``pnasnet5large`` (86.1 M), one cell type whose five
  combinations mix separable convolutions and max pools.
* PolyNet (Zhang et al. 2017): ``polynet``, Inception-ResNet blocks composed as 2-way
  (I + F + G) and poly-3 (I + F + G F + H G F) units with linearly decaying residual
  scales.  Parity unpinned: with three distinct blocks per poly-3 unit this has 120.8 M
  parameters, while the pretrainedmodels build is quoted at 95.4 M; the paper does not
  fix the difference and no copy of that build is available here.

Stride-2 branches use symmetric padding k // 2, which gives every branch of a cell the
same output size for odd and even inputs (the TF "SAME" shapes) without pad-and-crop
tricks.  All models end in ``last_linear`` and train on the torch engine.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import register

_EPS = 1e-3


def _bn(c):
    return nn.BatchNorm2d(c, eps=_EPS, momentum=0.1)


class _Sep(nn.Sequential):
    """Depthwise k x k (stride) + pointwise 1x1, no bias."""

    def __init__(self, cin, cout, k, stride=1):
        super().__init__(nn.Conv2d(cin, cin, k, stride, k // 2, groups=cin, bias=False),
                         nn.Conv2d(cin, cout, 1, bias=False))


class _BranchSep(nn.Sequential):
    """ReLU -> sep(k, stride) -> BN -> ReLU -> sep(k) -> BN.  The first separable
    convolution keeps the input width unless ``widen_first`` (stem cells)."""

    def __init__(self, cin, cout, k, stride=1, widen_first=False):
        mid = cout if widen_first else cin
        super().__init__(nn.ReLU(), _Sep(cin, mid, k, stride), _bn(mid), nn.ReLU(), _Sep(mid, cout, k), _bn(cout))


class _ReluConvBn(nn.Sequential):
    def __init__(self, cin, cout, k=1, stride=1):
        super().__init__(nn.ReLU(), nn.Conv2d(cin, cout, k, stride, k // 2, bias=False), _bn(cout))


class _FactorizedReduce(nn.Module):
    """Halve the resolution of a skip input with two offset 1x1 stride-2 paths (each
    half the output width) and one BN - NASNet's path for mismatched cell inputs."""

    def __init__(self, cin, cout, relu=True):
        super().__init__()
        self.relu = relu
        self.p1 = nn.Conv2d(cin, cout // 2, 1, bias=False)
        self.p2 = nn.Conv2d(cin, cout - cout // 2, 1, bias=False)
        self.bn = _bn(cout)

    def forward(self, x):
        if self.relu:
            x = F.relu(x)
        a = self.p1(x[:, :, ::2, ::2])
        b = self.p2(F.pad(x, (0, 1, 0, 1))[:, :, 1::2, 1::2])
        return self.bn(torch.cat([a, b], 1))


def _maxpool(stride):
    return nn.MaxPool2d(3, stride, 1)


def _avgpool(stride):
    return nn.AvgPool2d(3, stride, 1, count_include_pad=False)


# ---------------------------------------------------------------------------- NASNet-A
class _NasStem0(nn.Module):
    def __init__(self, cstem, nf):
        super().__init__()
        self.conv_1x1 = _ReluConvBn(cstem, nf)
        self.c0l, self.c0r = _BranchSep(nf, nf, 5, 2), _BranchSep(cstem, nf, 7, 2, widen_first=True)
        self.c1l, self.c1r = _maxpool(2), _BranchSep(cstem, nf, 7, 2, widen_first=True)
        self.c2l, self.c2r = _avgpool(2), _BranchSep(cstem, nf, 5, 2, widen_first=True)
        self.c3r = _avgpool(1)
        self.c4l, self.c4r = _BranchSep(nf, nf, 3, 1), _maxpool(2)
        self.out_channels = 4 * nf

    def forward(self, x):
        x1 = self.conv_1x1(x)
        c0 = self.c0l(x1) + self.c0r(x)
        c1 = self.c1l(x1) + self.c1r(x)
        c2 = self.c2l(x1) + self.c2r(x)
        c3 = self.c3r(c0) + c1
        c4 = self.c4l(c0) + self.c4r(x1)
        return torch.cat([c1, c2, c3, c4], 1)


class _NasReduction(nn.Module):
    """Reduction cell (also the second stem cell, whose skip input is the stem conv at
    twice the resolution and goes through a factorised reduction)."""

    def __init__(self, cin_prev, cin, nf, prev_reduce=False):
        super().__init__()
        self.prev = (_FactorizedReduce(cin_prev, nf) if prev_reduce else _ReluConvBn(cin_prev, nf))
        self.conv_1x1 = _ReluConvBn(cin, nf)
        self.c0l, self.c0r = _BranchSep(nf, nf, 5, 2), _BranchSep(nf, nf, 7, 2)
        self.c1l, self.c1r = _maxpool(2), _BranchSep(nf, nf, 7, 2)
        self.c2l, self.c2r = _avgpool(2), _BranchSep(nf, nf, 5, 2)
        self.c3r = _avgpool(1)
        self.c4l, self.c4r = _BranchSep(nf, nf, 3, 1), _maxpool(2)
        self.out_channels = 4 * nf

    def forward(self, x, x_prev):
        xr = self.conv_1x1(x)        # right: this cell's main input
        xl = self.prev(x_prev)       # left: the skip input
        c0 = self.c0l(xr) + self.c0r(xl)
        c1 = self.c1l(xr) + self.c1r(xl)
        c2 = self.c2l(xr) + self.c2r(xl)
        c3 = self.c3r(c0) + c1
        c4 = self.c4l(c0) + self.c4r(xr)
        return torch.cat([c1, c2, c3, c4], 1)


class _NasNormal(nn.Module):
    """Normal cell; ``first`` (the cell after a reduction) brings the skip input down to
    the new resolution with a factorised reduction."""

    def __init__(self, cin_prev, cin, nf, first=False):
        super().__init__()
        self.prev = _FactorizedReduce(cin_prev, nf) if first else _ReluConvBn(cin_prev, nf)
        self.conv_1x1 = _ReluConvBn(cin, nf)
        self.c0l, self.c0r = _BranchSep(nf, nf, 5), _BranchSep(nf, nf, 3)
        self.c1l, self.c1r = _BranchSep(nf, nf, 5), _BranchSep(nf, nf, 3)
        self.c2l = _avgpool(1)
        self.c3l, self.c3r = _avgpool(1), _avgpool(1)
        self.c4l = _BranchSep(nf, nf, 3)
        self.out_channels = 6 * nf

    def forward(self, x, x_prev):
        xl = self.prev(x_prev)
        xr = self.conv_1x1(x)
        c0 = self.c0l(xr) + self.c0r(xl)
        c1 = self.c1l(xl) + self.c1r(xl)
        c2 = self.c2l(xr) + xl
        c3 = self.c3l(xl) + self.c3r(xl)
        c4 = self.c4l(xr) + xr
        return torch.cat([xl, c0, c1, c2, c3, c4], 1)


class NASNetA(nn.Module):
    def __init__(self, num_classes=1000, stem_filters=96, penultimate=4032, cells_per_stage=6, in_channels=3,
                 dropout=0.5):
        super().__init__()
        f = penultimate // 24
        self.conv0 = nn.Sequential(nn.Conv2d(in_channels, stem_filters, 3, 2, 0, bias=False), _bn(stem_filters))
        self.stem0 = _NasStem0(stem_filters, f // 4)
        self.stem1 = _NasReduction(stem_filters, self.stem0.out_channels, f // 2, prev_reduce=True)
        cells: List[nn.Module] = []
        prev, cur = self.stem0.out_channels, self.stem1.out_channels
        for stage in range(3):
            nf = f * 2 ** stage
            if stage:
                red = _NasReduction(prev, cur, nf)
                cells.append(red)
                prev, cur = cur, red.out_channels
            for i in range(cells_per_stage):
                c = _NasNormal(prev, cur, nf, first=(i == 0))
                cells.append(c)
                prev, cur = cur, c.out_channels
        self.cells = nn.ModuleList(cells)
        self.dropout = nn.Dropout(dropout)
        self.last_linear = nn.Linear(cur, num_classes)

    def features(self, x):
        x0 = self.conv0(x)
        s0 = self.stem0(x0)
        prev, cur = s0, self.stem1(s0, x0)
        for c in self.cells:
            if isinstance(c, _NasReduction):   # the cell after a reduction skips back past it
                cur = c(cur, prev)
            else:
                prev, cur = cur, c(cur, prev)
        return F.relu(cur)

    def forward(self, x):
        return self.last_linear(self.dropout(torch.flatten(F.adaptive_avg_pool2d(self.features(x), 1), 1)))


@register('nasnetamobile')
def nasnetamobile(num_classes: int = 1000, **kw):
    return NASNetA(num_classes, stem_filters=32, penultimate=1056, cells_per_stage=4, **kw)


@register('nasnetalarge')
def nasnetalarge(num_classes: int = 1000, **kw):
    return NASNetA(num_classes, stem_filters=96, penultimate=4032, cells_per_stage=6, **kw)


# ---------------------------------------------------------------------------- PNASNet-5
class _PnasCell(nn.Module):
    """PNASNet-5 cell over (left = the input two cells back, right = the last output):
    sep5|max3 (left), sep7|max3, sep5|sep3, sep3(comb 2)|max3, sep3 (left)|identity or
    1x1 stride-2 (right) - five combinations concatenated."""

    def __init__(self, cin_left, cin_right, nf, reduction=False, match_left=False, stem=False):
        super().__init__()
        s = 2 if reduction else 1
        self.stem = stem
        if stem:   # the first stem cell sees one input (the stem conv) on both sides
            self.conv_1x1 = _ReluConvBn(cin_right, nf)
            self.c0l = _BranchSep(cin_left, nf, 5, s, widen_first=True)
            self.c0r = nn.Sequential(_maxpool(s), nn.Conv2d(cin_left, nf, 1, bias=False), _bn(nf))
            self.c4l = _BranchSep(cin_left, nf, 3, s, widen_first=True)
        else:
            self.prev = _FactorizedReduce(cin_left, nf) if match_left else _ReluConvBn(cin_left, nf)
            self.conv_1x1 = _ReluConvBn(cin_right, nf)
            self.c0l, self.c0r = _BranchSep(nf, nf, 5, s), _maxpool(s)
            self.c4l = _BranchSep(nf, nf, 3, s)
        self.c1l, self.c1r = _BranchSep(nf, nf, 7, s), _maxpool(s)
        self.c2l, self.c2r = _BranchSep(nf, nf, 5, s), _BranchSep(nf, nf, 3, s)
        self.c3l, self.c3r = _BranchSep(nf, nf, 3), _maxpool(s)
        self.c4r = _ReluConvBn(nf, nf, 1, s) if reduction else None
        self.out_channels = 5 * nf

    def forward(self, x_left, x_right=None):
        if self.stem:
            xr = self.conv_1x1(x_left)
            xl = x_left
        else:
            xl = self.prev(x_left)
            xr = self.conv_1x1(x_right)
        c0 = self.c0l(xl) + self.c0r(xl)
        c1 = self.c1l(xr) + self.c1r(xr)
        c2 = self.c2l(xr) + self.c2r(xr)
        c3 = self.c3l(c2) + self.c3r(xr)
        c4 = self.c4l(xl) + (self.c4r(xr) if self.c4r is not None else xr)
        return torch.cat([c0, c1, c2, c3, c4], 1)


class PNASNet5Large(nn.Module):
    def __init__(self, num_classes=1000, in_channels=3, dropout=0.5):
        super().__init__()
        self.conv_0 = nn.Sequential(nn.Conv2d(in_channels, 96, 3, 2, 0, bias=False), _bn(96))
        self.cell_stem_0 = _PnasCell(96, 96, 54, reduction=True, stem=True)
        # (width, reduction) of the following cells; the left input is matched by a
        # factorised reduction whenever it is one resolution step behind the right one
        plan = [(108, True)] + [(216, False)] * 4 + [(432, True)] + [(432, False)] * 3 + [(864, True)] + \
            [(864, False)] * 3
        cells = []
        prev_c, cur_c = 96, self.cell_stem_0.out_channels
        prev_red, cur_red = False, True          # did the input two back / one back reduce
        for nf, red in plan:
            c = _PnasCell(prev_c, cur_c, nf, reduction=red, match_left=cur_red)
            cells.append(c)
            prev_c, cur_c = cur_c, c.out_channels
            prev_red, cur_red = cur_red, red
        self.cells = nn.ModuleList(cells)
        self.dropout = nn.Dropout(dropout)
        self.last_linear = nn.Linear(cur_c, num_classes)

    def features(self, x):
        x0 = self.conv_0(x)
        prev, cur = x0, self.cell_stem_0(x0)
        for c in self.cells:
            prev, cur = cur, c(prev, cur)
        return F.relu(cur)

    def forward(self, x):
        return self.last_linear(self.dropout(torch.flatten(F.adaptive_avg_pool2d(self.features(x), 1), 1)))


@register('pnasnet5large')
def pnasnet5large(num_classes: int = 1000, **kw):
    return PNASNet5Large(num_classes, **kw)


# ---------------------------------------------------------------------------- PolyNet
def _bc(cin, cout, k, stride=1, padding=0, relu=True):
    mods = [nn.Conv2d(cin, cout, k, stride, padding, bias=False), _bn(cout)]
    if relu:
        mods.append(nn.ReLU(inplace=True))
    return nn.Sequential(*mods)


class _Cat(nn.Module):
    def __init__(self, *paths):
        super().__init__()
        self.paths = nn.ModuleList(paths)

    def forward(self, x):
        return torch.cat([p(x) for p in self.paths], 1)


def _block_a():
    return nn.Sequential(_Cat(_bc(384, 32, 1),
                              nn.Sequential(_bc(384, 32, 1), _bc(32, 48, 3, padding=1), _bc(48, 64, 3, padding=1)),
                              nn.Sequential(_bc(384, 32, 1), _bc(32, 32, 3, padding=1))),
                         _bc(128, 384, 1, relu=False))


def _block_b():
    return nn.Sequential(_Cat(nn.Sequential(_bc(1152, 128, 1), _bc(128, 160, (1, 7), padding=(0, 3)),
                                            _bc(160, 192, (7, 1), padding=(3, 0))),
                              _bc(1152, 192, 1)),
                         _bc(384, 1152, 1, relu=False))


def _block_c():
    return nn.Sequential(_Cat(nn.Sequential(_bc(2048, 192, 1), _bc(192, 224, (1, 3), padding=(0, 1)),
                                            _bc(224, 256, (3, 1), padding=(1, 0))),
                              _bc(2048, 192, 1)),
                         _bc(448, 2048, 1, relu=False))


class _TwoWay(nn.Module):
    """relu(x + scale * (F(x) + G(x)))."""

    def __init__(self, make, scale):
        super().__init__()
        self.f, self.g = make(), make()
        self.scale = scale

    def forward(self, x):
        return F.relu(x + self.scale * (self.f(x) + self.g(x)))


class _Poly3(nn.Module):
    """relu(x + scale * (F x + G F x + H G F x)) with three distinct blocks (mpoly-3)."""

    def __init__(self, make, scale):
        super().__init__()
        self.blocks = nn.ModuleList(make() for _ in range(3))
        self.scale = scale

    def forward(self, x):
        out, y = x, x
        for b in self.blocks:
            y = b(y)
            out = out + self.scale * y
        return F.relu(out)


class PolyNet(nn.Module):
    """Stem (as Inception-v4), 10 x 2-way A, reduction A, 10 x (poly-3 B, 2-way B),
    reduction B, 5 x (poly-3 C, 2-way C); residual scales decay linearly over the 40 units
    from 1 to 0.7."""

    def __init__(self, num_classes=1000, in_channels=3, dropout=0.2, stage_b_pairs=10, stage_c_pairs=5):
        super().__init__()
        self.stem = nn.Sequential(
            _bc(in_channels, 32, 3, 2), _bc(32, 32, 3), _bc(32, 64, 3, padding=1),
            _Cat(nn.MaxPool2d(3, 2), _bc(64, 96, 3, 2)),
            _Cat(nn.Sequential(_bc(160, 64, 1), _bc(64, 96, 3)),
                 nn.Sequential(_bc(160, 64, 1), _bc(64, 64, (7, 1), padding=(3, 0)), _bc(64, 64, (1, 7), padding=(0, 3)),
                               _bc(64, 96, 3))),
            _Cat(_bc(192, 192, 3, 2), nn.MaxPool2d(3, 2)))
        n = 10 + 2 * stage_b_pairs + 2 * stage_c_pairs
        scales = iter([1.0 - 0.3 * i / (n - 1) for i in range(n)])
        self.stage_a = nn.Sequential(*[_TwoWay(_block_a, next(scales)) for _ in range(10)])
        self.reduction_a = _Cat(nn.Sequential(_bc(384, 256, 1), _bc(256, 256, 3, padding=1), _bc(256, 384, 3, 2)),
                                _bc(384, 384, 3, 2), nn.MaxPool2d(3, 2))
        self.stage_b = nn.Sequential(*[m for _ in range(stage_b_pairs)
                                       for m in (_Poly3(_block_b, next(scales)), _TwoWay(_block_b, next(scales)))])
        self.reduction_b = _Cat(nn.Sequential(_bc(1152, 256, 1), _bc(256, 256, 3, padding=1), _bc(256, 256, 3, 2)),
                                nn.Sequential(_bc(1152, 256, 1), _bc(256, 256, 3, 2)),
                                nn.Sequential(_bc(1152, 256, 1), _bc(256, 384, 3, 2)),
                                nn.MaxPool2d(3, 2))
        self.stage_c = nn.Sequential(*[m for _ in range(stage_c_pairs)
                                       for m in (_Poly3(_block_c, next(scales)), _TwoWay(_block_c, next(scales)))])
        self.dropout = nn.Dropout(dropout)
        self.last_linear = nn.Linear(2048, num_classes)

    def features(self, x):
        x = self.stage_a(self.stem(x))
        x = self.stage_b(self.reduction_a(x))
        return self.stage_c(self.reduction_b(x))

    def forward(self, x):
        return self.last_linear(self.dropout(torch.flatten(F.adaptive_avg_pool2d(self.features(x), 1), 1)))


@register('polynet')
def polynet(num_classes: int = 1000, **kw):
    return PolyNet(num_classes, **kw)


__all__ = ['NASNetA', 'PNASNet5Large', 'PolyNet', 'nasnetamobile', 'nasnetalarge', 'pnasnet5large', 'polynet']
