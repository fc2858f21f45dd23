"""Feature encoders for the segmentation models
(`mlcomp/contrib/segmentation/encoders/*`: resnet/resnext, vgg, densenet, senet, dpn,
inceptionresnetv2; plus mobilenet_v2 and efficientnet here).

Every encoder returns its five feature maps at strides 32, 16, 8, 4, 2, deepest first,
and exposes ``out_shapes`` (their channel counts, measured once with a tiny dry run so
the table can never drift from the architecture).  There is no network access, so
``encoder_weights`` is ``None`` (random init) or a path to a local state dict
(``weights_only=True``); ``'imagenet'`` falls back to random init with a warning.
"""
from __future__ import annotations

import math
import warnings
from collections import OrderedDict
from typing import Callable, Dict, List

import torch
import torch.nn as nn
import torch.nn.functional as F

ENCODERS: Dict[str, Callable[[], nn.Module]] = OrderedDict()
PREPROCESSING = {'mean': (0.485, 0.456, 0.406), 'std': (0.229, 0.224, 0.225), 'input_range': (0, 1),
                 'input_space': 'RGB'}


def register_encoder(name):
    def deco(fn):
        ENCODERS[name] = fn
        return fn
    return deco


# ---------------------------------------------------------------------------- resnet family
class ResNetEncoder(nn.Module):
    def __init__(self, variant: str):
        super().__init__()
        from mlcomp_amd.models.resnet import resnet
        self.body = resnet(variant, include_top=False)

    def forward(self, x):
        return self.body.forward_features(x)


def _resnet_names():
    from mlcomp_amd.models.resnet import _SPECS
    return list(_SPECS)


for _n in ['resnet18', 'resnet34', 'resnet50', 'resnet101', 'resnet152', 'resnext50_32x4d',
           'resnext101_32x4d', 'resnext101_32x8d', 'resnext101_64x4d', 'wide_resnet50_2', 'wide_resnet101_2']:
    register_encoder(_n)((lambda v: (lambda: ResNetEncoder(v)))(_n))


# ---------------------------------------------------------------------------- vgg
_VGG = {'vgg11': [64, 'M', 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
        'vgg13': [64, 64, 'M', 128, 128, 'M', 256, 256, 'M', 512, 512, 'M', 512, 512, 'M'],
        'vgg16': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512, 'M'],
        'vgg19': [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 256, 'M', 512, 512, 512, 512, 'M',
                  512, 512, 512, 512, 'M']}


class VGGEncoder(nn.Module):
    """Five conv stages, each closed by a 2x2 max-pool; the pooled output of every
    stage is a feature (strides 2..32)."""

    def __init__(self, cfg, batch_norm=False, in_channels=3):
        super().__init__()
        stages, cur, c = [], [], in_channels
        for v in cfg:
            if v == 'M':
                cur.append(nn.MaxPool2d(2, 2))
                stages.append(nn.Sequential(*cur))
                cur = []
                continue
            cur.append(nn.Conv2d(c, v, 3, padding=1))
            if batch_norm:
                cur.append(nn.BatchNorm2d(v))
            cur.append(nn.ReLU(inplace=True))
            c = v
        self.stages = nn.ModuleList(stages)

    def forward(self, x):
        feats = []
        for s in self.stages:
            x = s(x)
            feats.append(x)
        return feats[::-1]


for _n, _c in _VGG.items():
    register_encoder(_n)((lambda c: (lambda: VGGEncoder(c)))(_c))
    register_encoder(_n + '_bn')((lambda c: (lambda: VGGEncoder(c, batch_norm=True)))(_c))


# ---------------------------------------------------------------------------- densenet
class _DenseLayer(nn.Module):
    def __init__(self, cin, growth, bn_size):
        super().__init__()
        self.body = nn.Sequential(nn.BatchNorm2d(cin), nn.ReLU(inplace=True),
                                  nn.Conv2d(cin, bn_size * growth, 1, bias=False),
                                  nn.BatchNorm2d(bn_size * growth), nn.ReLU(inplace=True),
                                  nn.Conv2d(bn_size * growth, growth, 3, padding=1, bias=False))

    def forward(self, x):
        return torch.cat([x, self.body(x)], 1)


class DenseNetEncoder(nn.Module):
    def __init__(self, growth=32, blocks=(6, 12, 24, 16), init=64, bn_size=4, in_channels=3):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(in_channels, init, 7, 2, 3, bias=False), nn.BatchNorm2d(init),
                                  nn.ReLU(inplace=True))
        self.pool = nn.MaxPool2d(3, 2, 1)
        c = init
        self.blocks = nn.ModuleList()
        self.transitions = nn.ModuleList()
        for i, n in enumerate(blocks):
            layers = []
            for _ in range(n):
                layers.append(_DenseLayer(c, growth, bn_size))
                c += growth
            self.blocks.append(nn.Sequential(*layers))
            if i != len(blocks) - 1:
                self.transitions.append(nn.Sequential(nn.BatchNorm2d(c), nn.ReLU(inplace=True),
                                                      nn.Conv2d(c, c // 2, 1, bias=False), nn.AvgPool2d(2, 2)))
                c //= 2
        self.final = nn.Sequential(nn.BatchNorm2d(c), nn.ReLU(inplace=True))

    def forward(self, x):
        x0 = self.stem(x)
        x = self.pool(x0)
        feats = [x0]
        for i, b in enumerate(self.blocks):
            x = b(x)
            if i < len(self.transitions):
                feats.append(x)
                x = self.transitions[i](x)
        feats.append(self.final(x))
        return feats[::-1]


for _n, _a in {'densenet121': (32, (6, 12, 24, 16), 64), 'densenet169': (32, (6, 12, 32, 32), 64),
               'densenet201': (32, (6, 12, 48, 32), 64), 'densenet161': (48, (6, 12, 36, 24), 96)}.items():
    register_encoder(_n)((lambda a: (lambda: DenseNetEncoder(a[0], a[1], a[2])))(_a))


# ---------------------------------------------------------------------------- senet
class _SE(nn.Module):
    def __init__(self, c, reduction=16):
        super().__init__()
        self.fc = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(c, c // reduction, 1), nn.ReLU(inplace=True),
                                nn.Conv2d(c // reduction, c, 1), nn.Sigmoid())

    def forward(self, x):
        return x * self.fc(x)


class _SEBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, groups, base_width, stride, downsample, reduction=16, senet154=False):
        super().__init__()
        if senet154:
            width, mid = planes * 2, planes * 4
        elif groups > 1:
            width = int(math.floor(planes * base_width / 64) * groups)
            mid = width
        else:
            width = mid = planes
        self.body = nn.Sequential(
            nn.Conv2d(cin, width, 1, bias=False), nn.BatchNorm2d(width), nn.ReLU(inplace=True),
            nn.Conv2d(width, mid, 3, stride, 1, groups=groups, bias=False), nn.BatchNorm2d(mid), nn.ReLU(inplace=True),
            nn.Conv2d(mid, planes * 4, 1, bias=False), nn.BatchNorm2d(planes * 4))
        self.se = _SE(planes * 4, reduction)
        self.downsample = downsample
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        r = x if self.downsample is None else self.downsample(x)
        return self.relu(self.se(self.body(x)) + r)


class SENetEncoder(nn.Module):
    """SE-ResNet / SE-ResNeXt / SENet-154 (Hu et al. 2018)."""

    def __init__(self, layers, groups=1, base_width=64, senet154=False, in_channels=3):
        super().__init__()
        if senet154:
            self.stem = nn.Sequential(
                nn.Conv2d(in_channels, 64, 3, 2, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                nn.Conv2d(64, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                nn.Conv2d(64, 128, 3, 1, 1, bias=False), nn.BatchNorm2d(128), nn.ReLU(inplace=True))
            c = 128
        else:
            self.stem = nn.Sequential(nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64),
                                      nn.ReLU(inplace=True))
            c = 64
        self.pool = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.stages = nn.ModuleList()
        for i, (planes, n) in enumerate(zip((64, 128, 256, 512), layers)):
            stride = 1 if i == 0 else 2
            ds = None
            if stride != 1 or c != planes * 4:
                k = 3 if (senet154 and i > 0) else 1
                ds = nn.Sequential(nn.Conv2d(c, planes * 4, k, stride, k // 2, bias=False), nn.BatchNorm2d(planes * 4))
            blocks = [_SEBottleneck(c, planes, groups, base_width, stride, ds, senet154=senet154)]
            c = planes * 4
            blocks += [_SEBottleneck(c, planes, groups, base_width, 1, None, senet154=senet154) for _ in range(1, n)]
            self.stages.append(nn.Sequential(*blocks))

    def forward(self, x):
        x0 = self.stem(x)
        x = self.pool(x0)
        feats = [x0]
        for s in self.stages:
            x = s(x)
            feats.append(x)
        return feats[::-1]


for _n, _a in {'se_resnet50': ((3, 4, 6, 3), 1, 64, False), 'se_resnet101': ((3, 4, 23, 3), 1, 64, False),
               'se_resnet152': ((3, 8, 36, 3), 1, 64, False), 'se_resnext50_32x4d': ((3, 4, 6, 3), 32, 4, False),
               'se_resnext101_32x4d': ((3, 4, 23, 3), 32, 4, False),
               'senet154': ((3, 8, 36, 3), 64, 4, True)}.items():
    register_encoder(_n)((lambda a: (lambda: SENetEncoder(*a)))(_a))


# ---------------------------------------------------------------------------- dpn
class _DualPathBlock(nn.Module):
    """Dual path block (Chen et al. 2017): a ResNeXt-style residual path of width
    ``inc_res`` summed into the first channels, plus a densely concatenated path growing
    by ``inc_dense`` channels."""

    def __init__(self, cin, r1, r2, inc_res, inc_dense, groups, kind):
        super().__init__()
        self.inc_res, self.kind = inc_res, kind
        stride = 2 if kind == 'down' else 1
        if kind in ('proj', 'down'):
            self.proj = nn.Sequential(nn.BatchNorm2d(cin), nn.ReLU(inplace=True),
                                      nn.Conv2d(cin, inc_res + 2 * inc_dense, 1, stride, bias=False))
        self.body = nn.Sequential(
            nn.BatchNorm2d(cin), nn.ReLU(inplace=True), nn.Conv2d(cin, r1, 1, bias=False),
            nn.BatchNorm2d(r1), nn.ReLU(inplace=True), nn.Conv2d(r1, r2, 3, stride, 1, groups=groups, bias=False),
            nn.BatchNorm2d(r2), nn.ReLU(inplace=True), nn.Conv2d(r2, inc_res + inc_dense, 1, bias=False))

    def forward(self, x):
        x = torch.cat(x, 1) if isinstance(x, tuple) else x
        if self.kind in ('proj', 'down'):
            p = self.proj(x)
            res, dense = p[:, :self.inc_res], p[:, self.inc_res:]
        else:
            res, dense = None, None
        y = self.body(x)
        yr, yd = y[:, :self.inc_res], y[:, self.inc_res:]
        if res is None:
            # x is the concatenation [res | dense] carried from the previous block
            res, dense = x[:, :self.inc_res], x[:, self.inc_res:]
        return torch.cat([res + yr, dense, yd], 1)


class DPNEncoder(nn.Module):
    def __init__(self, small, init, k_r, groups, k_sec, inc_sec, in_channels=3):
        super().__init__()
        k = 3 if small else 7
        self.stem = nn.Sequential(nn.Conv2d(in_channels, init, k, 2, k // 2, bias=False), nn.BatchNorm2d(init),
                                  nn.ReLU(inplace=True))
        self.pool = nn.MaxPool2d(3, 2, 1)
        bw_factor = 1 if small else 4
        self.stages = nn.ModuleList()
        c = init
        for i, (n, inc) in enumerate(zip(k_sec, inc_sec)):
            bw = (64 * 2 ** i) * bw_factor
            r = (k_r * bw) // (64 * bw_factor)
            blocks = [_DualPathBlock(c, r, r, bw, inc, groups, 'proj' if i == 0 else 'down')]
            c = bw + 3 * inc
            for _ in range(1, n):
                blocks.append(_DualPathBlock(c, r, r, bw, inc, groups, 'normal'))
                c += inc
            self.stages.append(nn.Sequential(*blocks))
        self.final = nn.Sequential(nn.BatchNorm2d(c), nn.ReLU(inplace=True))

    def forward(self, x):
        x0 = self.stem(x)
        x = self.pool(x0)
        feats = [x0]
        for i, s in enumerate(self.stages):
            x = s(x)
            feats.append(self.final(x) if i == len(self.stages) - 1 else x)
        return feats[::-1]


for _n, _a in {'dpn68': (True, 10, 128, 32, (3, 4, 12, 3), (16, 32, 32, 64)),
               'dpn92': (False, 64, 96, 32, (3, 4, 20, 3), (16, 32, 24, 128)),
               'dpn98': (False, 96, 160, 40, (3, 6, 20, 3), (16, 32, 32, 128)),
               'dpn107': (False, 128, 200, 50, (4, 8, 20, 3), (20, 64, 64, 128)),
               'dpn131': (False, 128, 160, 40, (4, 8, 28, 3), (16, 32, 32, 128))}.items():
    register_encoder(_n)((lambda a: (lambda: DPNEncoder(*a)))(_a))
# dpn68b (pretrainedmodels' ``b=True``) splits the last 1x1 convolution of every block
# into its residual and dense outputs: the same function and parameter count as dpn68
register_encoder('dpn68b')(lambda: DPNEncoder(True, 10, 128, 32, (3, 4, 12, 3), (16, 32, 32, 64)))


# ---------------------------------------------------------------------------- mobilenet v2
class _InvRes(nn.Module):
    def __init__(self, cin, cout, stride, expand, dilation=1):
        super().__init__()
        mid = cin * expand
        layers = []
        if expand != 1:
            layers += [nn.Conv2d(cin, mid, 1, bias=False), nn.BatchNorm2d(mid), nn.ReLU6(inplace=True)]
        layers += [nn.Conv2d(mid, mid, 3, stride, dilation, dilation=dilation, groups=mid, bias=False),
                   nn.BatchNorm2d(mid), nn.ReLU6(inplace=True),
                   nn.Conv2d(mid, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        self.body = nn.Sequential(*layers)
        self.res = stride == 1 and cin == cout

    def forward(self, x):
        y = self.body(x)
        return x + y if self.res else y


_MBV2 = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]


class MobileNetV2Encoder(nn.Module):
    def __init__(self, width=1.0, in_channels=3, output_stride=32):
        super().__init__()
        c = int(32 * width)
        self.stem = nn.Sequential(nn.Conv2d(in_channels, c, 3, 2, 1, bias=False), nn.BatchNorm2d(c),
                                  nn.ReLU6(inplace=True))
        blocks, stride_now, dil = [], 2, 1
        self.taps = []
        for t, ch, n, s in _MBV2:
            cout = int(ch * width)
            for i in range(n):
                st = s if i == 0 else 1
                if st == 2 and stride_now >= output_stride:
                    dil, st = dil * 2, 1
                elif st == 2:
                    self.taps.append(len(blocks))
                    stride_now *= 2
                blocks.append(_InvRes(c, cout, st, t, dilation=dil))
                c = cout
        self.blocks = nn.ModuleList(blocks)
        self.head = nn.Sequential(nn.Conv2d(c, 1280, 1, bias=False), nn.BatchNorm2d(1280), nn.ReLU6(inplace=True))

    def forward(self, x):
        x = self.stem(x)
        feats = []
        for i, b in enumerate(self.blocks):
            if i in self.taps:
                feats.append(x)
            x = b(x)
        feats.append(self.head(x))
        return feats[::-1]


register_encoder('mobilenet_v2')(lambda: MobileNetV2Encoder())


# ---------------------------------------------------------------------------- efficientnet
class EfficientNetEncoder(nn.Module):
    def __init__(self, variant):
        super().__init__()
        from mlcomp_amd.models.efficientnet import EfficientNet
        self.body = EfficientNet(variant, include_top=False, drop_connect=0.0)

    def forward(self, x):
        return self.body.forward_features(x)


for _v in ('b0', 'b1', 'b2', 'b3', 'b4', 'b5', 'b6', 'b7'):
    register_encoder(f'efficientnet-{_v}')((lambda v: (lambda: EfficientNetEncoder(v)))(_v))


# ---------------------------------------------------------------------------- inception-resnet-v2
def _bcr(cin, cout, k, stride=1, padding=0):
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, padding, bias=False), nn.BatchNorm2d(cout, eps=1e-3),
                         nn.ReLU(inplace=True))


class _Block35(nn.Module):
    def __init__(self, scale=0.17):
        super().__init__()
        self.scale = scale
        self.b0 = _bcr(320, 32, 1)
        self.b1 = nn.Sequential(_bcr(320, 32, 1), _bcr(32, 32, 3, padding=1))
        self.b2 = nn.Sequential(_bcr(320, 32, 1), _bcr(32, 48, 3, padding=1), _bcr(48, 64, 3, padding=1))
        self.conv = nn.Conv2d(128, 320, 1)

    def forward(self, x):
        y = self.conv(torch.cat([self.b0(x), self.b1(x), self.b2(x)], 1))
        return F.relu(x + self.scale * y)


class _Block17(nn.Module):
    def __init__(self, scale=0.10):
        super().__init__()
        self.scale = scale
        self.b0 = _bcr(1088, 192, 1)
        self.b1 = nn.Sequential(_bcr(1088, 128, 1), _bcr(128, 160, (1, 7), padding=(0, 3)),
                                _bcr(160, 192, (7, 1), padding=(3, 0)))
        self.conv = nn.Conv2d(384, 1088, 1)

    def forward(self, x):
        return F.relu(x + self.scale * self.conv(torch.cat([self.b0(x), self.b1(x)], 1)))


class _Block8(nn.Module):
    def __init__(self, scale=0.20, relu=True):
        super().__init__()
        self.scale, self.relu = scale, relu
        self.b0 = _bcr(2080, 192, 1)
        self.b1 = nn.Sequential(_bcr(2080, 192, 1), _bcr(192, 224, (1, 3), padding=(0, 1)),
                                _bcr(224, 256, (3, 1), padding=(1, 0)))
        self.conv = nn.Conv2d(448, 2080, 1)

    def forward(self, x):
        y = x + self.scale * self.conv(torch.cat([self.b0(x), self.b1(x)], 1))
        return F.relu(y) if self.relu else y


class InceptionResNetV2Encoder(nn.Module):
    """Inception-ResNet-v2 (Szegedy et al. 2016) with 'same' padding on the strided
    layers so the five features sit exactly at strides 2..32."""

    def __init__(self, in_channels=3):
        super().__init__()
        self.s2 = nn.Sequential(_bcr(in_channels, 32, 3, 2, 1), _bcr(32, 32, 3, padding=1), _bcr(32, 64, 3, padding=1))
        self.s4 = nn.Sequential(nn.MaxPool2d(3, 2, 1), _bcr(64, 80, 1), _bcr(80, 192, 3, padding=1))
        self.pool8 = nn.MaxPool2d(3, 2, 1)
        self.m5b = nn.ModuleList([_bcr(192, 96, 1),
                                  nn.Sequential(_bcr(192, 48, 1), _bcr(48, 64, 5, padding=2)),
                                  nn.Sequential(_bcr(192, 64, 1), _bcr(64, 96, 3, padding=1), _bcr(96, 96, 3, padding=1)),
                                  nn.Sequential(nn.AvgPool2d(3, 1, 1, count_include_pad=False), _bcr(192, 64, 1))])
        self.r35 = nn.Sequential(*[_Block35() for _ in range(10)])
        self.m6a = nn.ModuleList([_bcr(320, 384, 3, 2, 1),
                                  nn.Sequential(_bcr(320, 256, 1), _bcr(256, 256, 3, padding=1), _bcr(256, 384, 3, 2, 1)),
                                  nn.MaxPool2d(3, 2, 1)])
        self.r17 = nn.Sequential(*[_Block17() for _ in range(20)])
        self.m7a = nn.ModuleList([nn.Sequential(_bcr(1088, 256, 1), _bcr(256, 384, 3, 2, 1)),
                                  nn.Sequential(_bcr(1088, 256, 1), _bcr(256, 288, 3, 2, 1)),
                                  nn.Sequential(_bcr(1088, 256, 1), _bcr(256, 288, 3, padding=1), _bcr(288, 320, 3, 2, 1)),
                                  nn.MaxPool2d(3, 2, 1)])
        self.r8 = nn.Sequential(*[_Block8() for _ in range(9)], _Block8(relu=False))
        self.head = _bcr(2080, 1536, 1)

    def forward(self, x):
        x2 = self.s2(x)
        x4 = self.s4(x2)
        x8 = self.r35(torch.cat([b(self.pool8(x4)) for b in self.m5b], 1))
        x16 = self.r17(torch.cat([b(x8) for b in self.m6a], 1))
        x32 = self.head(self.r8(torch.cat([b(x16) for b in self.m7a], 1)))
        return [x32, x16, x8, x4, x2]


register_encoder('inceptionresnetv2')(lambda: InceptionResNetV2Encoder())


# ---------------------------------------------------------------------------- api
def _measure_out_shapes(enc: nn.Module) -> tuple:
    was = enc.training
    enc.eval()
    with torch.no_grad():
        feats = enc(torch.zeros(1, 3, 64, 64))
    enc.train(was)
    return tuple(int(f.shape[1]) for f in feats)


def get_encoder(name: str, encoder_weights=None) -> nn.Module:
    if name not in ENCODERS:
        raise KeyError(f'unknown encoder {name}; available: {list(ENCODERS)}')
    enc = ENCODERS[name]()
    enc.out_shapes = _measure_out_shapes(enc)
    if encoder_weights == 'imagenet':
        warnings.warn(f'{name}: no network access for ImageNet weights; random init '
                      f'(pass a local state-dict path as encoder_weights)')
    elif isinstance(encoder_weights, str):
        sd = torch.load(encoder_weights, map_location='cpu', weights_only=True)
        enc.load_state_dict(sd.get('state_dict', sd), strict=False)
    return enc


def get_encoder_names() -> List[str]:
    return list(ENCODERS)


def get_preprocessing_params(encoder_name: str = None, pretrained='imagenet') -> dict:
    return dict(PREPROCESSING)


def preprocess_input(x, mean=None, std=None, input_space='RGB', input_range=None, **kw):
    import numpy as np
    if input_space == 'BGR':
        x = x[..., ::-1].copy()
    if input_range is not None and x.max() > 1 and input_range[1] == 1:
        x = x / 255.0
    if mean is not None:
        x = x - np.array(mean)
    if std is not None:
        x = x / np.array(std)
    return x


__all__ = ['ENCODERS', 'get_encoder', 'get_encoder_names', 'get_preprocessing_params', 'preprocess_input',
           'register_encoder']
