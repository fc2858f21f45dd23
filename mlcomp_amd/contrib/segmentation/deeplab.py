"""DeepLab v3+ (Chen et al. 2018) with ResNet-101 / aligned Xception / MobileNetV2 / DRN-D-54
backbones (`mlcomp/contrib/segmentation/deeplabv3/*`).

backbone(x) -> (high-level features at ``output_stride``, low-level features at stride 4);
ASPP (1x1 + three atrous 3x3 at rates 6/12/18 for OS 16, doubled for OS 8, + image
pooling) -> 1x1 projection -> decoder (48-channel low-level projection, two 3x3 convs)
-> classifier -> bilinear upsampling to the input size.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.models import register


def _cbr(cin, cout, k=3, stride=1, dilation=1, groups=1):
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, (k // 2) * dilation, dilation, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


# ---------------------------------------------------------------------------- backbones
class ResNetBackbone(nn.Module):
    """ResNet-101 with the last stages dilated instead of strided (OS 16 or 8)."""
    low_channels, high_channels = 256, 2048

    def __init__(self, output_stride=16, variant='resnet101'):
        super().__init__()
        from mlcomp_amd.models.resnet import resnet
        dil = {16: (False, False, True), 8: (False, True, True)}[output_stride]
        self.body = resnet(variant, include_top=False, replace_stride_with_dilation=dil)

    def forward(self, x):
        b = self.body
        x = b.maxpool(b.stem(x))
        low = b.layer1(x)
        x = b.layer4(b.layer3(b.layer2(low)))
        return x, low


class _SepConv(nn.Sequential):
    """depthwise 3x3 (dilated) -> BN -> pointwise 1x1 -> BN (-> ReLU)."""

    def __init__(self, cin, cout, stride=1, dilation=1, relu_first=True):
        layers = [nn.ReLU(inplace=False)] if relu_first else []
        layers += [nn.Conv2d(cin, cin, 3, stride, dilation, dilation, groups=cin, bias=False), nn.BatchNorm2d(cin),
                   nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        super().__init__(*layers)


class _XBlock(nn.Module):
    def __init__(self, cin, cout, reps, stride=1, dilation=1, skip_conv=True):
        super().__init__()
        convs = []
        c = cin
        for i in range(reps):
            s = stride if i == reps - 1 else 1
            convs.append(_SepConv(c, cout, s, dilation))
            c = cout
        self.convs = nn.Sequential(*convs)
        self.skip = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
                     if skip_conv and (cin != cout or stride != 1) else None)

    def forward(self, x):
        y = self.convs(x)
        return y + (self.skip(x) if self.skip is not None else x)


class XceptionBackbone(nn.Module):
    """Aligned Xception (entry / 16 middle / exit flows), strides replaced by dilation
    beyond ``output_stride``."""
    low_channels, high_channels = 128, 2048

    def __init__(self, output_stride=16, middle_blocks=16):
        super().__init__()
        if output_stride == 16:
            s3, mid_dil, exit_dil = 2, 1, (1, 2)
        else:
            s3, mid_dil, exit_dil = 1, 2, (2, 4)
        self.stem = nn.Sequential(_cbr(3, 32, 3, 2), _cbr(32, 64, 3, 1))
        self.block1 = _XBlock(64, 128, 3, 2)
        self.block2 = _XBlock(128, 256, 3, 2)
        self.block3 = _XBlock(256, 728, 3, s3)
        self.middle = nn.Sequential(*[_XBlock(728, 728, 3, 1, mid_dil) for _ in range(middle_blocks)])
        self.exit = _XBlock(728, 1024, 3, 1, exit_dil[0])
        self.tail = nn.Sequential(_SepConv(1024, 1536, 1, exit_dil[1]), nn.ReLU(inplace=True),
                                  _SepConv(1536, 1536, 1, exit_dil[1], relu_first=False), nn.ReLU(inplace=True),
                                  _SepConv(1536, 2048, 1, exit_dil[1], relu_first=False), nn.ReLU(inplace=True))

    def forward(self, x):
        x = self.block1(self.stem(x))
        low = x
        x = self.block3(self.block2(x))
        x = self.tail(self.exit(self.middle(x)))
        return x, low


class MobileNetBackbone(nn.Module):
    low_channels, high_channels = 24, 320

    def __init__(self, output_stride=16):
        super().__init__()
        from .encoders import MobileNetV2Encoder
        enc = MobileNetV2Encoder(output_stride=output_stride)
        self.stem, self.blocks = enc.stem, enc.blocks
        self.low_idx = 3   # input of the first stride-8 block = stride-4 features (24 channels)

    def forward(self, x):
        x = self.stem(x)
        low = None
        for i, b in enumerate(self.blocks):
            if i == self.low_idx:
                low = x
            x = b(x)
        return x, low


class _DRNBlock(nn.Module):
    def __init__(self, cin, cout, stride=1, dilation=1, residual=True):
        super().__init__()
        self.body = nn.Sequential(
            nn.Conv2d(cin, cout // 4, 1, bias=False), nn.BatchNorm2d(cout // 4), nn.ReLU(inplace=True),
            nn.Conv2d(cout // 4, cout // 4, 3, stride, dilation, dilation, bias=False), nn.BatchNorm2d(cout // 4),
            nn.ReLU(inplace=True), nn.Conv2d(cout // 4, cout, 1, bias=False), nn.BatchNorm2d(cout))
        self.down = (nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))
                     if (cin != cout or stride != 1) else None)
        self.residual = residual

    def forward(self, x):
        y = self.body(x)
        if self.residual:
            y = y + (self.down(x) if self.down is not None else x)
        return F.relu(y)


class DRNBackbone(nn.Module):
    """DRN-D-54 (Yu et al. 2017): dilated residual network, output stride 8, with the
    de-gridding tail (dilation 2 and 1 layers without residuals)."""
    low_channels, high_channels = 256, 512

    def __init__(self, output_stride=8):
        super().__init__()
        self.layer0 = nn.Sequential(_cbr(3, 16, 7), _cbr(16, 16, 3))
        self.layer1 = _cbr(16, 16, 3)
        self.layer2 = _cbr(16, 32, 3, 2)
        layers = [(64, 3, 2, 1), (128, 4, 2, 1), (256, 6, 1, 2), (512, 3, 1, 4)]
        c = 32
        stages = []
        for cout_base, n, stride, dil in layers:
            cout = cout_base * 4
            blocks = [_DRNBlock(c, cout, stride, dil)]
            blocks += [_DRNBlock(cout, cout, 1, dil) for _ in range(1, n)]
            stages.append(nn.Sequential(*blocks))
            c = cout
        self.layer3, self.layer4, self.layer5, self.layer6 = stages
        self.layer7 = _cbr(c, 512, 3, 1, 2)
        self.layer8 = _cbr(512, 512, 3, 1, 1)

    def forward(self, x):
        x = self.layer2(self.layer1(self.layer0(x)))
        x = self.layer3(x)
        low = x
        x = self.layer6(self.layer5(self.layer4(x)))
        return self.layer8(self.layer7(x)), low


BACKBONES = {'resnet': ResNetBackbone, 'xception': XceptionBackbone, 'mobilenet': MobileNetBackbone,
             'drn': DRNBackbone}


# ---------------------------------------------------------------------------- head
class ASPP(nn.Module):
    def __init__(self, cin, output_stride=16, cout=256):
        super().__init__()
        rates = (6, 12, 18) if output_stride == 16 else (12, 24, 36)
        self.branches = nn.ModuleList([_cbr(cin, cout, 1)] + [_cbr(cin, cout, 3, 1, r) for r in rates])
        self.pool = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout),
                                  nn.ReLU(inplace=True))
        self.project = nn.Sequential(_cbr(5 * cout, cout, 1), nn.Dropout(0.5))

    def forward(self, x):
        ys = [b(x) for b in self.branches]
        ys.append(F.interpolate(self.pool(x), size=x.shape[-2:], mode='bilinear', align_corners=True))
        return self.project(torch.cat(ys, 1))


class Decoder(nn.Module):
    def __init__(self, low_channels, num_classes, cin=256):
        super().__init__()
        self.low = _cbr(low_channels, 48, 1)
        self.body = nn.Sequential(_cbr(cin + 48, 256, 3), nn.Dropout(0.5), _cbr(256, 256, 3), nn.Dropout(0.1),
                                  nn.Conv2d(256, num_classes, 1))

    def forward(self, x, low):
        low = self.low(low)
        x = F.interpolate(x, size=low.shape[-2:], mode='bilinear', align_corners=True)
        return self.body(torch.cat([x, low], 1))


@register('DeepLab')
class DeepLab(nn.Module):
    def __init__(self, backbone='resnet', output_stride=16, num_classes=21, freeze_bn=False):
        super().__init__()
        if backbone == 'drn':
            output_stride = 8
        if backbone not in BACKBONES:
            raise NotImplementedError(backbone)
        self.backbone = BACKBONES[backbone](output_stride)
        self.aspp = ASPP(self.backbone.high_channels, output_stride)
        self.decoder = Decoder(self.backbone.low_channels, num_classes)
        self._freeze = freeze_bn
        if freeze_bn:
            self.freeze_bn()

    def forward(self, inp):
        x, low = self.backbone(inp)
        x = self.decoder(self.aspp(x), low)
        return F.interpolate(x, size=inp.shape[-2:], mode='bilinear', align_corners=True)

    def train(self, mode=True):
        super().train(mode)
        if self._freeze:
            self.freeze_bn()
        return self

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def get_1x_lr_params(self):
        return (p for p in self.backbone.parameters() if p.requires_grad)

    def get_10x_lr_params(self):
        for mod in (self.aspp, self.decoder):
            for p in mod.parameters():
                if p.requires_grad:
                    yield p


__all__ = ['DeepLab', 'ASPP', 'Decoder', 'BACKBONES']
