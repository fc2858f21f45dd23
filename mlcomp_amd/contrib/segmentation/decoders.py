"""Decoders: U-Net, FPN, LinkNet, PSPNet (`mlcomp/contrib/segmentation/{unet,fpn,linknet,
pspnet}/decoder.py`).  All take the encoder's deepest-first feature list."""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .blocks import SCSE, ConvBnRelu, init_weights


# ---------------------------------------------------------------------------- U-Net
class UnetBlock(nn.Module):
    """x2 nearest upsample, concat skip, two 3x3 conv-BN-ReLU, optional scSE on both ends."""

    def __init__(self, cin, skip, cout, use_batchnorm=True, attention_type=None):
        super().__init__()
        att = attention_type == 'scse'
        self.att_in = SCSE(cin + skip) if att else nn.Identity()
        self.convs = nn.Sequential(ConvBnRelu(cin + skip, cout, 3, use_batchnorm=use_batchnorm),
                                   ConvBnRelu(cout, cout, 3, use_batchnorm=use_batchnorm))
        self.att_out = SCSE(cout) if att else nn.Identity()

    def forward(self, x, skip=None):
        x = F.interpolate(x, scale_factor=2, mode='nearest')
        if skip is not None:
            x = torch.cat([x, skip], 1)
        return self.att_out(self.convs(self.att_in(x)))


class UnetDecoder(nn.Module):
    def __init__(self, encoder_channels: Sequence[int], decoder_channels=(256, 128, 64, 32, 16), final_channels=1,
                 use_batchnorm=True, center=False, attention_type=None):
        super().__init__()
        head = encoder_channels[0]
        self.center = ConvBnRelu(head, head, 3, use_batchnorm=use_batchnorm) if center else nn.Identity()
        ins = [head] + list(decoder_channels[:-1])
        skips = list(encoder_channels[1:]) + [0]
        self.blocks = nn.ModuleList(UnetBlock(i, s, o, use_batchnorm, attention_type)
                                    for i, s, o in zip(ins, skips, decoder_channels))
        self.final_conv = nn.Conv2d(decoder_channels[-1], final_channels, 1)
        init_weights(self)

    def forward(self, feats):
        x = self.center(feats[0])
        skips = list(feats[1:]) + [None] * (len(self.blocks) - len(feats) + 1)
        for blk, skip in zip(self.blocks, skips):
            x = blk(x, skip)
        return self.final_conv(x)


# ---------------------------------------------------------------------------- FPN
class _GNUp(nn.Sequential):
    def __init__(self, cin, cout, upsample):
        super().__init__(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.GroupNorm(32, cout),
                         nn.ReLU(inplace=True))
        self.upsample = upsample

    def forward(self, x):
        x = super().forward(x)
        if self.upsample:
            x = F.interpolate(x, scale_factor=2, mode='bilinear', align_corners=True)
        return x


class FPNDecoder(nn.Module):
    def __init__(self, encoder_channels, pyramid_channels=256, segmentation_channels=128, final_channels=1,
                 dropout=0.2):
        super().__init__()
        self.lateral_top = nn.Conv2d(encoder_channels[0], pyramid_channels, 1)
        self.laterals = nn.ModuleList(nn.Conv2d(c, pyramid_channels, 1) for c in encoder_channels[1:4])
        # one segmentation head per pyramid level, upsampled to stride 4
        self.heads = nn.ModuleList()
        for n_up in (3, 2, 1, 0):
            layers = [_GNUp(pyramid_channels, segmentation_channels, n_up > 0)]
            layers += [_GNUp(segmentation_channels, segmentation_channels, True) for _ in range(1, n_up)]
            self.heads.append(nn.Sequential(*layers))
        self.dropout = nn.Dropout2d(p=dropout)
        self.final_conv = nn.Conv2d(segmentation_channels, final_channels, 1)
        init_weights(self)

    def forward(self, feats):
        p = self.lateral_top(feats[0])
        pyramid = [p]
        for lat, c in zip(self.laterals, feats[1:4]):
            p = F.interpolate(p, scale_factor=2, mode='nearest') + lat(c)
            pyramid.append(p)
        x = sum(h(p) for h, p in zip(self.heads, pyramid))
        x = self.final_conv(self.dropout(x))
        return F.interpolate(x, scale_factor=4, mode='bilinear', align_corners=True)


# ---------------------------------------------------------------------------- LinkNet
class _LinkBlock(nn.Module):
    """1x1 reduce to c/4 -> 4x4 stride-2 transposed conv -> 1x1 expand; + skip."""

    def __init__(self, cin, cout, use_batchnorm=True):
        super().__init__()
        q = max(1, cin // 4)
        up = [nn.ConvTranspose2d(q, q, 4, 2, 1)]
        if use_batchnorm:
            up.append(nn.BatchNorm2d(q))
        up.append(nn.ReLU(inplace=True))
        self.body = nn.Sequential(ConvBnRelu(cin, q, 1, use_batchnorm=use_batchnorm), *up,
                                  ConvBnRelu(q, cout, 1, use_batchnorm=use_batchnorm))

    def forward(self, x, skip=None):
        x = self.body(x)
        return x + skip if skip is not None else x


class LinknetDecoder(nn.Module):
    def __init__(self, encoder_channels, prefinal_channels=32, final_channels=1, use_batchnorm=True):
        super().__init__()
        chans = list(encoder_channels) + [prefinal_channels]
        self.blocks = nn.ModuleList(_LinkBlock(chans[i], chans[i + 1], use_batchnorm) for i in range(5))
        self.final_conv = nn.Conv2d(prefinal_channels, final_channels, 1)
        init_weights(self)

    def forward(self, feats):
        x = feats[0]
        skips = list(feats[1:5]) + [None]
        for blk, skip in zip(self.blocks, skips):
            x = blk(x, skip)
        return self.final_conv(x)


# ---------------------------------------------------------------------------- PSPNet
class PSPModule(nn.Module):
    def __init__(self, cin, sizes=(1, 2, 3, 6), use_batchnorm=True):
        super().__init__()
        out = cin // len(sizes)
        self.stages = nn.ModuleList(
            nn.Sequential(nn.AdaptiveAvgPool2d(s), ConvBnRelu(cin, out, 1, use_batchnorm=use_batchnorm and s > 1))
            for s in sizes)

    def forward(self, x):
        h, w = x.shape[-2:]
        ys = [F.interpolate(st(x), size=(h, w), mode='bilinear', align_corners=True) for st in self.stages]
        return torch.cat(ys + [x], 1)


class PSPDecoder(nn.Module):
    _LEVEL = {4: 3, 8: 2, 16: 1}

    def __init__(self, encoder_channels, downsample_factor=8, use_batchnorm=True, psp_out_channels=512,
                 final_channels=21, aux_output=False, dropout=0.2):
        super().__init__()
        if downsample_factor not in self._LEVEL:
            raise ValueError(f'Downsample factor should be in [4, 8, 16], got {downsample_factor}')
        self.factor = downsample_factor
        self.level = self._LEVEL[downsample_factor]
        c = encoder_channels[self.level]
        self.psp = PSPModule(c, use_batchnorm=use_batchnorm)
        self.conv = ConvBnRelu(4 * (c // 4) + c, psp_out_channels, 1, use_batchnorm=use_batchnorm)
        self.dropout = nn.Dropout2d(p=dropout) if dropout else nn.Identity()
        self.final_conv = nn.Conv2d(psp_out_channels, final_channels, 3, padding=1)
        self.aux = nn.Linear(c, final_channels) if aux_output else None
        init_weights(self)

    def forward(self, feats):
        f = feats[self.level]
        x = self.final_conv(self.dropout(self.conv(self.psp(f))))
        x = F.interpolate(x, scale_factor=self.factor, mode='bilinear', align_corners=True)
        if self.training and self.aux is not None:
            return [x, self.aux(F.adaptive_max_pool2d(f, 1).flatten(1))]
        return x


__all__ = ['UnetDecoder', 'FPNDecoder', 'LinknetDecoder', 'PSPDecoder', 'PSPModule']
