"""3D ResNe(X)t video classifiers (`mlcomp/contrib/model/video/resnext3d/*`):
post-activated 3D ResNe(X)t (Feichtenhofer et al. 2018), pre-activated 3D ResNe(X)t
(Ghadiyaram et al. 2019) and R(2+1)D factorised units (Tran et al. 2018).

Same constructor surface as the reference's ``ResNeXt3D`` (stem / skip / residual
transformation names, per-stage temporal kernel bases, strides, groups); single-pathway.
Input is ``[B, C, T, H, W]``; the head flattens the last stage, adaptively average-pools
the flat vector to ``in_plane`` values and applies a linear layer, like the reference.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.nn as nn

from mlcomp_amd.models import register


def _bn(c):
    return nn.BatchNorm3d(c, eps=1e-5, momentum=0.1)


def _r2p1_mid(cin, cout, t, s):
    # parameter-matched intermediate width (Tran et al. eq. 1)
    return max(1, int((t * s * s * cin * cout) / (s * s * cin + t * cout)))


def _conv(cin, cout, t, s, stride_t=1, stride_s=1, groups=1, r2p1=False):
    """t x s x s conv; factorised into (1,s,s) spatial + (t,1,1) temporal when ``r2p1``."""
    if not r2p1 or t == 1:
        return nn.Conv3d(cin, cout, (t, s, s), (stride_t, stride_s, stride_s), (t // 2, s // 2, s // 2),
                         groups=groups, bias=False)
    mid = _r2p1_mid(cin, cout, t, s)
    return nn.Sequential(
        nn.Conv3d(cin, mid, (1, s, s), (1, stride_s, stride_s), (0, s // 2, s // 2), bias=False), _bn(mid),
        nn.ReLU(inplace=True),
        nn.Conv3d(mid, cout, (t, 1, 1), (stride_t, 1, 1), (t // 2, 0, 0), bias=False))


# ---------------------------------------------------------------------------- stems
class ResNeXt3DStem(nn.Sequential):
    def __init__(self, temporal_kernel, spatial_kernel, input_planes, stem_planes, maxpool):
        layers = [nn.Conv3d(input_planes, stem_planes, (temporal_kernel, spatial_kernel, spatial_kernel),
                            (1, 2, 2), (temporal_kernel // 2, spatial_kernel // 2, spatial_kernel // 2), bias=False),
                  _bn(stem_planes), nn.ReLU(inplace=True)]
        if maxpool:
            layers.append(nn.MaxPool3d((1, 3, 3), (1, 2, 2), (0, 1, 1)))
        super().__init__(*layers)


class R2Plus1DStem(nn.Sequential):
    def __init__(self, temporal_kernel, spatial_kernel, input_planes, stem_planes, maxpool):
        mid = 45 if stem_planes == 64 else _r2p1_mid(input_planes, stem_planes, temporal_kernel, spatial_kernel)
        layers = [nn.Conv3d(input_planes, mid, (1, spatial_kernel, spatial_kernel), (1, 2, 2),
                            (0, spatial_kernel // 2, spatial_kernel // 2), bias=False), _bn(mid), nn.ReLU(inplace=True),
                  nn.Conv3d(mid, stem_planes, (temporal_kernel, 1, 1), 1, (temporal_kernel // 2, 0, 0), bias=False),
                  _bn(stem_planes), nn.ReLU(inplace=True)]
        if maxpool:
            layers.append(nn.MaxPool3d((1, 3, 3), (1, 2, 2), (0, 1, 1)))
        super().__init__(*layers)


STEMS = {'resnext3d_stem': ResNeXt3DStem, 'r2plus1d_stem': R2Plus1DStem}


# ---------------------------------------------------------------------------- residual transforms
class BasicTransformation(nn.Module):
    final_op = None

    def __init__(self, cin, cout, inner, t, temporal_conv_1x1, stride_t, stride_s, groups, preact, r2p1=False):
        super().__init__()
        self.preact = preact
        self.pre = nn.Sequential(_bn(cin), nn.ReLU(inplace=True)) if preact else nn.Identity()
        self.a = _conv(cin, cout, t, 3, stride_t, stride_s, r2p1=r2p1)
        self.a_post = nn.Sequential(_bn(cout), nn.ReLU(inplace=True))
        self.b = _conv(cout, cout, t, 3, r2p1=r2p1)
        self.b_bn = nn.Identity() if preact else _bn(cout)
        self.final_op = self.b if preact else self.b_bn

    def forward(self, x):
        return self.b_bn(self.b(self.a_post(self.a(self.pre(x)))))


class BasicR2Plus1DTransformation(BasicTransformation):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw, r2p1=True)


class BottleneckTransformation(nn.Module):
    def __init__(self, cin, cout, inner, t, temporal_conv_1x1, stride_t, stride_s, groups, preact):
        super().__init__()
        ta, tb = (t, 1) if temporal_conv_1x1 else (1, t)
        self.pre = nn.Sequential(_bn(cin), nn.ReLU(inplace=True)) if preact else nn.Identity()
        self.a = nn.Conv3d(cin, inner, (ta, 1, 1), (stride_t if temporal_conv_1x1 else 1, 1, 1), (ta // 2, 0, 0),
                           bias=False)
        self.b = nn.Conv3d(inner, inner, (tb, 3, 3), (1 if temporal_conv_1x1 else stride_t, stride_s, stride_s),
                           (tb // 2, 1, 1), groups=groups, bias=False)
        self.c = nn.Conv3d(inner, cout, 1, bias=False)
        self.mid = nn.ModuleList([nn.Sequential(_bn(inner), nn.ReLU(inplace=True)) for _ in range(2)])
        self.c_bn = nn.Identity() if preact else _bn(cout)
        self.final_op = self.c if preact else self.c_bn

    def forward(self, x):
        x = self.mid[0](self.a(self.pre(x)))
        x = self.mid[1](self.b(x))
        return self.c_bn(self.c(x))


class PostactivatedBottleneckTransformation(BottleneckTransformation):
    def __init__(self, *a, preact=False):
        super().__init__(*a, preact=False)


class PreactivatedBottleneckTransformation(BottleneckTransformation):
    pass


RESIDUAL = {'basic_transformation': BasicTransformation,
            'basic_r2plus1d_transformation': BasicR2Plus1DTransformation,
            'postactivated_bottleneck_transformation': PostactivatedBottleneckTransformation,
            'preactivated_bottleneck_transformation': PreactivatedBottleneckTransformation}
SKIP = ('postactivated_shortcut', 'preactivated_shortcut')


class ResBlock(nn.Module):
    def __init__(self, cin, cout, inner, t, t1x1, stride_t, stride_s, groups, skip_type, residual_type,
                 disable_pre_activation=False):
        super().__init__()
        self.preact = skip_type == 'preactivated_shortcut'
        res_preact = self.preact and not disable_pre_activation
        self.residual = RESIDUAL[residual_type](cin, cout, inner, t, t1x1, stride_t, stride_s, groups,
                                                preact=res_preact)
        self.skip = None
        if cin != cout or stride_t != 1 or stride_s != 1:
            pre = [_bn(cin), nn.ReLU(inplace=True)] if res_preact else []
            post = [] if self.preact else [_bn(cout)]
            self.skip = nn.Sequential(*pre, nn.Conv3d(cin, cout, 1, (stride_t, stride_s, stride_s), bias=False),
                                      *post)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        s = x if self.skip is None else self.skip(x)
        y = self.residual(x) + s
        return y if self.preact else self.relu(y)


class ResNeXt3D(nn.Module):
    def __init__(self, input_planes: int = 3, skip_transformation_type: str = 'postactivated_shortcut',
                 residual_transformation_type: str = 'basic_transformation', num_blocks: Sequence[int] = (2, 2, 2, 2),
                 stem_name: str = 'resnext3d_stem', stem_planes: int = 64, stem_temporal_kernel: int = 3,
                 stem_spatial_kernel: int = 7, stem_maxpool: bool = False, stage_planes: int = 64,
                 stage_temporal_kernel_basis: Sequence[List[int]] = ([3], [3], [3], [3]),
                 temporal_conv_1x1: Sequence[bool] = (False, False, False, False),
                 stage_temporal_stride: Sequence[int] = (1, 2, 2, 2), stage_spatial_stride: Sequence[int] = (1, 2, 2, 2),
                 num_groups: int = 1, width_per_group: int = 64, zero_init_residual_transform: bool = False,
                 in_plane: int = 512, num_classes: int = 2):
        super().__init__()
        if skip_transformation_type not in SKIP:
            raise ValueError(skip_transformation_type)
        n = len(num_blocks)
        outs = [stage_planes * 2 ** i for i in range(n)]
        ins = [stem_planes] + outs[:-1]
        inners = [num_groups * width_per_group * 2 ** i for i in range(n)]
        self.stem = STEMS[stem_name](stem_temporal_kernel, stem_spatial_kernel, input_planes, stem_planes, stem_maxpool)
        stages = []
        for s in range(n):
            blocks = []
            basis = stage_temporal_kernel_basis[s]
            for b in range(num_blocks[s]):
                blocks.append(ResBlock(ins[s] if b == 0 else outs[s], outs[s], inners[s], basis[b % len(basis)],
                                       temporal_conv_1x1[s], stage_temporal_stride[s] if b == 0 else 1,
                                       stage_spatial_stride[s] if b == 0 else 1, num_groups,
                                       skip_transformation_type, residual_transformation_type,
                                       disable_pre_activation=(s == 0 and b == 0)))
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.Sequential(*stages)
        self.final = (nn.Sequential(_bn(outs[-1]), nn.ReLU(inplace=True))
                      if skip_transformation_type == 'preactivated_shortcut' else nn.Identity())
        self.final_avgpool = nn.AdaptiveAvgPool1d(in_plane)
        self.head_fcl = nn.Linear(in_plane, num_classes)
        self._init(zero_init_residual_transform)

    def _init(self, zero_last):
        finals = {id(m.final_op) for m in self.modules() if hasattr(m, 'final_op') and m.final_op is not None}
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                if zero_last and id(m) in finals:
                    nn.init.zeros_(m.weight)
                else:
                    nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 0.0 if (zero_last and id(m) in finals) else 1.0)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, 0.01)
                nn.init.zeros_(m.bias)

    def forward(self, x):
        x = self.final(self.stages(self.stem(x)))
        x = self.final_avgpool(x.reshape(x.shape[0], 1, -1))
        return self.head_fcl(x.reshape(x.shape[0], -1))


register('ResNeXt3D')(ResNeXt3D)

__all__ = ['ResNeXt3D', 'ResBlock', 'STEMS', 'RESIDUAL', 'SKIP']
