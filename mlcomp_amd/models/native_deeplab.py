"""Native execution of DeepLab v3+ with the dilated-ResNet backbone
(:class:`mlcomp_amd.contrib.segmentation.deeplab.DeepLab`, ``backbone='resnet'``; the
reference's `mlcomp/contrib/segmentation/deeplab/`), sigmoid heads of <= 4 classes trained
with BCE + Dice (the segmentation engine's loss).

* backbone: the ResNet body with its last stage(s) dilated instead of strided, lowered like
  the classifier (:func:`~.native_resnet.lower_resnet_body`: the dilated 3x3 convs are the
  implicit-GEMM kernels with ``dil``); layer-1's output is the decoder's low-level feature.
* ASPP: the 1x1 and the three atrous 3x3 branches and the image-pool branch (global average
  -> 1x1 conv + BN + ReLU -> broadcast by the native bilinear kernel) are native ConvBN
  units; the projection 1x1 + BN + ReLU too; Dropout(0.5).
* decoder: low-level 1x1 (256 -> 48) + BN + ReLU, the ASPP output bilinearly resized to the
  low-level grid (native kernel), concat, two 3x3 conv + BN + ReLU (Dropout 0.5 / 0.1), the
  1x1 output conv with bias (a bias-epilogue GEMM) and the x4 bilinear resize of the logits
  to the input size in the loss head (:class:`~.native_fpn.UpsampledSegHead`).
Pooling, concat, dropout and the loss are PyTorch tensor ops on NHWC activations; every
convolution runs on the native MFMA kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.ops.layers import ConvBN, NativeContext
from .native_fpn import Conv1x1Bias, NativeFPN, UpsampledSegHead, _BilinearFn, _nchw, _nhwc
from .native_resnet import lower_resnet_body
from .native_unet import NativeUnet


def _cbr(ctx, name, seq):
    conv, bn = seq[0], seq[1]
    assert isinstance(bn, nn.BatchNorm2d)
    return ConvBN(ctx, name, conv, bn, act=True)


class NativeDeepLab(NativeUnet):
    """Same step interface as :class:`NativeUnet` (loss / predict / export / arena)."""

    def __init__(self, model, device, bce_w=1.0, dice_w=1.0, eps=1e-7):
        from mlcomp_amd.contrib.segmentation.deeplab import DeepLab, ResNetBackbone
        if not isinstance(model, DeepLab) or not isinstance(model.backbone, ResNetBackbone):
            raise NotImplementedError('native DeepLab: the ResNet backbone (use engine=torch for others)')
        if model._freeze:
            raise NotImplementedError('native DeepLab: freeze_bn=True (eval-mode BatchNorm) not supported')
        K = model.decoder.body[4].out_channels
        if K > 4:
            raise NotImplementedError('native DeepLab: <= 4 sigmoid classes (BCE + Dice)')
        self.torch_model = model
        ctx = self.ctx = NativeContext()
        ctx.default_dgrad_first(True)
        self.stem, self.pool, self.blocks, self.ends = lower_resnet_body(ctx, model.backbone.body,
                                                                          prefix='backbone.body.', s2d_stem=True)
        self.blocks[self.ends[0] + 1].prev = None      # layer-1's output also feeds the decoder
        a, d = model.aspp, model.decoder
        self.branches = [_cbr(ctx, f'aspp.branches.{i}', b) for i, b in enumerate(a.branches)]
        self.img_pool = ConvBN(ctx, 'aspp.pool', a.pool[1], a.pool[2], act=True)
        self.project = _cbr(ctx, 'aspp.project.0', a.project[0])
        self.p_drop = a.project[1].p
        self.low = _cbr(ctx, 'decoder.low', d.low)
        self.body1 = _cbr(ctx, 'decoder.body.0', d.body[0])
        self.body2 = _cbr(ctx, 'decoder.body.2', d.body[2])
        self.drops = (d.body[1].p, d.body[3].p)
        self.head = UpsampledSegHead(ctx, Conv1x1Bias(ctx, 'decoder.body.4', d.body[4], f32_out=True), K, 4,
                                     bce_w, dice_w, eps)
        self._finish_init(device)

    def _units(self):
        """BN-carrying units (their running statistics are flattened / broadcast)."""
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down
        yield from self.branches
        yield self.img_pool
        yield self.project
        yield self.low
        yield self.body1
        yield self.body2

    def _default_schedule(self):
        """The ResNet-101 backbone's long per-layer GEMMs keep the per-conv join (as
        ResNet-50 does): the unjoined chain measured 1,868 / 1,874 vs 1,989 / 1,985 img/s
        (profiles/round5/seg_wgrad_join_ab.txt); their split-K weight gradients add with
        atomics (1,971 / 1,976 -> 2,005 / 1,998, profiles/round5/wgrad_slab_ab.txt)."""
        self.ctx.default_wgrad_slab(False)

    def _finish_init(self, device):
        self.ctx.finalize(device)
        self._default_schedule()
        for u in self._units():
            u.load_from_torch()
        self.head.conv.load_from_torch()
        self.ctx.arena.decay.refresh_mirror()

    def _drop(self, x, p):
        return F.dropout(x, p, True) if self.ctx.training and p > 0 else x

    def features(self, x):
        """x: NHWC bf16 image -> decoder features [N, H/4, W/4, 256] bf16."""
        anchor = self.ctx.anchor
        y = self.pool(self.stem(x), anchor)
        low = None
        for i, blk in enumerate(self.blocks):
            y = blk(y)
            if i == self.ends[0]:
                low = y
        h, w = y.shape[1], y.shape[2]
        ys = [b(y) for b in self.branches]
        g = _nhwc(F.adaptive_avg_pool2d(_nchw(y), 1))
        ys.append(_BilinearFn.apply(self.img_pool(g).contiguous(), (h, w)))
        z = self._drop(self.project(torch.cat(ys, dim=-1)), self.p_drop)
        lo = self.low(low)
        z = _BilinearFn.apply(z.contiguous(), (lo.shape[1], lo.shape[2]))
        z = self._drop(self.body1(torch.cat([z, lo], dim=-1)), self.drops[0])
        z = self._drop(self.body2(z), self.drops[1])
        self.ctx.refresh_wt()    # transposed filters for the backward's dgrads
        return z

    def loss(self, x, target):
        return self.head.loss(self.head.logits(self.features(x)), target)

    predict = NativeFPN.predict

    def export_to_torch(self):
        for u in self._units():
            u.export_to_torch()
        self.head.conv.export_to_torch()
        return self.torch_model
