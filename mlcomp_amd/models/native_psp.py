"""Native execution of the PSPNet segmentation model
(:class:`mlcomp_amd.contrib.segmentation.models.PSPNet`; the reference's
`mlcomp/contrib/segmentation/pspnet/{model,decoder}.py`) with a ResNet encoder and a
sigmoid head of <= 4 classes trained with BCE + Dice (the segmentation engine's loss).

* encoder: the native ResNet body shared with the U-Net engine.
* pyramid pooling: adaptive average pools (1, 2, 3, 6) of the stride-``factor`` feature;
  each pooled map goes through a native 1x1 conv (+BN+ReLU: :class:`ConvBN`; the 1x1 level
  has no BN, a bias-epilogue GEMM + ReLU) and back to the feature size by the native
  bilinear kernels (align_corners=True); concat with the feature.
* fusion conv (1x1 + BN + ReLU, :class:`ConvBN`), Dropout2d, the 3x3 output conv with bias
  on the implicit-GEMM kernels, x ``factor`` bilinear, BCE + Dice
  (:class:`~.native_fpn.UpsampledSegHead`).
The pyramid's adaptive pools run on the native NHWC kernels (pool_loss.hip: PyTorch's bins,
fp32 sums); concat, dropout and the loss are PyTorch tensor ops on NHWC activations; every
convolution runs on the native MFMA kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import ConvBN
from .native_fpn import Conv1x1Bias, Conv3x3, NativeFPN, UpsampledSegHead, _BilinearFn, _nchw, _nhwc
from .native_unet import NativeUnet


class NativePSPNet(NativeUnet):
    """Same encoder / step interface as :class:`NativeUnet`; PSP decoder."""

    def __init__(self, model, device, bce_w=1.0, dice_w=1.0, eps=1e-7):
        from mlcomp_amd.contrib.segmentation.decoders import PSPDecoder
        dec = model.decoder
        if not isinstance(dec, PSPDecoder):
            raise NotImplementedError('NativePSPNet: a PSPDecoder model')
        if dec.aux is not None:
            raise NotImplementedError('native PSPNet: psp_aux_output not supported')
        if dec.final_conv.out_channels > 4:
            raise NotImplementedError('native PSPNet: <= 4 sigmoid classes (BCE + Dice)')
        ctx = self._lower_encoder(model)
        self.level, self.factor = dec.level, dec.factor
        # encoder blocks past the decoder's level are never run (see features()): their
        # slots are frozen, so the optimizer neither updates nor weight-decays them - what
        # torch.optim does with parameters whose grad stays None
        last = self.ends[3 - self.level]
        for blk in self.blocks[last + 1:]:
            for u in list(blk.units) + ([blk.down] if blk.down is not None else []):
                u.w.frozen = u.gamma.frozen = u.beta.frozen = True
        self.stages = []
        for i, st in enumerate(dec.psp.stages):
            pool, cbr = st[0], st[1]
            pre = f'decoder.psp.stages.{i}.1'
            if isinstance(cbr[1], nn.BatchNorm2d):
                unit = ConvBN(ctx, pre, cbr[0], cbr[1], act=True)
            else:
                unit = Conv1x1Bias(ctx, f'{pre}.0', cbr[0])
            self.stages.append((pool.output_size, unit))
        cv = dec.conv
        if not isinstance(cv[1], nn.BatchNorm2d):
            raise NotImplementedError('native PSPNet: psp_use_batchnorm=True required')
        self.fuse = ConvBN(ctx, 'decoder.conv', cv[0], cv[1], act=True)
        self.drop = dec.dropout.p if isinstance(dec.dropout, nn.Dropout2d) else 0.0
        self.head = UpsampledSegHead(ctx, Conv3x3(ctx, 'decoder.final_conv', dec.final_conv),
                                     dec.final_conv.out_channels, self.factor, bce_w, dice_w, eps)
        self._finish_init(device)

    def _units(self):
        """BN-carrying units (encoder, pyramid-level and fusion ConvBNs) - the set whose
        running statistics the step flattens and broadcasts."""
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down
        for _, u in self.stages:
            if isinstance(u, ConvBN):
                yield u
        yield self.fuse

    def _all_units(self):
        yield from self._units()
        for _, u in self.stages:
            if not isinstance(u, ConvBN):
                yield u
        yield self.head.conv

    def _finish_init(self, device):
        self.ctx.finalize(device)
        self._default_schedule()
        for u in self._all_units():
            u.load_from_torch()
        self.ctx.arena.decay.refresh_mirror()

    def features(self, x):
        """x: NHWC bf16 image -> the fused stride-``factor`` features [N, h, w, 512] bf16."""
        anchor = self.ctx.anchor
        x0 = self.stem(x)
        y = self.pool(x0, anchor)
        # the decoder reads one stage (deepest-first index ``level``): the deeper stages would
        # only feed nothing, so they are not run (their parameters get zero gradients, as in
        # the reference, where they do not reach the loss)
        want = 3 - self.level
        feats = []
        for i, blk in enumerate(self.blocks):
            y = blk(y)
            if i in self.ends:
                feats.append(y)
                if len(feats) > want:
                    break
        f = feats[want]
        h, w = f.shape[1], f.shape[2]
        ys = []
        for size, unit in self.stages:
            so = (size, size) if isinstance(size, int) else tuple(size)
            if f.shape[-1] % 8 == 0:
                p = Fn.AdaptiveAvgFn.apply(f.contiguous(), so[0], so[1])     # native bins, fp32 sums
            else:
                p = _nhwc(F.adaptive_avg_pool2d(_nchw(f), so))
            q = unit(p) if isinstance(unit, ConvBN) else torch.relu(unit(p))
            ys.append(_BilinearFn.apply(q.contiguous(), (h, w)))
        z = self.fuse(torch.cat(ys + [f], dim=-1))
        self.ctx.refresh_wt()    # transposed filters for the ConvBN dgrads
        if self.ctx.training and self.drop > 0:
            z = _nhwc(F.dropout2d(_nchw(z), self.drop, True))
        return z

    def loss(self, x, target):
        return self.head.loss(self.head.logits(self.features(x)), target)

    predict = NativeFPN.predict     # inference forward + loss through the upsampled head

    def export_to_torch(self):
        for u in self._all_units():
            u.export_to_torch()
        return self.torch_model
