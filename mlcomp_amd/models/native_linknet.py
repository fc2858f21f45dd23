"""Native (HIP-kernel) execution of the LinkNet segmentation model
(:class:`mlcomp_amd.contrib.segmentation.models.Linknet`; the reference's
`mlcomp/contrib/segmentation/linknet/{model,decoder}.py`) with a ResNet encoder.

* encoder: lowered exactly as for the U-Net (:func:`~.native_unet.lower_seg_encoder`), whose
  stage outputs and stem output feed the decoder's skip additions.
* decoder block (``_LinkBlock``): 1x1 conv+BN+ReLU to c/4 channels, 4x4 / stride-2
  transposed conv + BN + ReLU (:class:`~mlcomp_amd.ops.layers.ConvTBN`: the dgrad's
  parity-class GEMMs with the BN statistics in their epilogue), 1x1 conv+BN+ReLU to the
  next width, then + skip.  One autograd node per block: the last unit's dgrad epilogue
  masks and reduces the transposed conv's BN (``Fn.BnBwdSpec`` with the recomputed ReLU
  mask), the transposed conv's input gradient is a plain forward conv over its filter.
* head: the 1x1 output conv (32 -> K <= 4 classes) fused with BCE-with-logits + soft Dice
  (:class:`~.native_unet.SegHead`).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import ConvBN, ConvTBN
from .native_unet import NativeUnet, SegHead


class _LinkBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, skip, anchor, c1: ConvBN, ct: ConvTBN, c3: ConvBN):
        z1, r1 = c1.fwd(x)
        z2, r2 = ct.fwd(z1)
        z3, r3 = c3.fwd(z2)
        ctx.units = (c1, ct, c3)
        ctx.has_skip = skip is not None
        ctx.save_for_backward(*r1, *r2, *r3)
        return z3 + skip if skip is not None else z3

    @staticmethod
    def backward(ctx, dout):
        c1, ct, c3 = ctx.units
        s = ctx.saved_tensors
        r1, r2, r3 = s[0:3], s[3:6], s[6:9]
        dout = dout.contiguous()
        spec = Fn.BnBwdSpec(None, [ct.bn_target(r2)], affine=[(ct.scale, ct.shift)])   # z2 = relu(BN(y2))
        d2, _ = c3.bwd(dout, r3, dgrad_bn=spec)
        d1, _ = ct.bwd(d2, r2, prereduced=True)
        dx, _ = c1.bwd(d1, r1, need_dx=ctx.needs_input_grad[0])
        return dx, (dout if ctx.has_skip else None), None, None, None, None


def _conv_bn(seq):
    """(conv, bn) of a ConvBnRelu with BatchNorm, else NotImplementedError."""
    if not (isinstance(seq, nn.Sequential) and len(seq) == 3 and isinstance(seq[1], nn.BatchNorm2d)):
        raise NotImplementedError('native LinkNet: decoder_use_batchnorm=True required')
    return seq[0], seq[1]


class NativeLinknet(NativeUnet):
    """Same encoder, head, predict / export as :class:`NativeUnet`; LinkNet decoder."""

    def __init__(self, model, device, bce_w=1.0, dice_w=1.0, eps=1e-7):
        from mlcomp_amd.contrib.segmentation.decoders import LinknetDecoder
        dec = model.decoder
        if not isinstance(dec, LinknetDecoder):
            raise NotImplementedError('NativeLinknet: a LinknetDecoder model')
        ctx = self._lower_encoder(model)
        self.dec = []
        for i, blk in enumerate(dec.blocks):
            body = blk.body
            if len(body) != 5 or not isinstance(body[1], nn.ConvTranspose2d) or not isinstance(body[2], nn.BatchNorm2d):
                raise NotImplementedError('native LinkNet: decoder_use_batchnorm=True required')
            pre = f'decoder.blocks.{i}.body'
            c1, b1 = _conv_bn(body[0])
            c3, b3 = _conv_bn(body[4])
            self.dec.append((ConvBN(ctx, f'{pre}.0', c1, b1, act=True),
                             ConvTBN(ctx, f'{pre}.1', body[1], body[2], act=True),
                             ConvBN(ctx, f'{pre}.4', c3, b3, act=True)))
        self.head = SegHead(ctx, 'decoder.final_conv', dec.final_conv, bce_w, dice_w, eps)
        self._finish_init(device)

    def _units(self):
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down
        for units in self.dec:
            yield from units

    def features(self, x):
        """x: NHWC bf16 image (channels padded to 8, or the s2d image) -> [N, H, W, 32]."""
        anchor = self.ctx.anchor
        x0 = self.stem(x)
        y = self.pool(x0, anchor)
        feats = []
        for i, blk in enumerate(self.blocks):
            y = blk(y)
            if i in self.ends:
                feats.append(y)
        x1, x2, x3, x4 = feats
        d = x4
        for units, skip in zip(self.dec, [x3, x2, x1, x0, None]):
            d = _LinkBlockFn.apply(d, skip, anchor, *units)
        self.ctx.refresh_wt()    # transposed filters for the backward's dgrads
        return d
