"""Native (HIP-kernel) execution of the U-Net segmentation model
(:class:`mlcomp_amd.contrib.segmentation.models.Unet`, the reference's
`mlcomp/contrib/segmentation/unet/model.py:6-57`) with a ResNet encoder.

* encoder: the ResNet stem + four stages lowered exactly like the classifier
  (:func:`~mlcomp_amd.models.native_resnet.lower_resnet_body`): fused conv+BN(+residual)
  (+ReLU) nodes, BN statistics out of the conv epilogues, BN-backward reductions fused into
  the dgrad epilogues.  The outputs of stages 1-3 and of the stem also feed decoder skips,
  so their gradient is only complete after the skip gradient is added: the block after
  each of them is unlinked (``prev = None``) and reduces its own BN from the full sum.
* decoder block: one fused kernel for the x2 nearest upsample + skip concat
  (``ops.seg.upcat_*``), then two fused conv3x3+BN+ReLU nodes.
* head: the 1x1 output conv (16 -> K <= 4 classes, + bias) is K per-pixel dot products fused with
  BCE-with-logits + soft-Dice (``ops.seg.seg_head_*``).

Activations are NHWC bf16 end to end; parameters live in the flat arenas (fused Adam,
bucketed RCCL all-reduce).  ``export_to_torch()`` writes the weights back.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from mlcomp_amd.ops import seg
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import ConvBN, NativeContext
from .native_resnet import lower_resnet_body


class _UpCatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, lo, skip, anchor):
        ctx.c1 = lo.shape[3]
        ctx.has_skip = skip is not None
        return seg.upcat_fwd(lo, skip)

    @staticmethod
    def backward(ctx, d):
        dlo, dskip = seg.upcat_bwd(d, ctx.c1)
        return dlo, (dskip if ctx.has_skip else None), None


class _DecoderPairFn(torch.autograd.Function):
    """A decoder block's two conv+BN+ReLU units as one autograd node, so the second
    unit's dgrad epilogue also masks the first unit's output gradient and accumulates the
    first BN's backward sums (``Fn.BnBwdSpec``): no separate BN-backward reduction pass."""

    @staticmethod
    def forward(ctx, x, anchor, c1: ConvBN, c2: ConvBN):
        z1, r1 = c1.fwd(x)
        z2, r2 = c2.fwd(z1)
        ctx.units = (c1, c2)
        ctx.save_for_backward(*r1, *r2)
        return z2

    @staticmethod
    def backward(ctx, dz):
        c1, c2 = ctx.units
        s = ctx.saved_tensors
        r1, r2 = s[:3], s[3:]
        spec = Fn.BnBwdSpec(None, [c1.bn_target(r1)], affine=[(c1.scale, c1.shift)])   # z1 = relu(BN(y1))
        d1, _ = c2.bwd(dz.contiguous(), r2, dgrad_bn=spec)
        dx, _ = c1.bwd(d1, r1, prereduced=True, need_dx=ctx.needs_input_grad[0])
        return dx, None, None, None


class SegHead:
    """1x1 conv (C -> K <= 4 classes, bias) + per-class sigmoid BCE-with-logits + soft Dice
    over all classes (contrib.criterion.BCEDiceLoss), one forward and one backward kernel.
    Targets are [P, K] in pixel order (NHWC masks).  ``__call__`` returns the loss (device scalar); backward assumes
    d(loss) = 1."""

    def __init__(self, ctx: NativeContext, name: str, conv: nn.Conv2d, bce_w=1.0, dice_w=1.0, eps=1e-7):
        assert conv.out_channels <= 4 and conv.kernel_size == (1, 1), 'native SegHead: <= 4 classes, 1x1 conv'
        self.ctx = ctx
        self.conv = conv
        self.C = conv.in_channels
        self.K = conv.out_channels
        self.w = ctx.arena.weight(f'{name}.weight', (self.K, self.C))
        self.b = ctx.arena.vector(f'{name}.bias', (self.K,))
        self.bce_w, self.dice_w, self.eps = bce_w, dice_w, eps
        self.k_sums = ctx.ws.request(f'{name}.sums', 4)
        self.logits = None      # optional fp32 [P] buffer the forward fills (metrics/inference)

    def load_from_torch(self):
        dev = self.ctx.device
        self.w.master.copy_(self.conv.weight.detach().float().reshape(self.K, self.C).to(dev))
        b = self.conv.bias.detach().float() if self.conv.bias is not None else torch.zeros(self.K)
        self.b.master.copy_(b.to(dev))

    def export_to_torch(self):
        self.conv.weight.data.copy_(self.w.master.reshape(self.conv.weight.shape).to(self.conv.weight.device))
        if self.conv.bias is not None:
            self.conv.bias.data.copy_(self.b.master.to(self.conv.bias.device))

    def sums(self):
        return self.ctx.ws[self.k_sums]

    def __call__(self, x, target):
        return _SegHeadFn.apply(x, target, self.ctx.anchor, self)


class _SegHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, target, anchor, h: SegHead):
        xf = x.reshape(-1, h.C)
        sums = h.sums()
        seg.seg_head_fwd(xf, h.w.master, h.b.master, target, sums, logits=h.logits)
        ctx.h = h
        ctx.save_for_backward(x, target)
        return seg.seg_loss(sums, xf.shape[0] * h.K, h.bce_w, h.dice_w, h.eps)

    @staticmethod
    def backward(ctx, dloss):
        x, target = ctx.saved_tensors
        h: SegHead = ctx.h
        dx = seg.seg_head_bwd(x.reshape(-1, h.C), h.w.master, h.b.master, target, h.sums(), h.w.grad, h.b.grad,
                              h.bce_w, h.dice_w, h.eps)
        h.ctx.arena.mark_ready(h.w)
        h.ctx.arena.mark_ready(h.b)
        return dx.view(x.shape), None, None, None


class NativeUnet:
    def __init__(self, model, device, bce_w=1.0, dice_w=1.0, eps=1e-7):
        dec = model.decoder
        if not isinstance(dec.center, nn.Identity):
            raise NotImplementedError('native U-Net: center block not supported')
        ctx = self._lower_encoder(model)
        self.dec = []
        for i, blk in enumerate(dec.blocks):
            if not (isinstance(blk.att_in, nn.Identity) and isinstance(blk.att_out, nn.Identity)):
                raise NotImplementedError('native U-Net: scSE attention not supported')
            c1, c2 = blk.convs[0], blk.convs[1]
            if not (isinstance(c1[1], nn.BatchNorm2d) and isinstance(c2[1], nn.BatchNorm2d)):
                raise NotImplementedError('native U-Net: decoder_use_batchnorm=True required')
            pre = f'decoder.blocks.{i}.convs'
            self.dec.append((ConvBN(ctx, f'{pre}.0', c1[0], c1[1], act=True),
                             ConvBN(ctx, f'{pre}.1', c2[0], c2[1], act=True)))
        self.head = SegHead(ctx, 'decoder.final_conv', dec.final_conv, bce_w, dice_w, eps)
        # decoder blocks as one autograd node with the first BN's backward reduction fused
        # into the second conv's dgrad (MLC_UNET_PAIR=0: two separate nodes)
        self.fuse_pair = os.environ.get('MLC_UNET_PAIR', '1') == '1'
        self._finish_init(device)

    def _default_schedule(self):
        """Segmentation engines (32 images @256²: short per-layer GEMMs): the weight
        gradients form one unjoined side chain (joined before the optimizer) instead of a
        join per conv, each of which costs ~10 us of cross-queue latency.  Interleaved A/B on
        one MI355X, 2 rounds: U-Net 4,184 / 4,168 -> 4,565 / 4,563 img/s, LinkNet 4,533 / 4,632
        -> 5,003 / 4,979, FPN 4,052 / 4,072 -> 4,278 / 4,303 (profiles/round5/seg_wgrad_join_ab.txt).
        MLC_WGRAD_DEFER=0 restores the per-conv join."""
        self.ctx.default_wgrad_defer(True)

    def _lower_encoder(self, model) -> NativeContext:
        """Context + the ResNet encoder's native stem / pool / blocks (shared with the
        LinkNet engine).  The stage outputs that feed decoder skips unlink the next block."""
        from mlcomp_amd.contrib.segmentation.encoders import ResNetEncoder
        enc = model.encoder
        if not isinstance(enc, ResNetEncoder):
            raise NotImplementedError('native segmentation: ResNet encoders (use engine=torch for others)')
        self.torch_model = model
        ctx = self.ctx = NativeContext()
        ctx.default_dgrad_first(True)     # +1.8 % on the U-Net (profiles/round3/README.md)
        self.stem, self.pool, self.blocks, self.ends = lower_resnet_body(ctx, enc.body, prefix='encoder.body.',
                                                                          s2d_stem=True)
        for e in self.ends[:3]:          # stage outputs 1-3 feed skips (see module doc)
            self.blocks[e + 1].prev = None
        for blk in self.blocks:          # measured -0.9 % here (profiles/round2_ab): off unless asked
            blk.down_stream = os.environ.get('MLC_DOWN_STREAM_UNET', '0') == '1'
        return ctx

    def _finish_init(self, device):
        self.ctx.finalize(device)
        self._default_schedule()
        for u in self._units():
            u.load_from_torch()
        self.head.load_from_torch()
        self.ctx.arena.decay.refresh_mirror()

    def _units(self):
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down
        for c1, c2 in self.dec:
            yield c1
            yield c2

    # ------------------------------------------------------------------ execution
    def features(self, x):
        """x: NHWC bf16 image (channels padded to 8) -> decoder output [N, H, W, 16]."""
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
        for (c1, c2), skip in zip(self.dec, [x3, x2, x1, x0, None]):
            d = _UpCatFn.apply(d, skip, anchor)
            if self.fuse_pair:
                d = _DecoderPairFn.apply(d, anchor, c1, c2)
            else:
                d = c2(c1(d))
        self.ctx.refresh_wt()    # transposed filters for the backward's dgrads
        return d

    def loss(self, x, target):
        """BCE + Dice loss (device scalar); ``target`` fp32 [N*H*W*K] in pixel order."""
        return self.head(self.features(x), target)

    def predict(self, x, target=None):
        """Inference forward on the native kernels (BN running statistics, no autograd):
        x NHWC bf16 (channels padded to 8, or the stem's s2d image) -> fp32 logits
        [N, K, H, W]; with ``target`` ([N, K, H, W] / [N, H, W] masks) also the loss the
        training head computes (bce_w * BCE + dice_w * (1 - dice)) as a device scalar."""
        h = self.head
        was = self.ctx.training
        self.train(False)
        try:
            with torch.no_grad():
                d = self.features(x)
                N, H, W, _ = d.shape
                P = N * H * W
                logits = torch.empty(P, h.K, device=d.device, dtype=torch.float32)
                t = torch.zeros(P, h.K, device=d.device, dtype=torch.float32)
                if target is not None:
                    m = target.to(d.device).float()
                    t.copy_((m.permute(0, 2, 3, 1) if m.dim() == 4 else m.unsqueeze(-1)).reshape(P, h.K))
                sums = torch.zeros(4, device=d.device, dtype=torch.float32)
                seg.seg_head_fwd(d.reshape(P, h.C), h.w.master, h.b.master, t, sums, logits=logits)
                out = logits.view(N, H, W, h.K).permute(0, 3, 1, 2)
                loss = seg.seg_loss(sums, P * h.K, h.bce_w, h.dice_w, h.eps) if target is not None else None
            return out, loss
        finally:
            self.train(was)

    def train(self, mode=True):
        self.ctx.training = mode
        return self

    def eval(self):
        return self.train(False)

    @property
    def arena(self):
        return self.ctx.arena

    def export_to_torch(self):
        for u in self._units():
            u.export_to_torch()
        self.head.export_to_torch()
        return self.torch_model

    def num_params(self):
        return self.ctx.arena.num_params()
