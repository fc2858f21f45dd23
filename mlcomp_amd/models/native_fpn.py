"""Native execution of the FPN segmentation model
(:class:`mlcomp_amd.contrib.segmentation.models.FPN`; the reference's
`mlcomp/contrib/segmentation/fpn/{model,decoder}.py`) with a ResNet encoder.

* encoder: the native ResNet body shared with the U-Net engine
  (:meth:`NativeUnet._lower_encoder`): fused conv+BN(+residual)(+ReLU) nodes.
* every decoder convolution runs on the native MFMA GEMMs:
  - the 1x1 lateral convs (+ bias) and the 1x1 output conv are dense GEMMs over the NHWC
    pixel rows with the bias in the epilogue (``transformer.dense_fwd``), their weight and
    bias gradients one GEMM (``Fn.linear_wgrad_bias``), the input gradient ``dense_dgrad``;
  - the 3x3 convs of the segmentation heads are the implicit-GEMM conv kernels.
* the GroupNorm(32) + ReLU of the heads and the bilinear x2 upsamplings are native kernels
  (seg.hip; the CPU path uses tensor ops with the same explicit backward, :class:`_GNReluFn`);
  the nearest upsamplings, pyramid additions, Dropout2d and the BCE + Dice loss on the
  x4-upsampled logits are PyTorch tensor ops on the NHWC activations (no MIOpen / hipBLASLt
  call in the step).

Parameters live in the flat arenas (fused Adam, bucketed all-reduce) like the other engines.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.ops import _lib
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops import seg
from mlcomp_amd.ops import transformer as Tx
from .native_unet import NativeUnet


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _up(x, scale, mode):
    """NHWC upsampling (channels_last views, so no layout copies); the heads' bf16 bilinear
    x2 runs on the native kernels (:class:`_BilinearFn`)."""
    if mode == 'bilinear' and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return _BilinearFn.apply(x.contiguous(), scale)
    kw = {'align_corners': True} if mode == 'bilinear' else {}
    return _nhwc(F.interpolate(_nchw(x), scale_factor=scale, mode=mode, **kw))


class _BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        """``scale``: an integer factor or the output size (Ho, Wo)."""
        N, H, W, C = x.shape
        ctx.hw = (H, W)
        Ho, Wo = scale if isinstance(scale, tuple) else (H * scale, W * scale)
        return seg.bilinear_up_fwd(x, Ho, Wo)

    @staticmethod
    def backward(ctx, dy):
        return seg.bilinear_up_bwd(dy.contiguous(), *ctx.hw), None


# ---------------------------------------------------------------------------- units
class Conv1x1Bias:
    """1x1 conv with bias as a dense GEMM over pixel rows (NHWC)."""

    def __init__(self, ctx, name, conv: nn.Conv2d, f32_out=False):
        assert conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.groups == 1
        self.ctx, self.conv, self.f32_out = ctx, conv, f32_out
        self.Ci = conv.in_channels
        self.O = conv.out_channels
        # output channels padded to 8 (the GEMMs' column granularity: a 1-class output conv
        # is a [P, 8] GEMM); the padding rows stay zero (zero gradient, zero update) and
        # the caller slices the first O channels
        self.Co = (self.O + 7) // 8 * 8
        self.w = ctx.arena.weight(f'{name}.weight', (self.Co, self.Ci))
        self.b = ctx.arena.vector(f'{name}.bias', (self.Co,))

    def load_from_torch(self):
        dev = self.ctx.device
        self.w.master.zero_()
        self.b.master.zero_()
        self.w.master[:self.O].copy_(self.conv.weight.detach().float().reshape(self.O, self.Ci).to(dev))
        if self.conv.bias is not None:
            self.b.master[:self.O].copy_(self.conv.bias.detach().float().to(dev))

    def export_to_torch(self):
        self.conv.weight.data.copy_(self.w.master[:self.O].reshape(self.conv.weight.shape)
                                    .to(self.conv.weight.device))
        if self.conv.bias is not None:
            self.conv.bias.data.copy_(self.b.master[:self.O].to(self.conv.bias.device))

    def __call__(self, x):
        return _Conv1x1BiasFn.apply(x, self.ctx.anchor, self)


class _Conv1x1BiasFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, u: Conv1x1Bias):
        N, H, W, C = x.shape
        x2 = x.reshape(-1, C)
        if u.f32_out:
            y = Fn.linear_fwd(x2, u.w.bf16, u.b.master)
        else:
            y, _ = Tx.dense_fwd(x2, u.w.bf16, u.b.master)
        ctx.u = u
        ctx.save_for_backward(x2)
        return y.view(N, H, W, u.Co)

    @staticmethod
    def backward(ctx, dy):
        u: Conv1x1Bias = ctx.u
        (x2,) = ctx.saved_tensors
        shp = dy.shape
        d2 = dy.reshape(-1, u.Co).to(torch.bfloat16).contiguous()
        Fn.linear_wgrad_bias(d2, x2, u.w.grad, u.b.grad)
        dx = Tx.dense_dgrad(d2, u.w.bf16).view(*shp[:3], u.Ci) if ctx.needs_input_grad[0] else None
        u.ctx.arena.mark_ready(u.w)
        u.ctx.arena.mark_ready(u.b)
        return dx, None, None


class Conv3x3:
    """3x3 / stride 1 / pad 1 conv on the implicit-GEMM kernels.  With a bias (an output
    conv: PSPNet's head) the output channels are padded to 8 (zero filters, zero gradient)
    and the result is fp32 ``conv + bias`` over all padded channels (the caller slices)."""

    def __init__(self, ctx, name, conv: nn.Conv2d):
        assert conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
        assert conv.groups == 1
        self.ctx, self.conv = ctx, conv
        self.O, self.Ci = conv.out_channels, conv.in_channels
        self.has_bias = conv.bias is not None
        self.Co = (self.O + 7) // 8 * 8 if self.has_bias else self.O
        self.w = ctx.arena.weight(f'{name}.weight', (self.Co, 3, 3, self.Ci))
        self.b = ctx.arena.vector(f'{name}.bias', (self.Co,)) if self.has_bias else None

    def load_from_torch(self):
        self.w.master.zero_()
        self.w.master[:self.O].copy_(self.conv.weight.detach().permute(0, 2, 3, 1).float().to(self.ctx.device))
        if self.has_bias:
            self.b.master.zero_()
            self.b.master[:self.O].copy_(self.conv.bias.detach().float().to(self.ctx.device))

    def export_to_torch(self):
        self.conv.weight.data.copy_(self.w.master[:self.O].permute(0, 3, 1, 2).to(self.conv.weight.device))
        if self.has_bias:
            self.conv.bias.data.copy_(self.b.master[:self.O].to(self.conv.bias.device))

    def __call__(self, x):
        return _Conv3x3Fn.apply(x, self.ctx.anchor, self)


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, u: Conv3x3):
        ctx.u = u
        ctx.save_for_backward(x)
        y = Fn.conv2d_fwd(x, u.w.bf16, 1, 1)
        return y.float() + u.b.master if u.has_bias else y

    @staticmethod
    def backward(ctx, dy):
        u: Conv3x3 = ctx.u
        (x,) = ctx.saved_tensors
        if u.has_bias:
            u.b.grad.add_(dy.float().sum((0, 1, 2)))
            u.ctx.arena.mark_ready(u.b)
        dy = dy.to(torch.bfloat16).contiguous()
        Fn.conv2d_wgrad(dy, x, u.w.shape, 1, 1, out=u.w.grad, accumulate=True)
        dx = Fn.conv2d_dgrad(dy, u.w.bf16, x.shape, 1, 1) if ctx.needs_input_grad[0] else None
        u.ctx.arena.mark_ready(u.w)
        return dx, None, None


class GNRelu:
    """GroupNorm + ReLU over NHWC activations, parameters in the arena."""

    def __init__(self, ctx, name, gn: nn.GroupNorm):
        self.ctx, self.gn = ctx, gn
        self.G, self.C, self.eps = gn.num_groups, gn.num_channels, gn.eps
        self.g = ctx.arena.vector(f'{name}.weight', (self.C,))
        self.b = ctx.arena.vector(f'{name}.bias', (self.C,))

    def load_from_torch(self):
        self.g.master.copy_(self.gn.weight.detach().float().to(self.ctx.device))
        self.b.master.copy_(self.gn.bias.detach().float().to(self.ctx.device))

    def export_to_torch(self):
        self.gn.weight.data.copy_(self.g.master.to(self.gn.weight.device))
        self.gn.bias.data.copy_(self.b.master.to(self.gn.bias.device))

    def __call__(self, x):
        return _GNReluFn.apply(x, self.ctx.anchor, self)


def _gn_stats(u: GNRelu, x):
    N, H, W, C = x.shape
    xf = x.float().view(N, H * W, u.G, C // u.G)
    mean = xf.mean((1, 3), keepdim=True)
    rstd = torch.rsqrt(xf.var((1, 3), unbiased=False, keepdim=True) + u.eps)
    return xf, mean, rstd


def _gn_native(u: GNRelu, x) -> bool:
    C = x.shape[-1]
    return x.is_cuda and C % 8 == 0 and 256 % (C // 8) == 0 and C % u.G == 0


class _GNReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, u: GNRelu):
        ctx.u = u
        if _gn_native(u, x):      # seg.hip: per-(sample, channel) sums + one apply pass
            N, H, W, C = x.shape
            fst = torch.zeros(N, C, 2, device=x.device, dtype=torch.float32)
            z = torch.empty_like(x)
            _lib.call('mlc_gn_relu_fwd', _lib.ptr(x), _lib.ptr(u.g.master), _lib.ptr(u.b.master), _lib.ptr(z),
                      _lib.ptr(fst), N, H * W, C, u.G, float(u.eps), _lib.stream())
            ctx.native = True
            ctx.save_for_backward(x, fst)
            return z
        ctx.native = False
        xf, mean, rstd = _gn_stats(u, x)
        shape = (1, 1, u.G, u.C // u.G)
        y = (xf - mean) * rstd * u.g.master.view(shape) + u.b.master.view(shape)
        ctx.save_for_backward(x, mean, rstd)
        return torch.relu(y).to(torch.bfloat16).view(x.shape)

    @staticmethod
    def backward(ctx, dz):
        u: GNRelu = ctx.u
        if ctx.native:
            x, fst = ctx.saved_tensors
            N, H, W, C = x.shape
            bst = torch.zeros(N, C, 2, device=x.device, dtype=torch.float32)
            dx = torch.empty_like(x)
            _lib.call('mlc_gn_relu_bwd', _lib.ptr(x), _lib.ptr(dz.contiguous()), _lib.ptr(u.g.master),
                      _lib.ptr(u.b.master), _lib.ptr(fst), _lib.ptr(bst), _lib.ptr(dx), N, H * W, C, u.G,
                      float(u.eps), _lib.stream())
            sums = bst.sum(0)
            u.g.grad.add_(sums[:, 0])
            u.b.grad.add_(sums[:, 1])
            u.ctx.arena.mark_ready(u.g)
            u.ctx.arena.mark_ready(u.b)
            return dx, None, None
        x, mean, rstd = ctx.saved_tensors
        N, H, W, C = x.shape
        shape = (1, 1, u.G, C // u.G)
        xhat = (x.float().view(N, H * W, u.G, C // u.G) - mean) * rstd
        gam = u.g.master.view(shape)
        dy = dz.float().view(xhat.shape) * ((xhat * gam + u.b.master.view(shape)) > 0)
        u.g.grad.add_((dy * xhat).sum((0, 1)).reshape(C))
        u.b.grad.add_(dy.sum((0, 1)).reshape(C))
        u.ctx.arena.mark_ready(u.g)
        u.ctx.arena.mark_ready(u.b)
        dxh = dy * gam
        dx = rstd * (dxh - dxh.mean((1, 3), keepdim=True) - xhat * (dxh * xhat).mean((1, 3), keepdim=True))
        return dx.to(torch.bfloat16).view(x.shape), None, None


class UpsampledSegHead:
    """Output conv (``conv``: a :class:`Conv1x1Bias` with fp32 output or a biased
    :class:`Conv3x3`) -> x ``scale`` bilinear -> BCE + soft Dice (contrib.criterion.
    BCEDiceLoss) with the loss sums [BCE sum, sum s*t, sum s, sum t] kept in the workspace
    like :class:`~.native_unet.SegHead` (FPN: 1x1 at stride 4; PSPNet: 3x3 at stride 8)."""

    def __init__(self, ctx, conv, K, scale, bce_w=1.0, dice_w=1.0, eps=1e-7):
        assert K <= 4
        self.ctx = ctx
        self.conv = conv
        self.K, self.scale = K, scale
        self.bce_w, self.dice_w, self.eps = bce_w, dice_w, eps
        self.k_sums = ctx.ws.request('decoder.head.sums', 4)

    def sums(self):
        return self.ctx.ws[self.k_sums]

    def logits(self, x):
        """[N, H/scale, W/scale, C] bf16 -> fp32 logits [N, H, W, K] (NHWC)."""
        return _up(self.conv(x)[..., :self.K].float(), self.scale, 'bilinear')

    def loss(self, z, target):
        zf = z.reshape(-1)
        t = target.reshape(-1).float()
        s = torch.sigmoid(zf)
        sums = self.sums()
        bce = F.binary_cross_entropy_with_logits(zf, t, reduction='sum')
        st = (s * t).sum()
        ss = s.sum()
        with torch.no_grad():
            sums.copy_(torch.stack([bce.detach(), st.detach(), ss.detach(), t.sum()]))
        dice = (2 * st + self.eps) / (ss + t.sum() + self.eps)
        return self.bce_w * bce / zf.numel() + self.dice_w * (1 - dice)


class NativeFPN(NativeUnet):
    """Same encoder / step interface as :class:`NativeUnet`; FPN decoder."""

    def __init__(self, model, device, bce_w=1.0, dice_w=1.0, eps=1e-7):
        from mlcomp_amd.contrib.segmentation.decoders import FPNDecoder
        dec = model.decoder
        if not isinstance(dec, FPNDecoder):
            raise NotImplementedError('NativeFPN: an FPNDecoder model')
        ctx = self._lower_encoder(model)
        self.dec_m = dec
        self.lat_top = Conv1x1Bias(ctx, 'decoder.lateral_top', dec.lateral_top)
        self.laterals = [Conv1x1Bias(ctx, f'decoder.laterals.{i}', c) for i, c in enumerate(dec.laterals)]
        self.heads = []
        for i, h in enumerate(dec.heads):
            layers = []
            for j, gu in enumerate(h):
                pre = f'decoder.heads.{i}.{j}'
                layers.append((Conv3x3(ctx, f'{pre}.0', gu[0]), GNRelu(ctx, f'{pre}.1', gu[1]), gu.upsample))
            self.heads.append(layers)
        self.drop = dec.dropout.p
        self.head = UpsampledSegHead(ctx, Conv1x1Bias(ctx, 'decoder.final_conv', dec.final_conv, f32_out=True),
                                     dec.final_conv.out_channels, 4, bce_w, dice_w, eps)
        self._finish_init(device)

    def _units(self):
        yield self.stem
        for blk in self.blocks:
            yield from blk.units
            if blk.down is not None:
                yield blk.down

    def _dec_units(self):
        yield self.lat_top
        yield from self.laterals
        for layers in self.heads:
            for conv, gn, _ in layers:
                yield conv
                yield gn
        yield self.head.conv

    def _finish_init(self, device):
        self.ctx.finalize(device)
        self._default_schedule()
        for u in self._units():
            u.load_from_torch()
        for u in self._dec_units():
            u.load_from_torch()
        self.ctx.arena.decay.refresh_mirror()

    def features(self, x):
        """x: NHWC bf16 image -> the summed stride-4 head features [N, H/4, W/4, 128] bf16."""
        anchor = self.ctx.anchor
        x0 = self.stem(x)
        y = self.pool(x0, anchor)
        feats = []
        for i, blk in enumerate(self.blocks):
            y = blk(y)
            if i in self.ends:
                feats.append(y)
        x1, x2, x3, x4 = feats
        p = self.lat_top(x4)
        pyramid = [p]
        for lat, c in zip(self.laterals, (x3, x2, x1)):
            p = _up(p, 2, 'nearest') + lat(c)
            pyramid.append(p)
        acc = None
        for layers, t in zip(self.heads, pyramid):
            for conv, gn, up in layers:
                t = gn(conv(t))
                if up:
                    t = _up(t, 2, 'bilinear')
            acc = t.float() if acc is None else acc + t.float()
        self.ctx.refresh_wt()    # transposed filters for the encoder's backward dgrads
        if self.ctx.training and self.drop > 0:
            acc = _nhwc(F.dropout2d(_nchw(acc), self.drop, True))
        return acc.to(torch.bfloat16)

    def loss(self, x, target):
        """BCE + Dice loss (device scalar); ``target`` fp32 [N*H*W*K] in pixel order."""
        return self.head.loss(self.head.logits(self.features(x)), target)

    def predict(self, x, target=None):
        h = self.head
        was = self.ctx.training
        self.train(False)
        try:
            with torch.no_grad():
                z = h.logits(self.features(x))
                out = z.permute(0, 3, 1, 2)
                loss = None
                if target is not None:
                    m = target.to(z.device).float()
                    t = m.permute(0, 2, 3, 1) if m.dim() == 4 else m.unsqueeze(-1)
                    loss = h.loss(z, t.contiguous())
            return out, loss
        finally:
            self.train(was)

    def export_to_torch(self):
        for u in self._units():
            u.export_to_torch()
        for u in self._dec_units():
            u.export_to_torch()
        return self.torch_model
