"""Python entry points of the segmentation kernels (``csrc/kernels/seg.hip``): the fused
x2-upsample + skip-concat of the U-Net decoder and the fused 1x1 head + BCE-with-logits +
soft-Dice loss, each with an fp32 PyTorch reference used on CPU and by
the numerics tests.  Activations are NHWC bf16."""
from __future__ import annotations

import torch

from . import _lib
from .functional import _cuda


def upcat_fwd(lo, skip):
    """lo [N, h, w, C1], skip [N, 2h, 2w, C2] or None -> [N, 2h, 2w, C1 + C2]."""
    N, h, w, C1 = lo.shape
    C2 = skip.shape[3] if skip is not None else 0
    if _cuda(lo):
        assert lo.is_contiguous() and (skip is None or (skip.is_contiguous() and tuple(skip.shape) == (N, 2 * h, 2 * w, C2)))
        out = torch.empty(N, 2 * h, 2 * w, C1 + C2, device=lo.device, dtype=torch.bfloat16)
        _lib.call('mlc_upcat_fwd', _lib.ptr(lo), _lib.ptr(skip), _lib.ptr(out), N, h, w, C1, C2, _lib.stream())
        return out
    up = lo.repeat_interleave(2, 1).repeat_interleave(2, 2)
    return torch.cat([up, skip], 3) if skip is not None else up.contiguous()


def upcat_bwd(dout, C1):
    """Returns (dlo [N, h, w, C1], dskip [N, 2h, 2w, C2] or None)."""
    N, H, W, C = dout.shape
    h, w, C2 = H // 2, W // 2, C - C1
    if _cuda(dout):
        dout = dout.contiguous()
        dlo = torch.empty(N, h, w, C1, device=dout.device, dtype=torch.bfloat16)
        dskip = torch.empty(N, H, W, C2, device=dout.device, dtype=torch.bfloat16) if C2 else None
        _lib.call('mlc_upcat_bwd', _lib.ptr(dout), _lib.ptr(dlo), _lib.ptr(dskip), N, h, w, C1, C2, _lib.stream())
        return dlo, dskip
    d = dout.float()
    dlo = d[..., :C1].reshape(N, h, 2, w, 2, C1).sum((2, 4)).to(torch.bfloat16)
    dskip = d[..., C1:].to(torch.bfloat16).contiguous() if C2 else None
    return dlo, dskip


def seg_head_fwd(x, w, b, target, sums, logits=None):
    """x [P, C] bf16, w [K, C] (or [C] for one class) / b [K] fp32, target [P, K] (or [P])
    fp32.  Accumulates the loss sums over pixels and classes (BCE sum, sum s*t, sum s,
    sum t) into ``sums`` [4]; writes logits [P, K] if given."""
    P, C = x.shape
    K = w.numel() // C
    if _cuda(x) and not _lib.DETERMINISTIC:     # the kernel's loss sums use float atomics
        _lib.call('mlc_seg_head_fwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(target), _lib.ptr(logits),
                  _lib.ptr(sums), P, C, K, _lib.stream())
        return sums
    z = x.float() @ w.float().reshape(K, C).t() + b.float().reshape(1, K)
    t = target.float().reshape(P, K)
    s = torch.sigmoid(z)
    if logits is not None:
        logits.copy_(z.reshape(logits.shape))
    bce = torch.nn.functional.binary_cross_entropy_with_logits(z, t, reduction='sum')
    sums.add_(torch.stack([bce, (s * t).sum(), s.sum(), t.sum()]))
    return sums


def seg_loss(sums, n, bce_w=1.0, dice_w=1.0, eps=1e-7):
    """Loss value from the forward sums (a device scalar, no host sync); ``n`` = pixels x
    classes (the BCE mean's denominator)."""
    dice = (2 * sums[1] + eps) / (sums[2] + sums[3] + eps)
    return bce_w * sums[0] / n + dice_w * (1 - dice)


def seg_head_bwd(x, w, b, target, sums, dw, db, bce_w=1.0, dice_w=1.0, eps=1e-7):
    """Returns dx [P, C] bf16; dw [K, C] / db [K] are ACCUMULATED (+=)."""
    P, C = x.shape
    K = w.numel() // C
    if _cuda(x) and not _lib.DETERMINISTIC:     # dw / db use float atomics
        dx = torch.empty_like(x)
        _lib.call('mlc_seg_head_bwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(b), _lib.ptr(target), _lib.ptr(sums),
                  _lib.ptr(dx), _lib.ptr(dw), _lib.ptr(db), P, C, K, float(bce_w), float(dice_w), float(eps),
                  _lib.stream())
        return dx
    wk = w.float().reshape(K, C)
    z = x.float() @ wk.t() + b.float().reshape(1, K)
    t = target.float().reshape(P, K)
    s = torch.sigmoid(z)
    den = sums[2] + sums[3] + eps
    num = 2 * sums[1] + eps
    dz = bce_w * (s - t) / (P * K) + dice_w * (-2 * t / den + num / den ** 2) * s * (1 - s)
    dw.add_((dz.t() @ x.float()).reshape(dw.shape))
    db.add_(dz.sum(0).reshape(db.shape))
    return (dz @ wk).to(torch.bfloat16)


__all__ = ['upcat_fwd', 'upcat_bwd', 'seg_head_fwd', 'seg_head_bwd', 'seg_loss']


def bilinear_up_fwd(x, Ho, Wo):
    """NHWC bf16 bilinear upsampling with align_corners=True (C % 8 == 0 on the GPU)."""
    N, H, W, C = x.shape
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_bilinear_up_fwd', _lib.ptr(x), _lib.ptr(y), N, H, W, C, Ho, Wo, _lib.stream())
        return y
    y = torch.nn.functional.interpolate(x.permute(0, 3, 1, 2).float(), size=(Ho, Wo), mode='bilinear',
                                        align_corners=True)
    return y.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def bilinear_up_bwd(dy, H, W):
    """Input gradient of :func:`bilinear_up_fwd` (gather over the reading outputs, fp32)."""
    N, Ho, Wo, C = dy.shape
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_bilinear_up_bwd', _lib.ptr(dy.contiguous()), _lib.ptr(dx), N, H, W, C, Ho, Wo, _lib.stream())
        return dx
    with torch.enable_grad():     # (called from inside an autograd backward)
        x = torch.zeros(N, C, H, W, requires_grad=True)
        y = torch.nn.functional.interpolate(x, size=(Ho, Wo), mode='bilinear', align_corners=True)
        (g,) = torch.autograd.grad(y, x, dy.permute(0, 3, 1, 2).float())
    return g.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
