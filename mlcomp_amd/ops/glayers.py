"""Native layers of the generic engine (:mod:`mlcomp_amd.models.native_generic`).

The hand-lowered engines (ResNet, U-Net, BERT, ...) build their layers from
:mod:`mlcomp_amd.ops.layers` for one architecture each.  The generic engine lowers ANY
``nn.Module`` graph (torch.fx) onto the kernels, so its layers are written per op, not per
architecture:

* parameter sets (``ConvParams``, ``BNParams``, ``LinearParams``) - one per source module,
  slots of the shared :class:`~mlcomp_amd.ops.arena.ParamArena` in kernel layout, loaded
  from / exported to the torch module; a module used at several call sites shares them;
* sites (``ConvBNAct``, ``BNAct``, ``LinearAct``, ``MaxPool``, ``GlobalAvgPool``) - one per
  lowered call site of the fx graph (an ``nn.Module`` the graph calls), holding what a call
  needs (activation, residual, per-call statistics scratch) and an autograd Function.

Values between sites are ordinary logical-NCHW tensors, so every op the lowering leaves to
PyTorch (views, adds, concats, dropout, the loss ...) sees what it expects.  A site's
output is the NHWC kernel result viewed as NCHW (channels_last strides): the next site
reads it as NHWC without a copy.  Channel counts that are not a multiple of 8 are padded
inside a site (weights zero-padded in the arena, activations padded on the way in and
sliced on the way out) - only small stems / toy nets pay for that copy.

Gradients of weights go straight into the grad arena (the step zeroes it once, every wgrad
accumulates) and a slot is marked ready for the bucketer after the last backward use of
its weight in the step.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn

from . import functional as Fn
from . import seg as Seg
from .layers import NativeContext


def ceil8(c: int) -> int:
    return (c + 7) // 8 * 8


def to_nhwc(x: torch.Tensor, cp: Optional[int] = None) -> torch.Tensor:
    """Logical NCHW (any strides / float dtype) -> contiguous NHWC bf16, channels padded to
    ``cp``.  Free for a channels_last bf16 tensor with ``C == cp``."""
    y = x.permute(0, 2, 3, 1)
    if y.dtype != torch.bfloat16:
        y = y.to(torch.bfloat16)
    C = y.shape[-1]
    if cp is not None and cp != C:
        y = torch.nn.functional.pad(y, (0, cp - C))
    return y.contiguous()


def from_nhwc(y: torch.Tensor, C: int) -> torch.Tensor:
    """NHWC kernel output -> logical NCHW view (channels_last strides), padding dropped."""
    if y.shape[-1] != C:
        y = y[..., :C]
    return y.permute(0, 3, 1, 2)


def frames_of(x: torch.Tensor) -> torch.Tensor:
    """Logical [N, C, T, H, W] -> logical [N*T, C, H, W] (the T frames as images).  A view
    when x is channels_last_3d ([N, T, H, W, C] in memory), which every 3D site emits."""
    N, C, T, H, W = x.shape
    return x.transpose(1, 2).reshape(N * T, C, H, W)


def video_of(y: torch.Tensor, N: int) -> torch.Tensor:
    """Inverse of :func:`frames_of`: logical [N*T, C, H, W] -> [N, C, T, H, W] (a view of a
    channels_last frame tensor, i.e. channels_last_3d)."""
    NT, C, H, W = y.shape
    return y.reshape(N, NT // N, C, H, W).transpose(1, 2)


class Conv3dAs2d:
    """An nn.Conv3d (or nn.Conv1d) seen as the 2D conv over frames that computes it: the
    kt temporal taps are unfolded into the channels (channel c*kt + dt holds frame
    t*st + dt*dil - pad of channel c; per-group channels stay contiguous), so the filter is
    the conv's own weight viewed as [Co, Cg*kt, kh, kw] - no copy, exports write through.
    The 2D conv then runs over N*To frames on the implicit-GEMM / grouped / depthwise
    kernels, and a BatchNorm3d over its output is a BatchNorm2d over those frames."""

    def __init__(self, m: nn.Module):
        self.src3d = m
        if isinstance(m, nn.Conv1d):
            (kt,), (st,), (pt,), (dt,) = m.kernel_size, m.stride, m.padding, m.dilation
            kh = kw = 1
            self.stride, self.padding, self.dilation = (1, 1), (0, 0), (1, 1)
        else:
            kt, kh, kw = m.kernel_size
            st, pt, dt = m.stride[0], m.padding[0], m.dilation[0]
            self.stride, self.padding, self.dilation = tuple(m.stride[1:]), tuple(m.padding[1:]), tuple(m.dilation[1:])
        self.kt, self.st, self.pt, self.dt = kt, st, pt, dt
        self.kernel_size = (kh, kw)
        self.groups = m.groups
        self.padding_mode = m.padding_mode
        self.in_channels = m.in_channels * kt
        self.out_channels = m.out_channels
        self.bias = m.bias
        self._shape = (m.weight.shape[0], m.weight.shape[1] * kt, kh, kw)

    @property
    def weight(self):
        return self.src3d.weight.view(self._shape)

    def unfold(self, x: torch.Tensor, link: Optional['Frames'] = None) -> torch.Tensor:
        """Logical [N, C, T, H, W] (or [N, C, L]) -> the frames [N*To, C*kt, H, W] the 2D
        conv reads.  On the GPU (C % 8 == 0, kt <= 8) the native unfold / fold kernels
        (``csrc/kernels/video.hip``) build it from the channels_last_3d activation and fold
        the gradient back; elsewhere torch gather / pad ops (autograd folds the gradient).
        ``link``: the Frames site that owns this unfold takes part in a gradient hand-off
        (:class:`Frames`): the fold adds the other branch's gradient of ``x`` / hands its
        result to the sibling site - in the fold kernel on the native path, through
        :class:`_GradLink` (one add) elsewhere."""
        if x.dim() == 3:
            x = x[:, :, :, None, None]
        N, C, T, H, W = x.shape
        kt, st, pt, dt = self.kt, self.st, self.pt, self.dt
        native = x.is_cuda and C % 8 == 0 and kt <= 8 and not (kt == 1 and st == 1 and pt == 0)
        if link is not None and not native:
            x = _GradLink.apply(x, link)
        if kt == 1 and st == 1 and pt == 0:
            return frames_of(x)
        To = (T + 2 * pt - dt * (kt - 1) - 1) // st + 1
        if native:
            return _TemporalUnfold.apply(x, kt, st, pt, dt, To, link)
        if pt:
            x = torch.nn.functional.pad(x, (0, 0, 0, 0, pt, pt))
        idx = (torch.arange(To, device=x.device)[:, None] * st + torch.arange(kt, device=x.device)[None] * dt)
        g = x.index_select(2, idx.reshape(-1)).reshape(N, C, To, kt, H, W)
        return g.permute(0, 2, 1, 3, 4, 5).reshape(N * To, C * kt, H, W)

    def fold_out(self, y: torch.Tensor, N: int, one_d: bool) -> torch.Tensor:
        """The 2D conv's frame output back to the conv's logical output layout."""
        out = video_of(y, N)
        return out[:, :, :, 0, 0] if one_d else out

    def frames_like_out(self, r: torch.Tensor) -> torch.Tensor:
        """A tensor of the conv's output shape (a residual) as output frames."""
        return frames_of(r[:, :, :, None, None] if r.dim() == 3 else r)


def temporal_unfold(x5: torch.Tensor, kt: int, st: int, pt: int, dt: int, To: int) -> torch.Tensor:
    """[N, C, T, H, W] (any layout; channels_last_3d is free) -> frames [N*To, C*kt, H, W]
    (channels_last) on the native unfold kernel."""
    from . import _lib
    N, C, T, H, W = x5.shape
    xm = x5.permute(0, 2, 3, 4, 1)
    if xm.dtype != torch.bfloat16:
        xm = xm.to(torch.bfloat16)
    xm = xm.contiguous()
    out = torch.empty(N * To, H, W, C * kt, device=x5.device, dtype=torch.bfloat16)
    _lib.call('mlc_temporal_unfold', _lib.ptr(xm), _lib.ptr(out), N, T, H * W, C, kt, st, pt, dt, To, _lib.stream())
    return out.permute(0, 3, 1, 2)


def temporal_fold(dcol: torch.Tensor, N: int, C: int, T: int, H: int, W: int, kt: int, st: int, pt: int, dt: int,
                  To: int, addend: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gradient of :func:`temporal_unfold`: frames-gradient [N*To, C*kt, H, W] -> [N, C, T, H, W]
    (channels_last_3d), a gather over the taps (no atomics); ``addend`` (any tensor whose
    memory is the contiguous [N, T, H, W, C] bf16 gradient of the same activation, see
    :func:`_nthwc`) is summed in the same pass."""
    from . import _lib
    dm = dcol.permute(0, 2, 3, 1)
    if dm.dtype != torch.bfloat16:
        dm = dm.to(torch.bfloat16)
    dm = dm.contiguous()
    add = _nthwc(addend, N, C, T, H, W) if addend is not None else None
    dx = torch.empty(N, T, H, W, C, device=dcol.device, dtype=torch.bfloat16)
    _lib.call('mlc_temporal_fold', _lib.ptr(dm), _lib.ptr(add), _lib.ptr(dx), N, T, H * W, C, kt, st, pt, dt, To,
              _lib.stream())
    return dx.permute(0, 4, 1, 2, 3)


def _nthwc(g: torch.Tensor, N: int, C: int, T: int, H: int, W: int) -> torch.Tensor:
    """A hand-off gradient as the contiguous bf16 [N, T, H, W, C] tensor: either a site's NHWC
    frame gradient [N*T, H, W, C] or a logical [N, C, T, H, W] (channels_last_3d) one."""
    if g.dim() == 4:
        assert tuple(g.shape) == (N * T, H, W, C), (tuple(g.shape), (N, C, T, H, W))
        g = g.reshape(N, T, H, W, C)
    else:
        assert tuple(g.shape) == (N, C, T, H, W), (tuple(g.shape), (N, C, T, H, W))
        g = g.permute(0, 2, 3, 4, 1)
    return g.to(torch.bfloat16).contiguous()


def _link_grad(link: 'Frames', dx: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """Receiver / sender side of a Frames gradient hand-off around the input gradient ``dx``
    of the site's 5D input (None when the caller already summed the pending addend)."""
    if link.send_to is not None:
        object.__setattr__(link.send_to, '_pending', dx)     # summed by the sibling's fold
        return None
    return dx


def _take_pending(link: Optional['Frames']):
    if link is None:
        return None
    add = link._pending
    object.__setattr__(link, '_pending', None)
    if link.grad_expected and add is None:
        raise RuntimeError(f'{link.name}: the gradient hand-off of the other branch did not arrive '
                           '(backward order differs from the one the lowering assumed)')
    return add


class _TemporalUnfold(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kt, st, pt, dt, To, link=None):
        ctx.geom = (tuple(x.shape), kt, st, pt, dt, To, x.dtype)
        ctx.link = link
        return temporal_unfold(x, kt, st, pt, dt, To)

    @staticmethod
    def backward(ctx, g):
        (N, C, T, H, W), kt, st, pt, dt, To, dtype = ctx.geom
        link = ctx.link
        dx = temporal_fold(g, N, C, T, H, W, kt, st, pt, dt, To, addend=_take_pending(link)).to(dtype)
        if link is not None:
            dx = _link_grad(link, dx)
        return dx, None, None, None, None, None, None


class _GradLink(torch.autograd.Function):
    """Identity on a Frames site's 5D input whose backward does the site's gradient hand-off
    with one add (the CPU path and the unfold-free frame views; the native unfold does it in
    its fold kernel)."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        add = _take_pending(link)
        if add is not None:
            N, C, T, H, W = g.shape
            a = add.reshape(N, T, H, W, C).permute(0, 4, 1, 2, 3) if add.dim() == 4 else add
            g = g + a.to(g.dtype)
        return _link_grad(link, g), None


class TemporalAs2d:
    """A purely temporal nn.Conv3d - kernel (kt, 1, 1), stride 1, padding (pt, 0, 0), no
    dilation, groups 1 (R(2+1)D's temporal convs) - as the 2D conv with kernel (kt, 1) and
    padding (pt, 0) over the [N, T, H*W, C] image: a channels_last_3d activation already IS
    that image, so unlike the frame unfold (:class:`Conv3dAs2d`, kt copies of the input)
    there is no copy in either direction."""

    def __init__(self, m: nn.Module):
        kt = m.kernel_size[0]
        self.src3d = m
        self.kernel_size = (kt, 1)
        self.stride, self.padding, self.dilation = (1, 1), (m.padding[0], 0), (1, 1)
        self.groups = 1
        self.padding_mode = m.padding_mode
        self.in_channels, self.out_channels = m.in_channels, m.out_channels
        self.bias = m.bias
        self._shape = (m.weight.shape[0], m.weight.shape[1], kt, 1)
        self._hw = None

    @staticmethod
    def applies(m: nn.Module) -> bool:
        return (isinstance(m, nn.Conv3d) and tuple(m.kernel_size[1:]) == (1, 1) and tuple(m.stride) == (1, 1, 1)
                and tuple(m.padding[1:]) == (0, 0) and tuple(m.dilation) == (1, 1, 1) and m.groups == 1
                and not isinstance(m.padding, str))

    @property
    def weight(self):
        return self.src3d.weight.view(self._shape)

    def unfold(self, x: torch.Tensor) -> torch.Tensor:
        self._hw = x.shape[3:]
        return x.flatten(3)                  # [N, C, T, H*W], channels_last strides: a view

    def fold_out(self, y: torch.Tensor, N: int, one_d: bool) -> torch.Tensor:
        return y.unflatten(3, tuple(self._hw))

    def frames_like_out(self, r: torch.Tensor) -> torch.Tensor:
        return r.flatten(3)


class Frames(nn.Module):
    """Runs a 2D site over the frames of a 5D (or, for Conv1d, 3D) tensor: temporal unfold
    (convs), the site on N*T frames, the result back in the caller's layout."""

    def __init__(self, site: nn.Module, conv: Optional[Conv3dAs2d] = None, name: str = ''):
        super().__init__()
        self.site = site
        self._conv = conv
        self.name = name
        # gradient hand-offs around this site's temporal unfold (set by the lowering,
        # native_generic._Lowering._link_frames): ``grad_expected`` - another branch's gradient of the
        # input arrives in ``_pending`` (a residual block's identity path, handed over by the
        # block's last site, or the shortcut conv's input gradient) and the fold kernel sums
        # it; ``send_to`` - this site's input gradient is handed to that sibling site
        # instead of being returned to autograd (which would add the two in a pass of its own)
        object.__setattr__(self, '_pending', None)
        object.__setattr__(self, 'grad_expected', False)
        object.__setattr__(self, 'send_to', None)

    def forward(self, x, res=None):
        c = self._conv
        if c is not None:
            link = self if (self.grad_expected or self.send_to is not None) else None
            xf = c.unfold(x, link) if link is not None else c.unfold(x)
            rf = c.frames_like_out(res) if res is not None else None
            y = self.site(xf, rf) if rf is not None else self.site(xf)
            return c.fold_out(y, x.shape[0], x.dim() == 3)
        xf = frames_of(x)
        y = self.site(xf)
        return video_of(y, x.shape[0])


class _Uses:
    """Counts the forward calls of a parameter set in a step; backward marks its slots ready
    only after the last of them (weight sharing across call sites)."""

    def __init__(self):
        self.pending = 0

    def fwd(self):
        self.pending += 1

    def bwd_done(self) -> bool:
        self.pending -= 1
        return self.pending <= 0


# ---------------------------------------------------------------------------- parameters
class ConvParams:
    """nn.Conv2d -> kernel-layout slots: dense [Cop, KH, KW, Cip], grouped [Co, KH, KW, Cg],
    depthwise [KH, KW, Cp] (tap-major); nn.ConvTranspose2d -> 'tr' [Cip, KH, KW, Cop] (the
    filter of the conv whose input gradient the transposed conv is); optional bias [Cop]."""

    @staticmethod
    def s2d_ok(conv: nn.Module) -> bool:
        """A 7x7/2 pad-3 conv over <= 3 channels (an image stem): it can run as a 4x4/1 conv
        over the 2x2 space-to-depth image (kind 's2d', as the hand ResNet engine's stem)."""
        return (type(conv) is nn.Conv2d and conv.groups == 1 and conv.in_channels <= 3
                and tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2)
                and tuple(conv.padding) == (3, 3) and tuple(conv.dilation) == (1, 1))

    def __init__(self, ctx: NativeContext, name: str, conv: nn.Module, keep_bias: bool, s2d: bool = False):
        self.ctx, self.name, self.src = ctx, name, conv
        self.groups = conv.groups
        self.stride, self.pad, self.dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        if s2d:
            # the image stem as a 4x4/1 conv over the space-to-depth image (K = 256, and the
            # persistent stem kernel for 64 channels, csrc/kernels/stemconv.hip); its input is
            # the graph input.  Filter [Cop, 4, 4, 16]: the 7x7
            # filter zero-extended to 8x8 and regrouped (Fn.stem_w_to_s2d); the extension taps
            # and the 4 pad channels are masked out of every weight gradient
            assert ConvParams.s2d_ok(conv)
            Co = conv.out_channels
            self.kind = 's2d'
            self.Ci, self.Co, self.Cg = conv.in_channels, Co, conv.in_channels
            self.k = (7, 7)
            self.wt_idx = None
            self.Cip, self.Cop = ceil8(self.Ci), ceil8(Co)
            self.w = ctx.arena.weight(f'{name}.weight', (self.Cop, 4, 4, 16))
            self.b = ctx.arena.vector(f'{name}.bias', (self.Cop,)) if (keep_bias and conv.bias is not None) else None
            _freeze(self.w, conv.weight)
            _freeze(self.b, conv.bias)
            self.uses = _Uses()
            return
        if not isinstance(conv, nn.ConvTranspose2d) and conv.groups == 1 and conv.padding[0] != conv.padding[1]:
            self.pad = (conv.padding[0], conv.padding[1])   # per-axis (dense convs: Inception's 1x7 / 7x1)
        if isinstance(conv, nn.ConvTranspose2d):
            Ci, Co, KH, KW = conv.weight.shape
            self.kind = 'tr'
            self.Ci, self.Co, self.Cg = Ci, Co, Ci
            self.k = (KH, KW)
            self.out_pad = conv.output_padding[0]
            self.Cip, self.Cop = ceil8(Ci), ceil8(Co)
            self.w = ctx.arena.weight(f'{name}.weight', (self.Cip, KH, KW, self.Cop))
            self.b = ctx.arena.vector(f'{name}.bias', (self.Cop,)) if (keep_bias and conv.bias is not None) else None
            _freeze(self.w, conv.weight)
            _freeze(self.b, conv.bias)
            self.uses = _Uses()
            return
        Co, Cg, KH, KW = conv.weight.shape
        self.Ci, self.Co, self.Cg = Cg * conv.groups, Co, Cg
        self.k = (KH, KW)
        self.wt_idx = None
        if self.groups == 1:
            self.kind = 'dense'
            self.Cip, self.Cop = ceil8(self.Ci), ceil8(Co)
            self.w = ctx.arena.weight(f'{name}.weight', (self.Cop, KH, KW, self.Cip))
            if ctx.wt is not None:
                # the transposed, flipped filter copy (one batched refresh per training step,
                # GenericNet.__call__): the dgrad GEMM reads both operands K-contiguous (per-axis
                # pads too: Inception's 1x7 / 7x1 convs)
                self.wt_idx = ctx.wt.add(self.w)
        elif self.groups == self.Ci and Co == self.Ci:
            self.kind = 'dw'
            self.Cip = self.Cop = ceil8(Co)
            self.w = ctx.arena.weight(f'{name}.weight', (KH, KW, self.Cop))
        else:
            self.kind = 'grouped'
            self.Cip, self.Cop = self.Ci, Co
            self.w = ctx.arena.weight(f'{name}.weight', (Co, KH, KW, Cg))
        self.b = ctx.arena.vector(f'{name}.bias', (self.Cop,)) if (keep_bias and conv.bias is not None) else None
        _freeze(self.w, conv.weight)
        _freeze(self.b, conv.bias)
        self.uses = _Uses()

    def load_from_torch(self):
        w = self.src.weight.detach().float()
        dev = self.ctx.device
        if self.kind == 's2d':
            w = torch.nn.functional.pad(Fn.stem_w_to_s2d(w.cpu()), (0, 0, 0, 0, 0, 0, 0, self.Cop - self.Co))
            ones = torch.ones(self.Cop, self.Ci, 7, 7)
            self._gmask = (Fn.stem_w_to_s2d(ones) != 0).float().to(dev)
        elif self.kind == 'dense':
            w = w.permute(0, 2, 3, 1)
            w = torch.nn.functional.pad(w, (0, self.Cip - self.Ci, 0, 0, 0, 0, 0, self.Cop - self.Co))
        elif self.kind == 'tr':
            w = w.permute(0, 2, 3, 1)
            w = torch.nn.functional.pad(w, (0, self.Cop - self.Co, 0, 0, 0, 0, 0, self.Cip - self.Ci))
        elif self.kind == 'dw':
            w = torch.nn.functional.pad(w[:, 0].permute(1, 2, 0), (0, self.Cop - self.Co))
        else:
            w = w.permute(0, 2, 3, 1)
        self.w.master.copy_(w.to(dev))
        if self.b is not None:
            self.b.master.zero_()
            self.b.master[:self.Co].copy_(self.src.bias.detach().float().to(dev))

    def export_to_torch(self):
        m = self.w.master.detach()
        if self.kind == 's2d':
            w = Fn.stem_w_from_s2d(m[:self.Co].float().cpu(), self.Ci)
        elif self.kind == 'dense':
            w = m[:self.Co, :, :, :self.Ci].permute(0, 3, 1, 2)
        elif self.kind == 'tr':
            w = m[:self.Ci, :, :, :self.Co].permute(0, 3, 1, 2)
        elif self.kind == 'dw':
            w = m[..., :self.Co].permute(2, 0, 1)[:, None]
        else:
            w = m.permute(0, 3, 1, 2)
        self.src.weight.data.copy_(w.to(self.src.weight.device, self.src.weight.dtype))
        if self.b is not None:
            self.src.bias.data.copy_(self.b.master[:self.Co].to(self.src.bias.device, self.src.bias.dtype))

    def out_hw(self, H, W):
        if self.kind == 'tr':
            KH, KW = self.k
            s, p, d, op = self.stride, self.pad, self.dil, self.out_pad
            return (H - 1) * s - 2 * p + d * (KH - 1) + op + 1, (W - 1) * s - 2 * p + d * (KW - 1) + op + 1
        return Fn.conv_out_hw(H, W, self.k[0], self.k[1], self.stride, self.pad, self.dil)

    # ---- the three GEMMs by kind
    def fwd(self, x, stats=None, act=0, out=None):
        """x: NHWC bf16 with Cip channels -> y [N, Ho, Wo, Cop] (bias and a ReLU act fused for
        dense convs without BN: ``act`` 3).  ``out``: where a plain dense conv writes y (the
        channel slice of a DenseNet block's concat buffer)."""
        wb = self.w.bf16
        if self.kind == 's2d':       # x: the s2d image (s2d_input)
            if self.b is not None or act:
                assert stats is None
                return Fn.conv2d_fwd_ex(x, wb, self.b.master if self.b is not None else None, act, 1, 0, 1)
            return Fn.stem_conv_fwd(x, wb, stats=stats)
        if self.kind == 'dense':
            if self.b is not None or act:
                assert stats is None
                return Fn.conv2d_fwd_ex(x, wb, self.b.master if self.b is not None else None, act, self.stride,
                                        self.pad, self.dil)
            return Fn.conv2d_fwd(x, wb, self.stride, self.pad, self.dil, stats=stats, out=out)
        assert out is None
        if self.kind == 'dw':
            return Fn.dwconv_fwd(x, wb, self.stride, self.pad, self.dil, stats=stats)
        if self.kind == 'tr':     # the dgrad parity-class GEMMs (BN statistics in the epilogue)
            return Fn.conv_transpose2d_fwd(x, wb, self.out_hw(x.shape[1], x.shape[2]), self.stride, self.pad,
                                           self.dil, stats=stats)
        return Fn.gconv_fwd(x, wb, self.groups, self.stride, self.pad, self.dil, stats=stats)

    def dgrad(self, dy, x_shape, addend=None, bn=None):
        """Input gradient (+ ``addend``: another branch's gradient of the same input, summed
        in the dense GEMM's epilogue; ``bn``: the producing site's BatchNorm-backward
        reduction and ReLU mask in the same epilogue, dense convs only)."""
        wb = self.w.bf16
        if self.kind == 's2d':
            # rare (an input that requires grad): the s2d image's gradient, mapped back
            assert bn is None
            dxs = Fn.conv2d_dgrad(dy, wb, x_shape, 1, 0, 1)
            H, W = self._in_hw
            dx = Fn.stem_s2d_to_nhwc(dxs, 3)[:, :H, :W]
            dx = torch.nn.functional.pad(dx, (0, self.Cip - dx.shape[-1])).to(torch.bfloat16).contiguous()
            return dx if addend is None else dx.add_(addend)
        if self.kind == 'dense':
            wt = self.ctx.wt[self.wt_idx] if self.wt_idx is not None else None
            return Fn.conv2d_dgrad(dy, wb, x_shape, self.stride, self.pad, self.dil, addend=addend, bn=bn, wt=wt)
        assert bn is None
        if self.kind == 'dw':
            dx = Fn.dwconv_dgrad(dy, wb, x_shape, self.stride, self.pad, self.dil)
        elif self.kind == 'tr':     # a forward conv of dy over the same filter
            dx = Fn.conv2d_fwd(dy, wb, self.stride, self.pad, self.dil)
            assert tuple(dx.shape) == tuple(x_shape), (dx.shape, x_shape)
        else:
            dx = Fn.gconv_dgrad(dy, wb, x_shape, self.groups, self.stride, self.pad, self.dil)
        return dx if addend is None else dx.add_(addend)

    def s2d_input(self, xn):
        """[N, H, W, Cip] image -> the [N, (H+6)/2, (W+6)/2, 16] space-to-depth image of its
        pad-3 version (an odd H / W gets one zero row / column first: same output)."""
        H, W = xn.shape[1], xn.shape[2]
        self._in_hw = (H, W)                  # for an input gradient (dgrad)
        if H % 2 or W % 2:
            xn = torch.nn.functional.pad(xn, (0, 0, 0, W % 2, 0, H % 2))
        return Fn.stem_s2d(xn, 3)

    def wgrad(self, dy, x):
        acc = self.ctx.grad_prezeroed
        if self.kind == 's2d':
            if self.b is not None:
                Fn.conv2d_wgrad_bias(dy, x, self.w.shape, self.b.grad, 1, 0, 1, out=self.w.grad, accumulate=acc,
                                     slab=self.ctx.wgrad_slab)
            else:
                Fn.conv2d_wgrad(dy, x, self.w.shape, 1, 0, 1, out=self.w.grad, accumulate=acc, slab=self.ctx.wgrad_slab)
            self.w.grad.mul_(self._gmask)
            return
        if self.kind == 'dense':
            if self.b is not None:
                Fn.conv2d_wgrad_bias(dy, x, self.w.shape, self.b.grad, self.stride, self.pad, self.dil,
                                     out=self.w.grad, accumulate=acc, slab=self.ctx.wgrad_slab)
            else:
                Fn.conv2d_wgrad(dy, x, self.w.shape, self.stride, self.pad, self.dil, out=self.w.grad,
                                accumulate=acc, slab=self.ctx.wgrad_slab)
        elif self.kind == 'dw':
            Fn.dwconv_wgrad(dy, x, self.w.shape, self.stride, self.pad, self.dil, out=self.w.grad, accumulate=acc)
        elif self.kind == 'tr':   # the conv wgrad with the roles of x and dy swapped
            Fn.conv2d_wgrad(x, dy, self.w.shape, self.stride, self.pad, self.dil, out=self.w.grad, accumulate=acc,
                            slab=self.ctx.wgrad_slab)
        else:
            Fn.gconv_wgrad(dy, x, self.w.shape, self.groups, self.stride, self.pad, self.dil, out=self.w.grad,
                           accumulate=acc)

    def mark_ready(self):
        self.ctx.arena.mark_ready(self.w)
        if self.b is not None:
            self.ctx.arena.mark_ready(self.b)


def _freeze(slot, param, force=False):
    """A parameter the user froze (``requires_grad=False``: a fine-tuned backbone, the
    reference model executor's frozen layers) keeps its value: its arena slot is marked
    frozen, which the fused optimizers honour (no update, no weight decay), as torch.optim
    skips a parameter whose grad is None."""
    if slot is not None and (force or (param is not None and not param.requires_grad)):
        slot.frozen = True


class BNParams:
    """nn.BatchNorm2d / BatchNorm1d -> gamma / beta slots [Cp] + running statistics."""

    def __init__(self, ctx: NativeContext, name: str, bn: nn.modules.batchnorm._BatchNorm):
        self.ctx, self.name, self.src = ctx, name, bn
        self.C = bn.num_features
        self.Cp = ceil8(self.C)
        self.eps = bn.eps
        self.momentum = bn.momentum
        self.affine = bn.affine
        self.track = bn.track_running_stats
        self.gamma = ctx.arena.vector(f'{name}.weight', (self.Cp,))
        self.beta = ctx.arena.vector(f'{name}.bias', (self.Cp,))
        # affine=False: gamma = 1 / beta = 0 stay constants (the slots exist so the kernels
        # have something to read, but the optimizer never moves or decays them)
        _freeze(self.gamma, bn.weight if self.affine else None, force=not self.affine)
        _freeze(self.beta, bn.bias if self.affine else None, force=not self.affine)
        self.run_mean = self.run_var = None
        self.uses = _Uses()

    def load_from_torch(self):
        dev = self.ctx.device
        bn = self.src
        self.gamma.master.zero_()
        self.beta.master.zero_()
        self.gamma.master[:self.C].copy_(bn.weight.detach().float().to(dev) if self.affine else torch.ones(self.C))
        self.beta.master[:self.C].copy_(bn.bias.detach().float().to(dev) if self.affine else torch.zeros(self.C))
        if self.track:
            self.run_mean = torch.zeros(self.Cp, device=dev)
            self.run_var = torch.ones(self.Cp, device=dev)
            self.run_mean[:self.C].copy_(bn.running_mean.detach().float())
            self.run_var[:self.C].copy_(bn.running_var.detach().float())
            cb = getattr(self, 'conv_bias', None)
            if cb is not None:
                # the fused conv drops its bias (a batch-statistics BN cancels it), so the
                # running mean is kept bias-free and converted here and on export
                self.run_mean[:self.C].sub_(cb.detach().float().to(dev))

    def export_to_torch(self):
        bn = self.src
        if self.affine:
            bn.weight.data.copy_(self.gamma.master[:self.C].to(bn.weight.device, bn.weight.dtype))
            bn.bias.data.copy_(self.beta.master[:self.C].to(bn.bias.device, bn.bias.dtype))
        if self.track:
            rm = self.run_mean[:self.C]
            cb = getattr(self, 'conv_bias', None)
            if cb is not None:
                rm = rm + cb.detach().float().to(rm.device)
            bn.running_mean.copy_(rm.to(bn.running_mean.device))
            bn.running_var.copy_(self.run_var[:self.C].to(bn.running_var.device))
            if bn.num_batches_tracked is not None:
                bn.num_batches_tracked.add_(int(getattr(self, 'batches', 0)))
            self.batches = 0

    def batch_stats(self) -> bool:
        return self.ctx.training or not self.track

    def finalize(self, s1, s2, rows):
        """(scale, shift, mean, invstd) of this call - batch statistics (training) or the
        running ones (inference)."""
        dev = s1.device if s1 is not None else self.gamma.master.device
        st = torch.empty(4, self.Cp, device=dev, dtype=torch.float32)
        scale, shift, mean, inv = st[0], st[1], st[2], st[3]
        if self.batch_stats():
            upd = self.ctx.training and self.track
            mom = self.momentum if self.momentum is not None else 0.1
            Fn.bn_finalize(s1, s2, rows, self.gamma.master, self.beta.master, mean, inv, scale, shift,
                           self.run_mean if upd else None, self.run_var if upd else None, self.eps, mom)
            if upd:
                self.batches = getattr(self, 'batches', 0) + 1
        else:
            torch.rsqrt(self.run_var + self.eps, out=inv)
            torch.mul(inv, self.gamma.master, out=scale)
            torch.sub(self.beta.master, self.run_mean * scale, out=shift)
            mean.copy_(self.run_mean)
        return scale, shift, mean, inv

    def finalize_apply(self, s1, s2, y, res, act, alpha, res_affine=None, row_scale=None, prev_tot=None, prev_c=0,
                       tot_out=None):
        """:meth:`finalize` and the apply pass in one launch (Fn.bnact_fused) for batch
        statistics: (z, scale, shift, mean, invstd), or None when it does not apply."""
        if s1 is None or not self.batch_stats():
            return None
        st = torch.empty(4, self.Cp, device=s1.device, dtype=torch.float32)
        scale, shift, mean, inv = st[0], st[1], st[2], st[3]
        upd = self.ctx.training and self.track
        mom = self.momentum if self.momentum is not None else 0.1
        z = Fn.bnact_fused(y, res, s1, s2, self.gamma.master, self.beta.master, mean, inv, scale, shift,
                           self.run_mean if upd else None, self.run_var if upd else None, self.eps, mom, act, alpha,
                           res_affine=res_affine, row_scale=row_scale, prev_tot=prev_tot, prev_c=prev_c,
                           tot_out=tot_out)
        if z is None:
            return None
        if upd:
            self.batches = getattr(self, 'batches', 0) + 1
        return z, scale, shift, mean, inv

    def mark_ready(self):
        self.ctx.arena.mark_ready(self.gamma)
        self.ctx.arena.mark_ready(self.beta)


class LinearParams:
    """nn.Linear -> weight [Op, Ip] (decay arena, bf16 mirror) and bias [Op]."""

    def __init__(self, ctx: NativeContext, name: str, lin: nn.Linear):
        self.ctx, self.name, self.src = ctx, name, lin
        self.O, self.I = lin.weight.shape
        self.Op, self.Ip = ceil8(self.O), ceil8(self.I)
        self.w = ctx.arena.weight(f'{name}.weight', (self.Op, self.Ip))
        self.b = ctx.arena.vector(f'{name}.bias', (self.Op,)) if lin.bias is not None else None
        _freeze(self.w, lin.weight)
        _freeze(self.b, lin.bias)
        self.uses = _Uses()

    def load_from_torch(self):
        dev = self.ctx.device
        self.w.master.zero_()
        self.w.master[:self.O, :self.I].copy_(self.src.weight.detach().float().to(dev))
        if self.b is not None:
            self.b.master.zero_()
            self.b.master[:self.O].copy_(self.src.bias.detach().float().to(dev))

    def export_to_torch(self):
        lin = self.src
        lin.weight.data.copy_(self.w.master[:self.O, :self.I].to(lin.weight.device, lin.weight.dtype))
        if self.b is not None:
            lin.bias.data.copy_(self.b.master[:self.O].to(lin.bias.device, lin.bias.dtype))

    def mark_ready(self):
        self.ctx.arena.mark_ready(self.w)
        if self.b is not None:
            self.ctx.arena.mark_ready(self.b)


# ---------------------------------------------------------------------------- sites
class GradAcc:
    """One activation's input gradient summed across its N consumer sites in their own
    backward kernels, in whatever order autograd runs them (set by the lowering,
    ``_link_fanout``: an Inception block input feeding three convs and an average pool).
    Each consumer's backward passes the running sum as its kernel's addend (dgrad epilogue
    / pool-backward) and hands its output on; the last one returns the total to autograd,
    the others return no gradient - instead of autograd adding N gradients in N - 1 passes.
    ``left`` counts the consumers' gradient-tracking forwards of this step."""

    def __init__(self, name: str):
        self.name, self.left, self.buf = name, 0, None

    def enter(self, x):
        if torch.is_grad_enabled() and isinstance(x, torch.Tensor) and x.requires_grad:
            self.left += 1

    def give(self, dx):
        self.left -= 1
        if self.left <= 0:
            self.left, self.buf = 0, None
            return dx
        self.buf = dx
        return None


class Site(nn.Module):
    """A lowered call site: forward() runs the site's autograd Function.  Holds no
    nn.Parameters (the arena owns the weights)."""

    def __init__(self, ctx: NativeContext):
        super().__init__()
        object.__setattr__(self, 'ctx', ctx)   # not a submodule / not in state_dict
        object.__setattr__(self, 'acc', None)  # a GradAcc over its first input (the lowering)

    def _direct_bn_grads(self) -> bool:
        return bool(getattr(self.bn, 'single_site', False)) and bool(getattr(self.ctx, 'grad_prezeroed', False))

    def params(self):
        """The parameter sets this site reads (their use counts gate mark_ready)."""
        return [p for p in (getattr(self, 'conv', None), getattr(self, 'bn', None), getattr(self, 'lin', None))
                if p is not None]


class _SiteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, site, *inputs):
        for p in site.params():
            p.uses.fwd()
        out, saved, keep = site.fwd(*inputs)
        ctx.site = site
        ctx.keep = keep
        ctx.n_in = len(inputs)
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        grads = ctx.site.bwd(dout, ctx.saved_tensors, ctx.keep, [ctx.needs_input_grad[2 + i] for i in range(ctx.n_in)])
        return (None, None) + tuple(grads)


def _run(site, *inputs):
    anchor = site.ctx.anchor
    if torch.is_grad_enabled() and site.ctx.training:
        if site.acc is not None:      # counted out here: inside Function.forward grad mode is off
            site.acc.enter(inputs[0])
        return _SiteFn.apply(anchor, site, *inputs)
    with torch.no_grad():
        return site.fwd(*inputs)[0]


class ConvBNAct(Site):
    """conv [-> BN (batch stats in training)] [+ residual] [-> activation].  Without BN a
    dense conv fuses its bias (and a ReLU) into the GEMM epilogue; grouped / depthwise convs
    without BN add the bias with a torch op (rare)."""

    def __init__(self, ctx, conv: ConvParams, bn: Optional[BNParams], act: int = 0, alpha: float = 0.0,
                 residual: bool = False):
        super().__init__(ctx)
        object.__setattr__(self, 'conv', conv)
        object.__setattr__(self, 'bn', bn)
        self.act, self.alpha, self.residual = act, alpha, residual
        if bn is not None:
            assert bn.Cp == conv.Cop, (bn.C, conv.Co)
        # conv epilogue fusion for BN-less dense convs: bias and ReLU
        self.epi_act = 3 if (bn is None and conv.kind == 'dense' and act == 1 and not residual) else 0
        self.k_st = ctx.ws.request(f'{conv.name}@{id(self)}.st', 2 * Fn.NSTAT * conv.Cop) if bn is not None else None
        self.k_bw = ctx.ws.request(f'{conv.name}@{id(self)}.bw', 2 * Fn.NSTAT * conv.Cop) if bn is not None else None
        # identity-residual link (set by the lowering): this site's residual input is also
        # exactly one other site's conv input, and that site's backward runs later, so the
        # residual gradient is handed over and summed in that site's dgrad epilogue instead
        # of autograd adding the two branch gradients in a pass of its own
        object.__setattr__(self, 'res_link', None)
        object.__setattr__(self, '_pending', None)
        # BN-backward link (set by the lowering): ``bn_link`` is the site whose output is this
        # (dense) conv's only input; this site's dgrad epilogue applies that site's ReLU mask
        # and accumulates its BatchNorm-backward sums, so its backward skips the reduction
        # pass (``bn_prereduced``; the hand engines' BnBwdSpec, across fx sites)
        object.__setattr__(self, 'bn_link', None)
        object.__setattr__(self, 'bn_prereduced', False)
        object.__setattr__(self, '_bn_stash', None)
        object.__setattr__(self, '_bn_done', False)
        # input-gradient hand-off (set by the lowering): this site's input is also the input of
        # ``grad_link``, a dense conv site whose backward runs after this one's (a block's
        # first conv beside its downsample shortcut), so this site's input gradient is summed
        # in that site's dgrad epilogue instead of by autograd; ``grad_expected`` marks the
        # receiving site, which fails loudly if the hand-off did not arrive
        object.__setattr__(self, 'grad_link', None)
        object.__setattr__(self, 'grad_expected', False)
        # folded shortcut BatchNorm (set by the lowering): ``res_bn`` is the conv+BN site (no
        # activation) whose output is only this site's residual; it returns its pre-BN conv
        # output (``bn_folded``) and this site applies its BN as the residual's affine in its
        # own apply pass (the hand engine's downsample fold), so that BN costs no pass of its
        # own; the residual gradient this site returns is the gradient of that BN's output
        object.__setattr__(self, 'res_bn', None)
        object.__setattr__(self, 'bn_folded', False)
        object.__setattr__(self, '_fold', None)
        # fused 3x3/2 max-pool (set by the lowering): conv -> BN -> ReLU -> max-pool with the
        # activation used only by the pool (a ResNet stem) runs BN-apply + ReLU + pool in one
        # pass and its backward as pool-scatter + BN-backward passes (stem.hip); the full-
        # resolution activation is never written
        object.__setattr__(self, 'pool3', False)
        # stochastic depth folded in (set by the lowering): the BN output is multiplied by a
        # per-sample drop-path factor mask / drop_keep before the residual add (EfficientNet's
        # MBConv in training), in the same apply pass; the third input is the [N,1,1,1] mask
        object.__setattr__(self, 'drop_keep', None)
        # concat-buffer output (set by the lowering, _chain_dense_cats): this BN-less dense conv's
        # output is the new segment of a chained DenseCat, so it is written straight into the
        # block's concat buffer (channels [off, off + Co), rows of the buffer's width)
        object.__setattr__(self, 'cat_out', None)

    def _cat_slot(self, xn):
        dc = self.cat_out
        c = self.conv
        if dc is None or dc.chain is None or not xn.is_cuda:
            return None
        _, KH, KW, _ = c.w.bf16.shape
        Ho, Wo = Fn.conv_out_hw(xn.shape[1], xn.shape[2], KH, KW, c.stride, c.pad, c.dil)
        ch, N = dc.chain, xn.shape[0]
        buf = ch.buf
        if dc.chain_first or buf is None or tuple(buf.shape[:3]) != (N, Ho, Wo) or buf.device != xn.device:
            buf = ch.fresh(N, Ho, Wo, xn.device)
        return buf[..., dc.off:dc.off + c.Co]

    def forward(self, x, res=None, mask=None):
        if mask is not None:
            return _run(self, x, res, mask)
        return _run(self, x, res) if res is not None else _run(self, x)

    def fwd(self, x, res=None, mask=None):
        c, bn = self.conv, self.bn
        xn = to_nhwc(x, c.Cip)
        if c.kind == 's2d':
            xn = c.s2d_input(xn)              # saved for the weight gradient as well
        rn = to_nhwc(res, c.Cop) if res is not None else None
        if bn is not None:
            stats = None
            if bn.batch_stats():
                st = self.ctx.ws[self.k_st]
                n = Fn.NSTAT * c.Cop
                stats = (st[:n], st[n:])
            y = c.fwd(xn, stats)
            rows = y.numel() // y.shape[-1]
            rsh = None
            rsc = mask.reshape(-1).float() / self.drop_keep if mask is not None else None
            if not self.pool3 and not self.bn_folded and stats is not None:
                # one launch: finalize folded into the apply pass (Fn.BN_FUSED)
                if self.res_bn is not None and rn is not None:
                    rsh = self.res_bn._fold
                fused = bn.finalize_apply(stats[0], stats[1], y, rn, self.act, self.alpha, res_affine=rsh,
                                          row_scale=rsc)
                if fused is not None:
                    if rsh is not None:
                        object.__setattr__(self.res_bn, '_fold', None)
                    z, scale, shift, mean, inv = fused
                    return self._bn_out(xn, y, z, rn, scale, shift, mean, inv, rsh, rsc, stats)
                rsh = None
            scale, shift, mean, inv = bn.finalize(stats[0] if stats else None, stats[1] if stats else None, rows)
            if self.pool3:
                out, idx = Fn.stem_pool_fwd(y, scale, shift)
                return from_nhwc(out, c.Co), [xn, y, idx, y, scale, shift, mean, inv], False
            if self.bn_folded:
                z = y                                  # the consumer applies (scale, shift)
                object.__setattr__(self, '_fold', (scale, shift))
            else:
                if self.res_bn is not None and rn is not None:
                    rsh = self.res_bn._fold
                    object.__setattr__(self.res_bn, '_fold', None)
                z = Fn.bnact_apply(y, rn, scale, shift, self.act, self.alpha, res_affine=rsh, row_scale=rsc)
            return self._bn_out(xn, y, z, rn, scale, shift, mean, inv, rsh, rsc, stats)
        out = self._cat_slot(xn) if (rn is None and not self.epi_act and not self.act) else None
        y = c.fwd(xn, None, self.epi_act, out=out)      # dense: bias (+ ReLU) in the GEMM epilogue
        if c.b is not None and c.kind != 'dense':
            y = (y.float() + c.b.master).to(torch.bfloat16)
        a = y if rn is None else (y.float() + rn.float()).to(torch.bfloat16)
        z = Fn.act_fwd(a, self.act, self.alpha) if (self.act and not self.epi_act) else a
        # saved: input, pre-activation (the ReLU output when the epilogue applied it), output
        return from_nhwc(z, c.Co), [xn, a, z], rn is not None

    def _bn_out(self, xn, y, z, rn, scale, shift, mean, inv, rsh, rsc, stats):
        saved = [xn, y, z, rn if rn is not None else y, scale, shift, mean, inv]
        if rsh is not None:
            saved += list(rsh)
        if rsc is not None:
            saved.append(rsc)
        if self.bn_prereduced and stats is not None and self.ctx.training:
            object.__setattr__(self, '_bn_stash', (y, z, mean))   # read by the linked dgrad
            object.__setattr__(self, '_bn_done', False)
        return from_nhwc(z, self.conv.Co), saved, rn is not None

    def bwd(self, dout, saved, has_res, needs):
        c, bn = self.conv, self.bn
        dz = to_nhwc(dout, c.Cop)
        dres = None
        if bn is not None:
            xn, y, z, rn, scale, shift, mean, inv = saved[:8]
            rsc = saved[-1] if (self.drop_keep is not None and len(needs) > 2) else None
            nfold = len(saved) - 8 - (1 if rsc is not None else 0)
            rsh = tuple(saved[8:10]) if nfold == 2 else None
            ws = self.ctx.ws
            d = self._direct_bn_grads()
            if self.pool3:
                # dz: the pooled output's gradient; z holds the window argmax
                dy = Fn.stem_pool_bwd(dz.contiguous(), z, y, mean, inv, bn.gamma.master, _acc_view(bn.gamma, d),
                                      _acc_view(bn.beta, d), ws[self.k_bw],
                                      torch.empty(3 * c.Cop, device=dz.device, dtype=torch.float32))
            elif self.bn_prereduced and self._bn_done:
                # the consumer's dgrad already masked dz and reduced the BN-backward sums
                object.__setattr__(self, 'n_prereduced', getattr(self, 'n_prereduced', 0) + 1)
                dy, dres = Fn.bn_bwd(dz, None, y, mean, inv, bn.gamma.master, want_dres=has_res,
                                     dgamma=_acc_view(bn.gamma, d), dbeta=_acc_view(bn.beta, d), sums=ws[self.k_bw],
                                     prereduced=True)
            else:
                dy, dres = Fn.bnact_bwd(dz, z, y, rn if has_res else None, mean, scale, shift, inv,
                                        bn.gamma.master, self.act, self.alpha, dgamma=_acc_view(bn.gamma, d),
                                        dbeta=_acc_view(bn.beta, d), sums=ws[self.k_bw], want_dres=has_res,
                                        res_affine=rsh, row_scale=rsc)
            object.__setattr__(self, '_bn_stash', None)
            object.__setattr__(self, '_bn_done', False)
            _acc_commit(bn.gamma, d)
            _acc_commit(bn.beta, d)
            if bn.uses.bwd_done():
                bn.mark_ready()
        else:
            xn, a, z = saved
            if self.epi_act:                     # ReLU applied by the GEMM: mask from z
                dy = (dz.float() * (z.float() > 0)).to(torch.bfloat16)
            elif self.act:
                dy = Fn.act_bwd(dz, a, z, self.act, self.alpha)
            else:
                dy = dz
            if has_res:
                dres = dy
            if c.b is not None and c.kind != 'dense':
                c.b.grad.add_(dy.float().sum(dim=(0, 1, 2)))
        addend = self._pending                 # another site's gradient of our input
        object.__setattr__(self, '_pending', None)
        if self.acc is not None:
            addend = self.acc.buf              # the other consumers' running sum
        if self.grad_expected and needs[0] and addend is None:
            raise RuntimeError(f'{c.name}: the input-gradient hand-off of its sibling conv site did not arrive '
                               '(backward order differs from the one the lowering assumed)')
        spec = None
        src = self.bn_link
        if src is not None and needs[0] and src._bn_stash is not None:
            ya, za, mean_a = src._bn_stash
            ys = [(ya, mean_a, self.ctx.ws[src.k_bw])]
            fold = src.res_bn
            if fold is not None and fold._bn_stash is not None:
                # the producer's folded shortcut BN shares its output gradient: both sums here
                yf, _, mean_f = fold._bn_stash
                ys.append((yf, mean_f, self.ctx.ws[fold.k_bw]))
                object.__setattr__(fold, '_bn_done', True)
            spec = Fn.BnBwdSpec(za if src.act else None, ys)
            object.__setattr__(src, '_bn_done', True)
        side = self.ctx.wgrad_stream if needs[0] else None
        main = torch.cuda.current_stream(self.ctx.device) if side is not None else None
        if side is not None and main != side:
            # the weight gradient on the context's side stream, concurrently with the input
            # gradient (as the hand engines do), joined before the site's backward returns:
            # dy / xn are freed only after that join, in the main stream's order
            # captured weight gradient first (unless ctx.dgrad_first), as the hand conv
            # engines do: the first-dispatched GEMM takes the CUs, and a squeezed-in wgrad
            # would make the join below the critical path
            fork = torch.cuda.Event()
            fork.record(main)
            if self.ctx.dgrad_first:
                dx = c.dgrad(dy, xn.shape, addend, spec)
            side.wait_event(fork)
            with Fn.side_stream(side):
                c.wgrad(dy, xn)
            if not self.ctx.dgrad_first:
                dx = c.dgrad(dy, xn.shape, addend, spec)
            if self.ctx.wgrad_defer:
                # no per-site join (NativeContext.wgrad_defer): dy / xn stay alive for the side
                # stream, the bucketer waits on it, flush_wgrad joins it before the optimizer
                dy.record_stream(side)
                xn.record_stream(side)
            else:
                main.wait_stream(side)
        else:
            c.wgrad(dy, xn)
            dx = c.dgrad(dy, xn.shape, addend, spec) if needs[0] else None
        if c.uses.bwd_done():
            c.mark_ready()
        if dx is not None and self.grad_link is not None:
            object.__setattr__(self.grad_link, '_pending', dx)       # summed by the sibling's dgrad
            dx = None
        if dx is not None and self.acc is not None:
            dx = self.acc.give(dx)
        out = [from_nhwc(dx, c.Ci) if dx is not None else None]
        if has_res:
            if needs[1] and self.res_link is not None:
                object.__setattr__(self.res_link, '_pending', dres)    # summed by the linked dgrad
                out.append(None)
            else:
                out.append(from_nhwc(dres, c.Co) if needs[1] else None)
        if len(needs) > 2:
            out.append(None)                      # the drop-path mask
        return out


def _acc_view(slot, direct=False):
    """BN dgamma / dbeta targets: the kernels overwrite, so a shared (multi-site) BN writes a
    scratch that _acc_commit adds into the grad arena; a single-site BN (``direct``) writes
    the grad arena itself (zeroed once per step, so overwrite == accumulate)."""
    if direct and slot.grad is not None:
        return slot.grad
    buf = getattr(slot, '_scratch', None)
    if buf is None or buf.device != slot.grad.device:
        buf = torch.empty_like(slot.grad)
        slot._scratch = buf
    return buf


def _acc_commit(slot, direct=False):
    if not direct:
        slot.grad.add_(slot._scratch)


class BNAct(Site):
    """A BatchNorm no conv epilogue feeds (statistics pass of its own) [+ residual] [+ act]."""

    def __init__(self, ctx, bn: BNParams, act: int = 0, alpha: float = 0.0, residual: bool = False):
        super().__init__(ctx)
        object.__setattr__(self, 'bn', bn)
        self.act, self.alpha, self.residual = act, alpha, residual
        self.k_st = ctx.ws.request(f'{bn.name}@{id(self)}.st', 2 * Fn.NSTAT * bn.Cp)
        self.k_bw = ctx.ws.request(f'{bn.name}@{id(self)}.bw', 2 * Fn.NSTAT * bn.Cp)
        # concat statistics (set by the lowering, _link_cat_stats): this BN's input is
        # cat([a, tail], 1) and ``cat_prev`` is the BN site over ``a`` (a DenseNet layer's
        # first BN; it runs earlier in the step): a's per-channel sums are copied from that
        # site's statistics and only ``tail`` (the new growth channels, passed as the second
        # input) is reduced - not the whole concatenation again
        object.__setattr__(self, 'cat_prev', None)
        object.__setattr__(self, '_last_stats', None)
        # per-channel totals [2, Cp] published by the folded-finalize apply (read by the next BN
        # of a concat chain); _tot_ok: this step's forward wrote them
        self.k_tot = ctx.ws.request(f'{bn.name}@{id(self)}.tot', 2 * bn.Cp)
        object.__setattr__(self, '_tot_ok', False)
        # concat-gradient hand-off (set by the lowering, _lower_dense_cats): this site's input
        # is also the first operand of a DenseCat whose backward runs first and leaves its
        # gradient slice here; the apply pass adds it (no copy, no autograd add)
        object.__setattr__(self, 'slice_expected', False)
        object.__setattr__(self, '_slice_pending', None)
        # split input gradient (set by the lowering, _split_cat_grads): this site's input is a
        # DenseCat's output whose gradient only this site produces; the apply pass stores it
        # as the concat's two operand gradients, each dense, handed to that DenseCat (no slice
        # copies); autograd gets a zero-stride placeholder
        object.__setattr__(self, 'split_to', None)
        object.__setattr__(self, '_ph', None)

    def forward(self, x, res=None):
        return _run(self, x, res) if res is not None else _run(self, x)

    def _stats(self, yn, tail, s1, s2, use_tot):
        """Fill the partial copies; returns (prev_tot, prev_c) when the older segment's sums are
        to come from the previous BN's published totals instead of copies (folded finalize)."""
        A = self.cat_prev
        prev = A._last_stats if A is not None else None
        if prev is None or tail is None:
            Fn.bn_stats(yn, s1, s2)
            return None, 0
        Cp, Ca = self.bn.Cp, A.bn.Cp
        tn = tail.permute(0, 2, 3, 1)
        if Fn.rows_ld(tn) is None or tn.dtype != torch.bfloat16:    # (in place in a concat buffer: no copy)
            tn = to_nhwc(tail, tail.shape[1])
        s1v, s2v = s1.view(-1, Cp), s2.view(-1, Cp)
        Fn.bn_stats(tn, s1v[:, Ca:], s2v[:, Ca:], ld=Cp)
        if use_tot and A._tot_ok:
            return self.ctx.ws[A.k_tot], Ca
        s1v[:, :Ca].copy_(prev[0].view(-1, Ca))
        s2v[:, :Ca].copy_(prev[1].view(-1, Ca))
        return None, 0

    def _placeholder(self, like):
        """A zero-stride zero tensor of ``like``'s shape: the input gradient autograd carries to
        the DenseCat that takes the real one from ``_split_pending``."""
        ph = self._ph
        if ph is None or ph.device != like.device or ph.dtype != like.dtype:
            ph = torch.zeros((), device=like.device, dtype=like.dtype)
            object.__setattr__(self, '_ph', ph)
        return ph.expand(like.shape)

    def _to(self, x, keep_rows=False):
        if keep_rows and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] == self.bn.Cp:
            y = x.permute(0, 2, 3, 1)
            if Fn.rows_ld(y) is not None:    # the leading channels of a DenseNet concat buffer: no copy
                return y
        if x.dim() == 2:              # BatchNorm1d over [N, C] / [N, C, L]
            x = x[:, :, None, None]
        elif x.dim() == 3:
            x = x[:, :, :, None]
        elif x.dim() == 5:            # BatchNorm3d: per channel over (N, T, H, W) = N*T frames
            x = frames_of(x)
        return to_nhwc(x, self.bn.Cp)

    def _from(self, z, like):
        out = from_nhwc(z, self.bn.C)
        if like.dim() == 2:
            return out[:, :, 0, 0]
        if like.dim() == 5:
            return video_of(out, like.shape[0])
        return out[..., 0] if like.dim() == 3 else out

    def fwd(self, x, res=None):
        bn = self.bn
        tail = None
        if self.cat_prev is not None:         # the second input is the concat's new segment
            tail, res = res, None
        yn = self._to(x, keep_rows=True)
        rn = self._to(res) if res is not None else None
        rows = yn.numel() // yn.shape[-1]
        stats = None
        prev_tot, prev_c = None, 0
        use_tot = yn.is_cuda and Fn._bn_fused_ok(bn.Cp, Fn.NSTAT)
        if bn.batch_stats():
            st = self.ctx.ws[self.k_st]
            n = Fn.NSTAT * bn.Cp
            stats = (st[:n], st[n:])
            prev_tot, prev_c = self._stats(yn, tail, *stats, use_tot)
        object.__setattr__(self, '_last_stats', stats)
        object.__setattr__(self, '_tot_ok', False)
        fused = bn.finalize_apply(stats[0], stats[1], yn, rn, self.act, self.alpha, prev_tot=prev_tot, prev_c=prev_c,
                                  tot_out=self.ctx.ws[self.k_tot]) if stats else None
        if prev_tot is not None and fused is None:
            raise RuntimeError(f'{bn.name}: concat statistics expected the folded-finalize path')
        if fused is not None:
            object.__setattr__(self, '_tot_ok', True)
            z, scale, shift, mean, inv = fused
        else:
            scale, shift, mean, inv = bn.finalize(stats[0] if stats else None, stats[1] if stats else None, rows)
            z = Fn.bnact_apply(yn, rn, scale, shift, self.act, self.alpha)
        self._dim = x.dim()
        return self._from(z, x), [yn, z, rn if rn is not None else yn, scale, shift, mean, inv], rn is not None

    def bwd(self, dout, saved, has_res, needs):
        bn = self.bn
        yn, z, rn, scale, shift, mean, inv = saved
        dz = self._to(dout)
        d = self._direct_bn_grads()
        addend = self._slice_pending
        object.__setattr__(self, '_slice_pending', None)
        if self.slice_expected and needs[0] and addend is None:
            raise RuntimeError(f'{bn.name}: the concat gradient hand-off did not arrive (backward order differs '
                               'from the one the lowering assumed)')
        D = self.split_to
        split = D.off if (D is not None and needs[0] and dout.dim() == 4) else None
        dy, dres = Fn.bnact_bwd(dz, z, yn, rn if has_res else None, mean, scale, shift, inv, bn.gamma.master,
                                self.act, self.alpha, dgamma=_acc_view(bn.gamma, d), dbeta=_acc_view(bn.beta, d),
                                sums=self.ctx.ws[self.k_bw], want_dres=has_res, addend=addend, split=split)
        _acc_commit(bn.gamma, d)
        _acc_commit(bn.beta, d)
        if bn.uses.bwd_done():
            bn.mark_ready()
        like = dout
        if split:
            object.__setattr__(D, '_split_pending', dy)
            out = [self._placeholder(dout)]
        else:
            out = [self._from(dy, like) if needs[0] else None]
        if has_res:
            out.append(self._from(dres, like) if needs[1] else None)
        return out + [None] * (len(needs) - len(out))      # the concat tail: statistics only


class LinearAct(Site):
    """x [..., I] -> act(x W^T + b) [+ r] on the dense GEMM (bias / ReLU / the residual add
    in the epilogue; a residual only without an activation)."""

    def __init__(self, ctx, lin: LinearParams, act: int = 0, residual: bool = False):
        super().__init__(ctx)
        object.__setattr__(self, 'lin', lin)
        self.act = act            # 0 or 3 (ReLU; the epilogue's code)
        self.residual = residual
        assert not (residual and (act or lin.Op != lin.O)), 'a fused residual needs act 0 and an unpadded output'

    def forward(self, x, r=None):
        return _run(self, x, r) if r is not None else _run(self, x)

    def fwd(self, x, r=None):
        p = self.lin
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        if p.Ip != p.I:
            x2 = torch.nn.functional.pad(x2, (0, p.Ip - p.I))
        x2 = x2.contiguous()
        B = x2.shape[0]
        r2 = None
        if r is not None:
            r2 = r.expand(*lead, p.O).reshape(B, p.O)
            if r2.dtype != torch.bfloat16:
                r2 = r2.to(torch.bfloat16)
            r2 = r2.contiguous()
        if x2.is_cuda:
            from . import _lib
            y = torch.empty(B, p.Op, device=x2.device, dtype=torch.bfloat16)
            _lib.call('mlc_gemm_bf16_ex', _lib.ptr(x2), _lib.ptr(p.w.bf16), _lib.ptr(y), B, p.Op, p.Ip, p.Ip, p.Ip,
                      p.Op, 0, 1, _lib.ptr(p.b.master if p.b is not None else None), int(self.act), None,
                      _lib.ptr(r2), None, None, 0, _lib.stream())
        else:
            yf = x2.float() @ p.w.bf16.float().t()
            if p.b is not None:
                yf = yf + p.b.master
            if self.act == 3:
                yf = yf.clamp_min(0)
            if r2 is not None:
                yf = yf + r2.float()
            y = yf.to(torch.bfloat16)
        out = y[:, :p.O] if p.Op != p.O else y
        keep = None if r is None else (tuple(r.shape), r.dtype)
        return out.reshape(*lead, p.O), [x2, y], keep

    def bwd(self, dout, saved, keep, needs):
        p = self.lin
        x2, y = saved
        d = dout.reshape(-1, p.O)
        if d.dtype != torch.bfloat16:
            d = d.to(torch.bfloat16)
        if p.Op != p.O:
            d = torch.nn.functional.pad(d, (0, p.Op - p.O))
        if self.act == 3:
            d = (d.float() * (y.float() > 0)).to(torch.bfloat16)
        d = d.contiguous()
        if p.b is not None:
            Fn.linear_wgrad_bias(d, x2, p.w.grad, p.b.grad)
        else:
            Fn.linear_wgrad(d, x2, out=p.w.grad, accumulate=True)
        dx = Fn.linear_dgrad(d, p.w.bf16) if needs[0] else None
        if p.uses.bwd_done():
            p.mark_ready()
        if dx is not None:
            if p.Ip != p.I:
                dx = dx[:, :p.I]
            dx = dx.reshape(*dout.shape[:-1], p.I)
        out = [dx]
        if keep is not None:           # the residual's gradient is the output gradient
            from .gtransformer import _reduce_to
            out.append(_reduce_to(dout, keep[0], keep[1]) if needs[1] else None)
        return out


class DenseChain:
    """The concat buffer of a run of :class:`DenseCat` sites (one DenseNet block: x_{i+1} =
    cat(x_i, b_i) for i = 0 .. L-1): one NHWC tensor of the block's final width; x_i is the view
    of its leading C_i channels (rows of stride C_L), so each layer copies only its own b_i into
    the buffer instead of the whole concatenation - the block's forward copies its channels
    once, not quadratically many times.  ``width``: C_L, set by the lowering."""

    def __init__(self, width: int):
        self.width, self.buf = width, None

    def fresh(self, N, H, W, device):
        self.buf = torch.empty(N, H, W, self.width, device=device, dtype=torch.bfloat16)
        return self.buf

    def placed(self, t, off) -> bool:
        """t (NHWC) is channels [off, off + C) of the current buffer, in place."""
        buf = self.buf
        return (buf is not None and t.shape[:3] == buf.shape[:3] and t.device == buf.device
                and t.data_ptr() == buf.data_ptr() + off * buf.element_size() and Fn.rows_ld(t) == self.width)


class DenseCat(Site):
    """``torch.cat([a, b], 1)`` of a DenseNet layer (x_{i+1} = cat(x_i, layer_i(x_i))) whose first
    operand's other consumer is a BN site (``a_site``, the layer's first BN, whose backward runs
    after this one): the backward leaves a's gradient - a channel slice of the output gradient,
    no copy - with that site, whose apply pass adds it; autograd adds nothing.  With a
    ``chain`` (the lowering, ``_chain_dense_cats``) the forward writes b into the block's
    concat buffer and returns a view of it (:class:`DenseChain`)."""

    def __init__(self, ctx, a_site: 'BNAct'):
        super().__init__(ctx)
        object.__setattr__(self, 'a_site', a_site)
        object.__setattr__(self, 'chain', None)
        object.__setattr__(self, 'chain_first', False)
        object.__setattr__(self, 'chain_last', False)
        object.__setattr__(self, 'off', a_site.bn.C)   # a's channel count (b's offset in the buffer)
        # the output's gradient arrives split in two from the consumer BN site's apply pass
        # (BNAct.split_to); the autograd gradient is then a placeholder
        object.__setattr__(self, 'split_expected', False)
        object.__setattr__(self, '_split_pending', None)

    def forward(self, a, b):
        return _run(self, a, b)

    def fwd(self, a, b):
        Ca, Cb = a.shape[1], b.shape[1]
        ch = self.chain
        if ch is None or a.dim() != 4 or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or Ca + Cb > ch.width:
            return torch.cat([a, b], 1), [], (Ca, Cb)
        an, bn = a.permute(0, 2, 3, 1), b.permute(0, 2, 3, 1)
        # b is normally in place already (its conv site wrote it into the buffer, ConvBNAct
        # .cat_out), and a is the buffer's leading Ca channels except at the block's first
        # concat; whatever is not in place is copied in (a fresh buffer when it does not fit)
        b_in = ch.placed(bn, Ca)
        a_in = ch.placed(an, 0)
        if not (b_in or a_in):
            ch.fresh(*an.shape[:3], a.device)
        buf = ch.buf
        # the copies extend the buffer past every view handed out so far; the views' saved
        # copies (earlier BN sites' inputs) are unchanged, so their version stays valid
        with torch.autograd._unsafe_preserve_version_counter(buf):
            if not a_in:
                buf[..., :Ca].copy_(an)
            if not b_in:
                buf[..., Ca:Ca + Cb].copy_(bn)
        ch.buf = None if self.chain_last else buf
        return buf[..., :Ca + Cb].permute(0, 3, 1, 2), [], (Ca, Cb)

    def bwd(self, dout, saved, keep, needs):
        Ca, Cb = keep
        sp = self._split_pending
        object.__setattr__(self, '_split_pending', None)
        if sp is not None:
            da, db = sp
            if needs[0]:
                object.__setattr__(self.a_site, '_slice_pending', da)
            return [None, from_nhwc(db, Cb) if needs[1] else None]
        if self.split_expected and dout.stride() == (0,) * dout.dim():
            raise RuntimeError('DenseCat: the split gradient hand-off did not arrive (backward order differs from '
                               'the one the lowering assumed)')
        g = to_nhwc(dout, Ca + Cb)                 # the channels_last view, no copy
        if needs[0]:
            object.__setattr__(self.a_site, '_slice_pending', g[..., :Ca])
        return [None, from_nhwc(g[..., Ca:], Cb) if needs[1] else None]


class UpCat(Site):
    """``F.interpolate(x, scale_factor=2, mode='nearest')`` [-> ``torch.cat([up, skip], 1)``]
    as one NHWC pass (``seg.hip`` upcat: the U-Net decoder's input) and its backward (2x2
    sum-pool of the upsampled channels, slice of the skip's).  Channel counts that are not
    multiples of 8 take the same math in torch ops."""

    def forward(self, x, skip=None):
        return _run(self, x, skip) if skip is not None else _run(self, x)

    def fwd(self, x, skip=None):
        if x.dim() != 4:
            raise ValueError(f'UpCat: a {x.dim()}-D input (the native upsample takes NCHW images)')
        C1, C2 = x.shape[1], (skip.shape[1] if skip is not None else 0)
        xn = to_nhwc(x)
        sn = to_nhwc(skip) if skip is not None else None
        if xn.is_cuda and (C1 % 8 or C2 % 8):
            up = xn.repeat_interleave(2, 1).repeat_interleave(2, 2)
            out = torch.cat([up, sn], 3) if sn is not None else up.contiguous()
        else:
            out = Seg.upcat_fwd(xn, sn)
        return from_nhwc(out, C1 + C2), [], (C1, C2)

    def bwd(self, dout, saved, keep, needs):
        C1, C2 = keep
        dn = to_nhwc(dout)
        if dn.is_cuda and (C1 % 8 or C2 % 8):
            N, H, W, _ = dn.shape
            d = dn.float()
            dlo = d[..., :C1].reshape(N, H // 2, 2, W // 2, 2, C1).sum((2, 4)).to(torch.bfloat16)
            dskip = d[..., C1:].to(torch.bfloat16).contiguous() if C2 else None
        else:
            dlo, dskip = Seg.upcat_bwd(dn, C1)
        out = [from_nhwc(dlo, C1) if needs[0] else None]
        if C2:
            out.append(from_nhwc(dskip, C2) if needs[1] else None)
        return out


class ChannelGate(Site):
    """``act(y * g [+ res])`` with g = [N, C, 1, 1] a gate computed from y's global average
    (squeeze-excitation: EfficientNet's MBConv; SE-ResNeXt's block tail with its residual add
    and ReLU): one NHWC pass forward, one backward (ReLU mask, the residual's gradient,
    dy = d * g and dg = sum over pixels of d * y together)."""

    def __init__(self, ctx, relu: bool = False, residual: bool = False):
        super().__init__(ctx)
        self.relu, self.residual = relu, residual

    def forward(self, y, g, res=None):
        return _run(self, y, g, res) if res is not None else _run(self, y, g)

    def fwd(self, y, g, res=None):
        N, C = y.shape[:2]
        if y.dim() != 4 or tuple(g.shape) != (N, C, 1, 1):
            raise ValueError(f'ChannelGate: {tuple(y.shape)} * {tuple(g.shape)} is not an image times a '
                             'per-channel gate')
        Cp = ceil8(C)
        yn = to_nhwc(y, Cp)
        rn = to_nhwc(res, Cp) if res is not None else None
        gn = g.reshape(N, C).to(torch.bfloat16)
        if Cp != C:
            gn = torch.nn.functional.pad(gn, (0, Cp - C))
        gn = gn.contiguous()
        z = Fn.chscale_fwd(yn, gn, rn, self.relu)
        return from_nhwc(z, C), [yn, gn, z if self.relu else gn], (C, g.dtype, rn is not None)

    def bwd(self, dout, saved, keep, needs):
        yn, gn, z = saved
        C, gdt, has_res = keep
        addend = self.acc.buf if self.acc is not None and needs[0] else None
        dy, dg, dres = Fn.chscale_bwd(to_nhwc(dout, yn.shape[-1]), yn, gn, z if self.relu else None,
                                      want_dres=has_res and needs[2], addend=addend)
        if self.acc is not None and needs[0]:
            dy = self.acc.give(dy)
        N = yn.shape[0]
        out = [from_nhwc(dy, C) if needs[0] and dy is not None else None,
               dg[:, :C].to(gdt).reshape(N, C, 1, 1) if needs[1] else None]
        if has_res:
            out.append(from_nhwc(dres, C) if needs[2] else None)
        return out


class BilinearUp(Site):
    """``F.interpolate(x, size | scale_factor, mode='bilinear', align_corners=True)`` on the
    NHWC kernels (``seg.hip``; channels padded to 8)."""

    def __init__(self, ctx, scale=None):
        super().__init__(ctx)
        self.scale = scale

    def forward(self, x, size=None):
        return _run(self, x, size) if size is not None else _run(self, x)

    def fwd(self, x, size=None):
        N, C, H, W = x.shape
        if size is not None:
            Ho, Wo = (int(size), int(size)) if isinstance(size, int) else (int(size[0]), int(size[1]))
        else:
            sh, sw = self.scale
            Ho, Wo = int(H * sh), int(W * sw)
        xn = to_nhwc(x, ceil8(C))
        y = Seg.bilinear_up_fwd(xn, Ho, Wo)
        return from_nhwc(y, C), [], (C, H, W)

    def bwd(self, dout, saved, keep, needs):
        C, H, W = keep
        dx = Seg.bilinear_up_bwd(to_nhwc(dout, ceil8(C)), H, W)
        return [from_nhwc(dx, C)] + ([None] if len(needs) > 1 else [])


class MaxPool(Site):
    def __init__(self, ctx, k, s, p, ceil_mode=False):
        super().__init__(ctx)
        self.k, self.s, self.p, self.ceil = k, s, p, ceil_mode

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        C = x.shape[1]
        xn = to_nhwc(x, ceil8(C))
        y, idx = Fn.maxpool_fwd(xn, self.k, self.s, self.p, self.ceil)
        return from_nhwc(y, C), [idx], tuple(xn.shape)

    def bwd(self, dout, saved, xshape, needs):
        (idx,) = saved
        C = dout.shape[1]
        dx = Fn.maxpool_bwd(to_nhwc(dout, xshape[-1]), idx, xshape, self.k, self.s, self.p)
        return [from_nhwc(dx, C)]


class AvgPool(Site):
    """avg_pool2d(x, k, s, p) (square, floor mode, no divisor override) as one NHWC pass each way
    (pool_loss.hip): Inception's 3x3/1 branch pools, DenseNet's 2x2/2 transitions."""

    def __init__(self, ctx, k, s, p, count_include_pad=True):
        super().__init__(ctx)
        self.k, self.s, self.p, self.cip = k, s, p, bool(count_include_pad)

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        C = x.shape[1]
        xn = to_nhwc(x, ceil8(C))
        y = Fn.avgpool2d_fwd(xn, self.k, self.s, self.p, self.cip)
        return from_nhwc(y, C), [], tuple(xn.shape)

    def bwd(self, dout, saved, xshape, needs):
        C = dout.shape[1]
        addend = self.acc.buf if self.acc is not None else None
        dx = Fn.avgpool2d_bwd(to_nhwc(dout, xshape[-1]), xshape, self.k, self.s, self.p, self.cip, addend=addend)
        if self.acc is not None:
            dx = self.acc.give(dx)
        return [from_nhwc(dx, C) if dx is not None else None]


class AdaptiveAvgPool(Site):
    """adaptive_avg_pool2d(x, (Ho, Wo)) with output > 1 (PSPNet's pyramid, any model's fixed-
    size pool): PyTorch's overlapping bins, fp32 sums, one NHWC pass each way (pool_loss.hip)."""

    def __init__(self, ctx, Ho, Wo):
        super().__init__(ctx)
        self.Ho, self.Wo = int(Ho), int(Wo)

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        C = x.shape[1]
        xn = to_nhwc(x, ceil8(C))
        y = Fn.adaptive_avg_fwd(xn, self.Ho, self.Wo)
        return from_nhwc(y, C), [], tuple(xn.shape)

    def bwd(self, dout, saved, xshape, needs):
        C = dout.shape[1]
        return [from_nhwc(Fn.adaptive_avg_bwd(to_nhwc(dout, xshape[-1]), xshape), C)]


class GlobalAvgPool(Site):
    """adaptive_avg_pool2d(x, 1): [N, C, H, W] -> [N, C, 1, 1]."""

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        C = x.shape[1]
        xn = to_nhwc(x, ceil8(C))
        y = Fn.avgpool_fwd(xn)              # [N, Cp]
        return y[:, :C, None, None], [], tuple(xn.shape)

    def bwd(self, dout, saved, xshape, needs):
        N, H, W, Cp = xshape
        C = dout.shape[1]
        d = dout.reshape(N, C).to(torch.bfloat16)
        if Cp != C:
            d = torch.nn.functional.pad(d, (0, Cp - C))
        addend = self.acc.buf if self.acc is not None else None
        dx = Fn.avgpool_bwd(d.contiguous(), xshape, addend=addend)
        if self.acc is not None:
            dx = self.acc.give(dx)
        return [from_nhwc(dx, C) if dx is not None else None]


class VolumePool(nn.Module):
    """Global average pooling of a [N, C, *spatial] tensor (video / 1-D) on the native pooling
    kernel: the channels_last(_3d) activation viewed as the image [N, C, prod(spatial), 1]
    (a view, no copy).

    * ``flat_bins=None``: ``AdaptiveAvgPool3d(1)`` / ``AdaptiveAvgPool1d(1)`` ->
      [N, C, 1, ...];
    * ``flat_bins=K``: the ResNeXt3D head's ``AdaptiveAvgPool1d(K)`` over ``x.reshape(N, 1,
      -1)`` (`mlcomp/contrib/model/video/resnext3d/resnext3d.py`): with C == K every bin is
      exactly one channel's T*H*W values, i.e. a global average pool -> [N, 1, K]; other
      sizes run the torch ops."""

    def __init__(self, ctx, flat_bins=None):
        super().__init__()
        self.gap = GlobalAvgPool(ctx)
        self.flat_bins = flat_bins

    def forward(self, x):
        N, C = x.shape[:2]
        if self.flat_bins is not None and C != self.flat_bins:
            return torch.nn.functional.adaptive_avg_pool1d(x.reshape(N, 1, -1), self.flat_bins)
        y = self.gap(x.flatten(2).unsqueeze(-1))            # [N, C, 1, 1]
        if self.flat_bins is not None:
            return y.reshape(N, 1, C)
        return y.reshape(N, C, *([1] * (x.dim() - 2)))


__all__ = ['ConvParams', 'BNParams', 'LinearParams', 'ConvBNAct', 'BNAct', 'LinearAct', 'MaxPool',
           'GlobalAvgPool', 'VolumePool', 'to_nhwc', 'from_nhwc', 'ceil8']
