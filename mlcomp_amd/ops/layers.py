"""Native layers: autograd Functions over the HIP kernels + arena-backed parameters.

A native layer is a small Python object (not an ``nn.Module``) whose parameters are
slots of a :class:`~mlcomp_amd.ops.arena.ParamArena`.  Its autograd Function writes
parameter gradients *directly* into the arena's grad buffer (wgrad epilogues, BN
dgamma/dbeta) and notifies the arena (``mark_ready``) so the gradient bucketer can
launch the all-reduce (and the optimizer update) of a completed bucket while backward
continues; a slot is marked only after the last backward kernel that reads its weight.  Autograd only
carries activation gradients; every Function takes the model's ``anchor`` tensor
(requires_grad=True) so the graph is built even though the input image needs no grad.

Per-step scratch that must start at zero (BN forward partial sums, BN backward sums,
loss / accuracy accumulators) lives in one ``Workspace`` buffer cleared by a single
memset at the start of the step.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.nn as nn

from . import functional as Fn
from .arena import ParamArena, Slot

# MLC_DGRAD_FIRST=1/0: capture a layer's input-gradient GEMM before / after its side-stream
# weight gradient (both forked from the same point).  It changes which hardware queue the
# HIP graph executor gives each chain, and the measured effect is engine-dependent
# (profiles/round3/README.md): U-Net +1.8 % with dgrad first, ResNet-50 -1 %, BERT-base -3 %.
# Unset: the engine's default (NativeContext.dgrad_first; the U-Net engine turns it on).
DGRAD_FIRST_ENV = os.environ.get('MLC_DGRAD_FIRST')


class Workspace:
    """One zero-per-step fp32 buffer carved into named views."""

    def __init__(self):
        self._req: List[tuple] = []
        self.buf = None
        self.views = {}

    def request(self, key, n):
        self._req.append((key, int(n)))
        return key

    def finalize(self, device):
        total = sum((n + 63) // 64 * 64 for _, n in self._req) or 64
        self.buf = torch.zeros(total, device=device, dtype=torch.float32)
        off = 0
        for key, n in self._req:
            self.views[key] = self.buf[off:off + n]
            off += (n + 63) // 64 * 64

    def __getitem__(self, key):
        return self.views[key]

    def zero(self):
        self.buf.zero_()


class NativeContext:
    """Shared state of one native model: arena, workspace, anchor, train flag."""

    def __init__(self):
        self.arena = ParamArena()
        self.ws = Workspace()
        self.anchor = None
        self.training = True
        self.device = None
        # True when the step zeroes the whole grad arena once up front: the wgrad kernels
        # then accumulate (atomics) instead of issuing one memset per layer
        self.grad_prezeroed = False
        # MLC_WGRAD_STREAM=1 (default): a layer's weight gradient runs on a second stream,
        # concurrently with its input gradient, and joins before the layer's backward returns
        # (so no tensor outlives its stream's use); both read the same output gradient.
        # Measured +3 % ResNet-50, +1 % U-Net (profiles/round2_ab); 0 turns it off
        self.wgrad_stream = None
        # MLC_DGRAD_WT=1 (default): the convs keep a transposed, flipped filter copy
        # (Fn.WtTable) so their input-gradient GEMMs read the filter K-contiguous (stride 1:
        # on the forward conv's loaders); the model refreshes it once per step after the
        # forward pass (refresh_wt)
        self.wt = Fn.WtTable() if os.environ.get('MLC_DGRAD_WT', '1') == '1' else None
        self.wt_stale = False
        # MLC_WGRAD_LAG=N (engines may set a default): a layer's side-stream weight gradient
        # is joined N layers later (event per layer) instead of at the end of its own
        # backward, so the main stream does not stall on a wgrad that just started;
        # flush_wgrad joins the remaining ones
        self.wgrad_lag = int(os.environ.get('MLC_WGRAD_LAG', '0') or 0)
        # wgrad_defer (engines opt in; MLC_WGRAD_DEFER overrides): the side-stream weight
        # gradients are never joined per layer - they form one free-running chain beside the
        # input-gradient chain, their operands are kept alive for the side stream with
        # record_stream, the gradient bucketer waits on the side stream as well, and the
        # chain joins once, in flush_wgrad (bucketer.finish, before the optimizer)
        self.wgrad_defer = False
        self._pending_wgrad = []       # (event, operands kept alive, slots to mark), oldest first
        self.dgrad_first = DGRAD_FIRST_ENV == '1'
        # split-K conv weight gradients through fp32 slabs + a reduce pass (True) or straight
        # fp32 atomics (False); engines pick their measured default, MLC_WGRAD_SLAB overrides
        self.wgrad_slab = os.environ.get('MLC_WGRAD_SLAB', '1') != '0'

    def default_wgrad_slab(self, on: bool):
        """Engine default for the conv weight-gradient split-K reduction (MLC_WGRAD_SLAB
        overrides).  Interleaved A/B, profiles/round5/wgrad_slab_ab.txt: atomics win on ResNet-50
        (hand +0.6 %, generic +1.2 %) and DeepLab (+1.3 %), slabs on U-Net (+1.5 %)."""
        if os.environ.get('MLC_WGRAD_SLAB') is None:
            self.wgrad_slab = on

    def default_dgrad_first(self, on: bool):
        """Engine default for the capture order (MLC_DGRAD_FIRST overrides it)."""
        if DGRAD_FIRST_ENV is None:
            self.dgrad_first = on

    def finalize(self, device):
        self.device = torch.device(device)
        self.arena.finalize(device)
        self.ws.finalize(device)
        if self.wt is not None:
            self.wt.finalize(self.device)
        self.anchor = torch.zeros(1, device=device, requires_grad=True)
        self.arena.flush = self.flush_wgrad
        if self.device.type == 'cuda' and os.environ.get('MLC_WGRAD_STREAM', '1') in ('1', '2'):
            self.wgrad_stream = torch.cuda.Stream(self.device)
        self.default_wgrad_defer(False)

    def default_wgrad_defer(self, on: bool):
        """Engine default for the deferred weight-gradient join (MLC_WGRAD_DEFER overrides)."""
        env = os.environ.get('MLC_WGRAD_DEFER')
        self.wgrad_defer = (env == '1') if env is not None else on
        self.arena.grad_streams = [self.wgrad_stream] if (self.wgrad_defer and self.wgrad_stream) else []

    def flush_wgrad(self):
        """Join the lagged weight gradient (if any) into the current stream and mark its
        slot ready; with wgrad_defer, join the whole side-stream chain.  Must run before
        anything reads the gradient arena (the bucketer's finish() calls it through
        ``arena.flush``)."""
        if self.wgrad_defer and self.wgrad_stream is not None:
            cur = torch.cuda.current_stream(self.device)
            if cur != self.wgrad_stream:
                cur.wait_stream(self.wgrad_stream)
        self.join_wgrads(0)

    def default_wgrad_lag(self, n: int):
        """Engine default for the lagged join depth (MLC_WGRAD_LAG overrides it)."""
        if os.environ.get('MLC_WGRAD_LAG') is None:
            self.wgrad_lag = n

    def lag_wgrad(self, ev, keep, slots):
        """Queue a side-stream weight gradient (``ev`` recorded after it; ``keep``: its operands,
        held until the join so their memory is not reused early) and join the ones beyond
        the lag depth."""
        self._pending_wgrad.append((ev, keep, slots))
        self.join_wgrads(self.wgrad_lag)

    def join_wgrads(self, keep_last: int):
        """Join queued weight gradients into the current stream, oldest first, until at most
        ``keep_last`` remain, and mark their slots ready."""
        q = self._pending_wgrad
        while len(q) > keep_last:
            ev, _keep, slots = q.pop(0)
            cur = torch.cuda.current_stream(self.device)
            if cur != self.wgrad_stream:
                cur.wait_event(ev)
            for s in (slots if isinstance(slots, (list, tuple)) else (slots,)):
                self.arena.mark_ready(s)

    def refresh_wt(self):
        """Re-derive the transposed filters from the current weights (one launch, on the
        current stream).  Called by the model at the end of its training forward pass."""
        if self.wt is not None and self.training:
            self.wt.refresh()
        self.wt_stale = False


def flatten_bn_buffers(units) -> Optional[torch.Tensor]:
    """One fp32 buffer holding every unit's BatchNorm running mean and variance; the units
    are re-pointed at views of it.  Call after the units loaded their weights and before a
    graph is captured: the rank-0 buffer broadcast (:meth:`GraphedStep.broadcast_buffers`)
    is then one collective of ~2 x sum(C) floats."""
    units = [u for u in units if getattr(u, 'run_mean', None) is not None]
    if not units:
        return None
    flat = torch.empty(sum(2 * u.run_mean.numel() for u in units), device=units[0].run_mean.device)
    off = 0
    for u in units:
        C = u.run_mean.numel()
        flat[off:off + C].copy_(u.run_mean)
        flat[off + C:off + 2 * C].copy_(u.run_var)
        u.run_mean, u.run_var = flat[off:off + C], flat[off + C:off + 2 * C]
        off += 2 * C
    return flat


# ---------------------------------------------------------------------------- conv+bn
class ConvBN:
    """conv (no bias) -> BatchNorm (train-mode batch stats) -> [+residual] -> [ReLU]."""

    def __init__(self, ctx: NativeContext, name: str, conv: nn.Conv2d, bn: nn.BatchNorm2d,
                 act: bool, cin_pad: Optional[int] = None, s2d: bool = False):
        assert conv.groups == 1, 'native ConvBN supports groups=1'
        self.ctx = ctx
        self.name = name
        Co, Ci, KH, KW = conv.weight.shape
        self.cin = Ci
        self.cin_p = cin_pad or Ci
        self.Co = Co
        self.k = (KH, KW)
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.dil = conv.dilation[0]
        # s2d: a 7x7/2 pad-3 stem over <= 3 channels runs as a 4x4/1 conv over the 2x2
        # space-to-depth input (Fn.stem_s2d): K = 256 instead of 392 padded to 448
        self.s2d = s2d
        if s2d:
            assert (KH, KW, self.stride, self.pad, self.dil) == (7, 7, 2, 3, 1) and Ci <= 3, \
                's2d stem needs a 7x7/2 pad-3 conv over <= 3 channels'
            self.k, self.stride, self.pad, self.cin_p = (4, 4), 1, 0, 16
            KH = KW = 4
        self.act = act
        self.eps = bn.eps
        self.momentum = bn.momentum if bn.momentum is not None else 0.1
        self.w = ctx.arena.weight(f'{name}.conv.weight', (Co, KH, KW, self.cin_p))
        self.wt_idx = None
        if ctx.wt is not None and not s2d:
            self.wt_idx = ctx.wt.add(self.w)
        self.gamma = ctx.arena.vector(f'{name}.bn.weight', (Co,))
        self.beta = ctx.arena.vector(f'{name}.bn.bias', (Co,))
        self._src = (conv, bn)
        self.k_s1 = ctx.ws.request(f'{name}.s1', Fn.NSTAT * Co)
        self.k_s2 = ctx.ws.request(f'{name}.s2', Fn.NSTAT * Co)
        self.k_bw = ctx.ws.request(f'{name}.bwd', Fn.NSTAT * 2 * Co)

    def load_from_torch(self):
        conv, bn = self._src
        dev = self.ctx.device
        if self.s2d:
            w = Fn.stem_w_to_s2d(conv.weight.detach().cpu())
            # taps of the zero-extended 8x8 filter (row/col 7) and the 4 pad channels must
            # stay zero: their gradients are masked after every wgrad
            self._gmask = (Fn.stem_w_to_s2d(torch.ones(self.Co, self.cin, 7, 7)) != 0).float().to(dev)
        else:
            w = conv.weight.detach().permute(0, 2, 3, 1).float()
            if self.cin_p != self.cin:
                w = torch.nn.functional.pad(w, (0, self.cin_p - self.cin))
        self.w.master.copy_(w.to(dev))
        self.gamma.master.copy_(bn.weight.detach().to(dev))
        self.beta.master.copy_(bn.bias.detach().to(dev))
        self.run_mean = bn.running_mean.detach().clone().float().to(dev)
        self.run_var = bn.running_var.detach().clone().float().to(dev)
        Co = self.Co
        b = torch.zeros(7, Co, device=dev)
        self.save_mean, self.save_invstd, self.scale, self.shift = b[0], b[1], b[2], b[3]
        self.coef = b[4:7].reshape(-1)

    def export_to_torch(self):
        conv, bn = self._src
        if self.s2d:
            w = Fn.stem_w_from_s2d(self.w.master.detach().float().cpu(), self.cin)
        else:
            w = self.w.master[..., :self.cin].permute(0, 3, 1, 2).contiguous()
        conv.weight.data.copy_(w.to(conv.weight.device))
        bn.weight.data.copy_(self.gamma.master.to(bn.weight.device))
        bn.bias.data.copy_(self.beta.master.to(bn.bias.device))
        bn.running_mean.copy_(self.run_mean.to(bn.running_mean.device))
        bn.running_var.copy_(self.run_var.to(bn.running_var.device))

    def __call__(self, x, res=None):
        return _ConvBNFn.apply(x, res, self.ctx.anchor, self)

    # raw (autograd-free) halves, composed by the block-level Functions
    def fwd(self, x, res=None, defer=False, in_affine=None):
        """z = act(BN(conv(x)) [+ res]); ``res`` is a tensor or a deferred BN output
        ``(y, scale, shift)`` (applied in the same pass).  ``defer=True`` stops after the
        statistics: z is not materialised (returns None; scale/shift are ready).
        ``in_affine = (sc, sh)``: ``x`` is the pre-BN output of the previous (ReLU) unit,
        whose BN + ReLU the conv applies while loading its operand."""
        ws = self.ctx.ws
        if self.s2d and x.shape[-1] != 16:
            x = Fn.stem_s2d(x, 3)
        raff = None
        if isinstance(res, tuple):
            res, rs, rh = res
            raff = (rs, rh)
        if not self.ctx.training:  # inference BN: running statistics, no stat epilogue
            y = self._conv(x, None, in_affine)
            torch.rsqrt(self.run_var + self.eps, out=self.scale).mul_(self.gamma.master)
            torch.sub(self.beta.master, self.run_mean * self.scale, out=self.shift)
            if defer:
                return None, (x, y, None)
            z = Fn.bn_apply(y, res, self.scale, self.shift, self.act, res_affine=raff)
            return z, (x, y, z)
        s1, s2 = ws[self.k_s1], ws[self.k_s2]
        self.ctx.wt_stale = True
        y = self._conv(x, (s1, s2), in_affine)
        training = self.ctx.training
        z = Fn.bn_fwd_apply(y, res, s1, s2, self.gamma.master, self.beta.master, self.save_mean,
                            self.save_invstd, self.run_mean if training else None,
                            self.run_var if training else None, self.eps, self.momentum, self.act,
                            scale=self.scale, shift=self.shift, res_affine=raff, apply=not defer)
        return z, (x, y, z)

    # the three GEMMs of the unit (overridden by ConvTBN)
    def _conv(self, x, stats, in_affine=None):
        if self.s2d and in_affine is None:
            return Fn.stem_conv_fwd(x, self.w.bf16, stats=stats)
        return Fn.conv2d_fwd(x, self.w.bf16, self.stride, self.pad, self.dil, stats=stats, in_affine=in_affine)

    def _dgrad(self, dy, x_shape, addend=None, out=None, bn=None):
        wt = None
        if self.wt_idx is not None:
            if self.ctx.wt_stale:
                raise RuntimeError('transposed filters are stale: the model must call '
                                   'ctx.refresh_wt() after its training forward pass')
            wt = self.ctx.wt[self.wt_idx]
        return Fn.conv2d_dgrad(dy, self.w.bf16, x_shape, self.stride, self.pad, self.dil,
                               addend=addend, out=out, bn=bn, wt=wt)

    def dgrad_covers_all(self) -> bool:
        """True when the dgrad GEMM epilogue writes every dx row, i.e. a BN-backward
        reduction can be fused into it.  Always true: strided dgrads run one GEMM per
        stride-parity class, and a class no filter tap reaches is still written (0 +
        addend) by a K = 0 launch."""
        return True

    def bn_target(self, rec):
        """(y, mean, sums) of this unit's BN for a fused dgrad epilogue."""
        x, y, z = rec
        return (y, self.save_mean, self.ctx.ws[self.k_bw])

    def wgrad(self, dy, x, in_affine=None):
        """Weight gradient into the arena (masked for the s2d stem).  The caller marks the
        slot ready once nothing later in backward reads the weight (its dgrad): a marked
        bucket may be updated by the optimizer right away (GradBucketer)."""
        Fn.conv2d_wgrad(dy, x, self.w.shape, self.stride, self.pad, self.dil, out=self.w.grad,
                        accumulate=self.ctx.grad_prezeroed, in_affine=in_affine, slab=self.ctx.wgrad_slab)
        if self.s2d:
            self.w.grad.mul_(self._gmask)

    def bwd(self, dz, rec, want_dres=False, dx_addend=None, need_dx=True, dx_out=None,
            prereduced=False, dgrad_bn=None, in_affine=None, defer: Optional[list] = None):
        """``defer`` (with a wgrad stream): leave the weight gradient running on the side
        stream; (dy, x, weight slot) is appended so the caller keeps the tensors alive, joins
        the stream later and then marks the slot ready."""
        x, y, z = rec
        arena = self.ctx.arena
        dy, dres = Fn.bn_bwd(dz, z if self.act else None, y, self.save_mean, self.save_invstd,
                             self.gamma.master, want_dres=want_dres, dgamma=self.gamma.grad,
                             dbeta=self.beta.grad, sums=self.ctx.ws[self.k_bw], zero_sums=False,
                             coef=self.coef, prereduced=prereduced)
        arena.mark_ready(self.gamma)
        arena.mark_ready(self.beta)
        side = self.ctx.wgrad_stream if need_dx else None
        if side is not None and torch.cuda.current_stream(self.ctx.device) == side:
            side = None            # already on the side stream (a forked branch): run inline
        fork = None
        if side is not None:
            main = torch.cuda.current_stream(self.ctx.device)
            fork = torch.cuda.Event()
            fork.record(main)                      # dy, x and the grad slot are ready
            if not self.ctx.dgrad_first:
                side.wait_event(fork)
                with Fn.side_stream(side):
                    self.wgrad(dy, x, in_affine)
        else:
            self.wgrad(dy, x, in_affine)
        dx = None
        if need_dx:
            dx = self._dgrad(dy, x.shape, addend=dx_addend, out=dx_out, bn=dgrad_bn)
        if side is not None and self.ctx.dgrad_first:
            # captured after the dgrad but forked from the point before it: the dgrad is the
            # first child of the previous node, so graph replay keeps the dgrad -> BN chain
            # on one hardware queue and only the weight gradient crosses queues
            side.wait_event(fork)
            with Fn.side_stream(side):
                self.wgrad(dy, x, in_affine)
        if side is not None and defer is not None:
            defer.append((dy, x, self.w))
            return dx, dres
        if side is not None and self.ctx.wgrad_defer:
            # no per-layer join (NativeContext.wgrad_defer): dy / x stay alive for the side
            # stream, the bucketer waits on it, flush_wgrad joins it before the optimizer
            dy.record_stream(side)
            x.record_stream(side)
            arena.mark_ready(self.w)
            return dx, dres
        if side is not None and self.ctx.wgrad_lag:
            ev = torch.cuda.Event()
            ev.record(side)
            self.ctx.lag_wgrad(ev, (dy, x), self.w)   # keeps dy, x alive until joined
            return dx, dres
        if side is not None:
            main.wait_stream(side)                 # join: the weight gradient is complete
        arena.mark_ready(self.w)   # after the dgrad: the last reader of w in backward
        return dx, dres


class ConvTBN(ConvBN):
    """transposed conv (``nn.ConvTranspose2d``) -> BatchNorm (train-mode batch stats) ->
    [ReLU]: LinkNet's x2 up-convolution (`mlcomp/contrib/segmentation/linknet/decoder.py`,
    4x4 / stride 2 / pad 1).  Its three GEMMs are the conv GEMMs with the roles turned
    round (:func:`Fn.conv_transpose2d_fwd`): forward = the dgrad parity-class GEMMs with the
    BN statistics in their epilogue, input gradient = a forward conv over the same filter,
    weight gradient = the conv wgrad with x and dy swapped.

    The conv's bias is not applied: a training-mode BatchNorm subtracts the batch mean, so
    the bias changes neither the output nor any gradient (its gradient is exactly zero and it
    stays untouched).  It only shifts the running mean, which is kept bias-free here and
    converted on load / export."""

    def __init__(self, ctx: NativeContext, name: str, conv: nn.ConvTranspose2d, bn: nn.BatchNorm2d, act: bool):
        assert conv.groups == 1 and conv.dilation[0] == conv.dilation[1], 'native ConvTBN: groups=1'
        assert conv.stride[0] == conv.stride[1] and conv.padding[0] == conv.padding[1]
        self.ctx = ctx
        self.name = name
        Cin, Cout, KH, KW = conv.weight.shape
        assert bn.num_features == Cout
        self.cin = self.cin_p = Cout          # last dim of the [Cin, KH, KW, Cout] filter
        self.Co = Cout
        self.k = (KH, KW)
        self.stride, self.pad, self.dil = conv.stride[0], conv.padding[0], conv.dilation[0]
        self.out_pad = conv.output_padding
        self.s2d = False
        self.act = act
        self.eps = bn.eps
        self.momentum = bn.momentum if bn.momentum is not None else 0.1
        self.w = ctx.arena.weight(f'{name}.conv.weight', (Cin, KH, KW, Cout))
        self.wt_idx = None
        self.gamma = ctx.arena.vector(f'{name}.bn.weight', (Cout,))
        self.beta = ctx.arena.vector(f'{name}.bn.bias', (Cout,))
        self._src = (conv, bn)
        self.k_s1 = ctx.ws.request(f'{name}.s1', Fn.NSTAT * Cout)
        self.k_s2 = ctx.ws.request(f'{name}.s2', Fn.NSTAT * Cout)
        self.k_bw = ctx.ws.request(f'{name}.bwd', Fn.NSTAT * 2 * Cout)

    def _bias(self):
        conv = self._src[0]
        return conv.bias.detach().float().to(self.ctx.device) if conv.bias is not None else None

    def load_from_torch(self):
        super().load_from_torch()
        b = self._bias()
        if b is not None:
            self.run_mean.sub_(b)

    def export_to_torch(self):
        super().export_to_torch()
        b = self._bias()
        if b is not None:
            bn = self._src[1]
            bn.running_mean.add_(b.to(bn.running_mean.device))

    def out_hw(self, H, W):
        KH, KW = self.k
        return ((H - 1) * self.stride - 2 * self.pad + self.dil * (KH - 1) + self.out_pad[0] + 1,
                (W - 1) * self.stride - 2 * self.pad + self.dil * (KW - 1) + self.out_pad[1] + 1)

    def _conv(self, x, stats, in_affine=None):
        assert in_affine is None
        return Fn.conv_transpose2d_fwd(x, self.w.bf16, self.out_hw(x.shape[1], x.shape[2]), self.stride,
                                       self.pad, self.dil, stats=stats)

    def _dgrad(self, dy, x_shape, addend=None, out=None, bn=None):
        assert addend is None and out is None and bn is None, 'ConvTBN input gradient: plain conv'
        dx = Fn.conv2d_fwd(dy, self.w.bf16, self.stride, self.pad, self.dil)
        assert tuple(dx.shape) == tuple(x_shape), (dx.shape, x_shape)
        return dx

    def wgrad(self, dy, x, in_affine=None):
        assert in_affine is None
        Fn.conv2d_wgrad(x, dy, self.w.shape, self.stride, self.pad, self.dil, out=self.w.grad,
                        accumulate=self.ctx.grad_prezeroed)


class _ConvBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, anchor, m: ConvBN):
        z, rec = m.fwd(x, res)
        ctx.m = m
        ctx.has_res = res is not None
        ctx.save_for_backward(*rec)
        return z

    @staticmethod
    def backward(ctx, dz):
        m: ConvBN = ctx.m
        dx, dres = m.bwd(dz.contiguous(), ctx.saved_tensors, want_dres=ctx.has_res,
                         need_dx=ctx.needs_input_grad[0])
        return dx, dres, None, None


class ResidualBlock:
    """units[0..n-1] chained, the last one adding the shortcut (identity or ``down(x)``)
    before its ReLU.  One autograd node for the whole block: backward fuses the gradient
    sum at the branch point into the dgrad epilogue of the first unit.

    BN-backward fusion: the dgrad that produces a BN's output gradient also masks it by
    the ReLU and accumulates that BN's backward sums (``Fn.BnBwdSpec``), so no separate
    reduction pass runs.  Inside a block, unit i+1's dgrad serves unit i; the first
    unit's dgrad (the block's input gradient) serves the PREVIOUS block's last BN and its
    downsample BN, linked through ``prev`` and flagged by ``dout_prereduced``."""

    def __init__(self, units: List[ConvBN], down: Optional[ConvBN]):
        self.units = units
        self.down = down
        self.ctx = units[0].ctx
        self.prev: Optional['ResidualBlock'] = None
        self.fuse_bn_bwd = True
        # shortcut conv (forward and backward) on the side stream, concurrently with the main
        # branch (MLC_DOWN_STREAM; ResNet-50 +1.3 %, the U-Net engine turns it off)
        self.down_stream = os.environ.get('MLC_DOWN_STREAM', '1') == '1'
        # BN-apply fusion (MLC_FUSE_BN_FWD: 0 off, 1 into 1x1 consumers, 2 into every
        # consumer): an inner unit's output z_i = relu(BN(y_i)) is not written; unit i+1
        # reads y_i and applies BN+ReLU in its conv and weight-gradient operand loaders.
        # Measured on MI355X (docs/kernels.md): the loader transform costs the 3x3 convs
        # more than the saved pass, so the default is off.
        # Mode 3: only into 1x1 consumers over <= 64 channels, whose GEMM is a single K-tile
        # on the register-staged loop anyway (no LDS-DMA given up for the transform).
        mode = int(os.environ.get('MLC_FUSE_BN_FWD', '0'))
        one = lambda u: u.k == (1, 1) and u.stride == 1 and u.pad == 0  # noqa: E731
        self.fuse_into = [False] + [
            mode >= 1 and prev.act and (mode == 2 or (one(u) and (mode != 3 or u.cin <= 64)))
            for prev, u in zip(units[:-1], units[1:])]
        self.dout_prereduced = False
        self._last = None   # (rec of the last unit, rec of down) of the latest forward

    @property
    def fuse_bn_fwd(self) -> bool:
        return any(self.fuse_into)

    @fuse_bn_fwd.setter
    def fuse_bn_fwd(self, on: bool):
        self.fuse_into = [False] + [bool(on) and p.act for p in self.units[:-1]]

    def in_affines(self):
        """Input transform of each unit: (scale, shift) of the previous unit's BN where the
        BN-apply is fused into this unit's loaders, else None."""
        return [None] + [(p.scale, p.shift) if f else None for p, f in zip(self.units[:-1], self.fuse_into[1:])]

    def __call__(self, x):
        return _ResidualBlockFn.apply(x, self.ctx.anchor, self)

    def output_bn_spec(self):
        """BnBwdSpec for the gradient of this block's output (used by the next block).
        With a downsample branch the output is relu(bn3(y3) + bn_d(y_d)), so the ReLU
        mask is recomputed from the two pre-BN tensors the reduction reads anyway."""
        rec, rd = self._last
        last = self.units[-1]
        ys = [last.bn_target(rec)]
        if self.down is not None and not self.down.act:
            ys.append(self.down.bn_target(rd))
            return Fn.BnBwdSpec(None, ys, affine=[(last.scale, last.shift),
                                                  (self.down.scale, self.down.shift)])
        if self.down is not None:
            ys.append(self.down.bn_target(rd))
        return Fn.BnBwdSpec(rec[2], ys)


class _ResidualBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, blk: ResidualBlock):
        recs = []
        # MLC_DOWN_STREAM=1 (default; +0.7 % ResNet-50): the shortcut conv runs on the side stream, concurrently with the
        # main branch, and joins before the last unit (the only reader of its output)
        side = blk.ctx.wgrad_stream if (blk.down is not None and blk.down_stream) else None
        if side is not None:
            main = torch.cuda.current_stream(blk.ctx.device)
            side.wait_stream(main)
        if blk.down is not None:
            # the downsample BN (no activation) is applied inside the last unit's pass
            if side is not None:
                with Fn.side_stream(side):
                    _, rd = blk.down.fwd(x, defer=not blk.down.act)
            else:
                _, rd = blk.down.fwd(x, defer=not blk.down.act)
            identity = rd[2] if blk.down.act else (rd[1], blk.down.scale, blk.down.shift)
        else:
            identity, rd = x, None
        y = x
        affs = blk.in_affines()
        for i, u in enumerate(blk.units[:-1]):
            if blk.fuse_into[i + 1]:
                _, r = u.fwd(y, defer=True, in_affine=affs[i])
                y = r[1]           # pre-BN output; the next conv applies BN + ReLU
            else:
                y, r = u.fwd(y, in_affine=affs[i])
            recs.append(r)
        if side is not None:
            main.wait_stream(side)
        out, r = blk.units[-1].fwd(y, identity, in_affine=affs[-1])
        recs.append(r)
        blk._last = (r, rd)
        ctx.blk = blk
        ctx.n = len(recs)
        flat = [t for r in recs for t in r]
        if rd is not None:
            flat += list(rd)
        ctx.save_for_backward(*flat)
        return out

    @staticmethod
    def backward(ctx, dout):
        blk: ResidualBlock = ctx.blk
        saved = ctx.saved_tensors
        recs = [saved[3 * i:3 * i + 3] for i in range(ctx.n)]
        rd = saved[3 * ctx.n:3 * ctx.n + 3] if blk.down is not None else None
        dout = dout.contiguous()
        need_dx = ctx.needs_input_grad[0]
        pre = blk.dout_prereduced
        blk.dout_prereduced = False
        units = blk.units
        fuse = blk.fuse_bn_bwd
        affs = blk.in_affines()
        if blk.fuse_bn_fwd:
            assert fuse, 'the BN-apply fusion needs the fused BN-backward reductions (z is not stored)'

        def spec_for(i):  # fused reduction of unit i's BN in unit i+1's dgrad
            u = units[i]
            if not fuse or not units[i + 1].dgrad_covers_all():
                return None
            if u.act:   # z = relu(y*scale + shift): mask recomputed from y, z not read
                return Fn.BnBwdSpec(None, [u.bn_target(recs[i])], affine=[(u.scale, u.shift)])
            return Fn.BnBwdSpec(None, [u.bn_target(recs[i])])

        # with a wgrad stream the block's weight gradients overlap its whole input-gradient
        # chain and join once at the end (MLC_WGRAD_STREAM=2; 1 joins per unit)
        side = units[0].ctx.wgrad_stream
        pend = [] if side is not None and os.environ.get('MLC_WGRAD_STREAM') == '2' else None
        # last unit: its dres is the shortcut-branch gradient
        sp = spec_for(len(units) - 2) if len(units) > 1 else None
        d, dres = units[-1].bwd(dout, recs[-1], want_dres=True, prereduced=pre, dgrad_bn=sp,
                                in_affine=affs[-1], defer=pend)
        fused = sp is not None
        # MLC_DOWN_STREAM: the shortcut branch's backward runs on the side stream while the
        # main branch's inner units run; its dx buffer is allocated on the main stream (it
        # becomes the first unit's dgrad output) and the streams join before that dgrad
        down_side = side if (blk.down is not None and pend is None and blk.down_stream) else None
        short = dres
        if down_side is not None:
            main = torch.cuda.current_stream(units[0].ctx.device)
            short_buf = torch.empty(rd[0].shape, device=rd[0].device, dtype=rd[0].dtype) if need_dx else None
            down_side.wait_stream(main)
            with Fn.side_stream(down_side):
                short, _ = blk.down.bwd(dres, rd, need_dx=need_dx, prereduced=pre, dx_out=short_buf)
        for i in range(len(units) - 2, 0, -1):
            sp = spec_for(i - 1)
            d, _ = units[i].bwd(d, recs[i], prereduced=fused, dgrad_bn=sp, in_affine=affs[i], defer=pend)
            fused = sp is not None
        if down_side is not None:
            main.wait_stream(down_side)
        elif blk.down is not None:
            # shortcut conv first; its dx becomes the addend of the first unit's dgrad
            short, _ = blk.down.bwd(dres, rd, need_dx=need_dx, prereduced=pre, defer=pend)
        prev_spec = None
        if need_dx and fuse and blk.prev is not None and blk.prev._last is not None \
                and units[0].dgrad_covers_all():
            prev_spec = blk.prev.output_bn_spec()
        dx, _ = units[0].bwd(d, recs[0], dx_addend=short if need_dx else None, need_dx=need_dx,
                             dx_out=short if (need_dx and blk.down is not None) else None,
                             prereduced=fused, dgrad_bn=prev_spec, defer=pend)
        if prev_spec is not None:
            blk.prev.dout_prereduced = True
        if pend:
            torch.cuda.current_stream(units[0].ctx.device).wait_stream(side)
            for _, _, w in pend:
                units[0].ctx.arena.mark_ready(w)
            pend.clear()
        return dx, None, None


# ---------------------------------------------------------------------------- pooling
class MaxPool:
    def __init__(self, k=3, s=2, p=1):
        self.k, self.s, self.p = k, s, p

    def __call__(self, x, anchor):
        return _MaxPoolFn.apply(x, anchor, self)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, m):
        y, idx = Fn.maxpool_fwd(x, m.k, m.s, m.p)
        ctx.m = m
        ctx.xshape = tuple(x.shape)
        ctx.save_for_backward(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        m = ctx.m
        return Fn.maxpool_bwd(dy.contiguous(), idx, ctx.xshape, m.k, m.s, m.p), None, None


class StemPool:
    """The classifier stem: conv -> BN -> ReLU -> maxpool 3x3/2 with the ReLU output never
    materialised.  The conv epilogue accumulates the BN statistics, one fused pass applies
    BN + ReLU + max-pool (csrc/kernels/stem.hip), and the backward recomputes the pooled
    gradient scatter inside the two BN-backward passes.  (U-Net keeps ``stem`` + ``MaxPool``:
    its decoder reads the un-pooled stem activation as a skip connection.)"""

    def __init__(self, stem: ConvBN):
        assert stem.act, 'StemPool fuses the stem ReLU'
        self.stem = stem
        self.ctx = stem.ctx

    def __call__(self, x):
        return _StemPoolFn.apply(x, self.ctx.anchor, self)


class _StemPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, m: StemPool):
        st = m.stem
        if not st.ctx.training:
            z, _ = st.fwd(x)
            out, _ = Fn.maxpool_fwd(z)
            return out
        _, (x_, y, _) = st.fwd(x, defer=True)
        out, idx = Fn.stem_pool_fwd(y, st.scale, st.shift)
        ctx.m = m
        ctx.save_for_backward(x_, y, idx)
        return out

    @staticmethod
    def backward(ctx, dp):
        st: ConvBN = ctx.m.stem
        x, y, idx = ctx.saved_tensors
        arena = st.ctx.arena
        dy = Fn.stem_pool_bwd(dp.contiguous(), idx, y, st.save_mean, st.save_invstd, st.gamma.master,
                              st.gamma.grad, st.beta.grad, st.ctx.ws[st.k_bw], st.coef)
        arena.mark_ready(st.gamma)
        arena.mark_ready(st.beta)
        st.wgrad(dy, x)
        arena.mark_ready(st.w)
        return None, None, None


# ---------------------------------------------------------------------------- head
class ClassifierHead:
    """global avg-pool -> linear (+bias) -> fused softmax cross-entropy."""

    def __init__(self, ctx: NativeContext, name: str, fc: nn.Linear, smoothing: float = 0.0):
        self.ctx = ctx
        self.name = name
        self.fc = fc
        self.O, self.I = fc.weight.shape
        # output rows padded to a multiple of 8 (16-byte MFMA operand chunks); the
        # padded rows stay zero and the loss ignores their logits
        self.Op = (self.O + 7) // 8 * 8
        self.w = ctx.arena.weight(f'{name}.weight', (self.Op, self.I))
        self.b = ctx.arena.vector(f'{name}.bias', (self.Op,))
        self.smoothing = smoothing
        self.k_loss = ctx.ws.request(f'{name}.loss', 1)
        self.k_correct = ctx.ws.request(f'{name}.correct', 1)

    def load_from_torch(self):
        dev = self.ctx.device
        self.w.master[:self.O].copy_(self.fc.weight.detach().float().to(dev))
        self.b.master[:self.O].copy_(self.fc.bias.detach().float().to(dev))

    def export_to_torch(self):
        self.fc.weight.data.copy_(self.w.master[:self.O].to(self.fc.weight.device))
        self.fc.bias.data.copy_(self.b.master[:self.O].to(self.fc.bias.device))

    def loss_sum(self):
        return self.ctx.ws[self.k_loss]

    def correct(self):
        return self.ctx.ws[self.k_correct]

    def __call__(self, x, labels):
        return _HeadFn.apply(x, labels, self.ctx.anchor, self)

    def logits(self, x):
        pooled = Fn.avgpool_fwd(x)
        return Fn.linear_fwd(pooled, self.w.bf16, self.b.master)[:, :self.O]


class _HeadFn(torch.autograd.Function):
    """Returns the summed loss (fp32 [1]); backward assumes d(loss) = 1 and scales the
    logits gradient by 1/B inside the CE kernel (mean reduction)."""

    @staticmethod
    def forward(ctx, x, labels, anchor, h: ClassifierHead):
        pooled = Fn.avgpool_fwd(x)
        logits = Fn.linear_fwd(pooled, h.w.bf16, h.b.master)
        ws = h.ctx.ws
        dl = Fn.softmax_ce(logits, labels, ws[h.k_loss], ws[h.k_correct],
                           scale=1.0 / labels.shape[0], smoothing=h.smoothing, num_classes=h.O)
        ctx.h = h
        ctx.xshape = tuple(x.shape)
        ctx.save_for_backward(pooled, dl)
        # the workspace slot itself (no copy kernel): it is read before the next step's
        # workspace zeroing, and the backward never reads it
        return ws[h.k_loss].view(1)

    @staticmethod
    def backward(ctx, dloss):
        pooled, dl = ctx.saved_tensors
        h: ClassifierHead = ctx.h
        arena = h.ctx.arena
        Fn.linear_wgrad(dl, pooled, out=h.w.grad)
        Fn.colsum(dl, h.b.grad)
        dpooled = Fn.linear_dgrad(dl, h.w.bf16)
        arena.mark_ready(h.w)      # after the dgrad (the last reader of w)
        arena.mark_ready(h.b)
        dx = Fn.avgpool_bwd(dpooled, ctx.xshape)
        return dx, None, None, None
