"""Functional NHWC ops of the native engine.

Tensors on a GPU go to the hand-written HIP kernels (``csrc/kernels``); tensors on the
CPU run the mathematically identical PyTorch reference below, which is what the CPU
test-suite exercises (and what the GPU numerics tests compare the kernels against).
There is no silent fallback for device tensors: a kernel that rejects a shape raises.

Layout conventions
  activations  NHWC bf16, contiguous ([N, H, W, C])
  conv weight  [Co, KH, KW, Ci] (bf16 for compute; fp32 master/grad in the same order)
  linear       weight [O, I] bf16, bias fp32
"""
from __future__ import annotations

from typing import Optional, Tuple

import contextlib
import math
import os
import threading

import torch
import torch.nn.functional as F

from . import _lib


def _cuda(t):
    return t is not None and t.is_cuda


def conv_out_hw(H, W, KH, KW, stride, pad, dil):
    ph, pw = (pad, pad) if isinstance(pad, int) else tuple(pad)
    Ho = (H + 2 * ph - dil * (KH - 1) - 1) // stride + 1
    Wo = (W + 2 * pw - dil * (KW - 1) - 1) // stride + 1
    return Ho, Wo


def pack_pad(pad) -> int:
    """The ``pad`` argument of the dense conv kernels: an int pads both axes, (pad_h, pad_w)
    with different values is packed as (1 << 30) | (pad_w << 15) | pad_h (convgeom.h)."""
    if isinstance(pad, int):
        return pad
    ph, pw = (int(v) for v in pad)
    return ph if ph == pw else (1 << 30) | (pw << 15) | ph


# ---------------------------------------------------------------- conv
def bn_relu_input(x: torch.Tensor, in_affine) -> torch.Tensor:
    """relu(x * sc + sh) per channel (NHWC) - the conv input an ``in_affine`` stands for."""
    sc, sh = in_affine
    return torch.relu(x.float() * sc + sh).to(torch.bfloat16)


def conv2d_fwd(x: torch.Tensor, w: torch.Tensor, stride=1, pad=0, dil=1,
               stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
               out: Optional[torch.Tensor] = None, in_affine=None) -> torch.Tensor:
    """y = conv(x, w) in NHWC; if ``stats`` given (see :func:`stat_buffers`: two
    [NSTAT*Co] fp32 buffers), accumulates per-channel partial sums of y and y^2 into
    them (the BN forward statistics, reduced over the NSTAT copies by bn_fwd_apply).
    ``in_affine = (sc, sh)``: ``x`` is the pre-BN tensor of a ReLU BatchNorm and the conv
    input is relu(x*sc + sh), applied inside the kernel's operand loader."""
    N, H, W, C = x.shape
    Co, KH, KW, Ci = w.shape
    assert Ci == C, (w.shape, x.shape)
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, pad, dil)
    if _cuda(x):
        y = out if out is not None else torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.bfloat16)
        ldy = rows_ld(y)
        if ldy != Co:       # out: the channel slice of wider rows (a DenseNet block's concat buffer)
            assert ldy is not None and stats is None and in_affine is None, (y.shape, y.stride())
            _lib.call('mlc_conv_fwd_ld', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), ldy, N, H, W, C, Co, KH, KW, stride,
                      pack_pad(pad), dil, Ho, Wo, _lib.stream())
            return y
        s1, s2 = (stats if stats is not None else (None, None))
        sc, sh = in_affine if in_affine is not None else (None, None)
        _lib.call('mlc_conv_fwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(s1), _lib.ptr(s2),
                  N, H, W, C, Co, KH, KW, stride, pack_pad(pad), dil, Ho, Wo, _lib.ptr(sc), _lib.ptr(sh), _lib.stream())
        return y
    if in_affine is not None:
        x = bn_relu_input(x, in_affine)
    yf = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, stride, pad, dil)
    if stats is not None:
        stats[0][:Co].add_(yf.sum(dim=(0, 2, 3)))
        stats[1][:Co].add_((yf * yf).sum(dim=(0, 2, 3)))
    y = yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
    if out is not None:
        out.copy_(y)
        return out
    return y


def conv_transpose2d_fwd(x: torch.Tensor, w: torch.Tensor, out_hw, stride=2, pad=1, dil=1,
                         stats: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """y = conv_transpose(x, w) in NHWC, no bias: x [N, Hi, Wi, Cin], w [Cin, KH, KW, Cout]
    (nn.ConvTranspose2d's [Cin, Cout, KH, KW] with the taps first), y [N, *out_hw, Cout].
    It is the input gradient of the conv y -> x over w, so the GPU path runs the dgrad's
    parity-class GEMMs (``mlc_conv_tr_fwd``); ``stats`` as in :func:`conv2d_fwd`.  Its own
    input gradient is :func:`conv2d_fwd` of dy over w, its weight gradient
    :func:`conv2d_wgrad` (dy=x, x=dy)."""
    N, Hi, Wi, Cin = x.shape
    Cw, KH, KW, Cout = w.shape
    assert Cw == Cin, (w.shape, x.shape)
    Ho, Wo = out_hw
    assert conv_out_hw(Ho, Wo, KH, KW, stride, pad, dil) == (Hi, Wi), (out_hw, x.shape)
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, Cout, device=x.device, dtype=torch.bfloat16)
        s1, s2 = (stats if stats is not None else (None, None))
        _lib.call('mlc_conv_tr_fwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(s1), _lib.ptr(s2),
                  N, Hi, Wi, Cin, Cout, KH, KW, stride, pack_pad(pad), dil, Ho, Wo, _lib.stream())
        return y
    oph = Ho - ((Hi - 1) * stride - 2 * pad + dil * (KH - 1) + 1)
    opw = Wo - ((Wi - 1) * stride - 2 * pad + dil * (KW - 1) + 1)
    yf = F.conv_transpose2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), None, stride, pad,
                            (oph, opw), 1, dil)
    if stats is not None:
        stats[0][:Cout].add_(yf.sum(dim=(0, 2, 3)))
        stats[1][:Cout].add_((yf * yf).sum(dim=(0, 2, 3)))
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


class BnBwdSpec:
    """Backward reduction of up to two BatchNorms fused into a dgrad epilogue: the dgrad
    output is their (shared) output gradient dU.  ``mask`` (the BN output z, or None)
    applies the ReLU; ``ys`` = [(y, mean, sums)] with ``sums`` the NSTAT*2*C scratch
    :func:`bn_bwd` later consumes with ``prereduced=True``.  ``affine`` = [(scale,
    shift)] per y recomputes the ReLU mask as  sum_k y_k*scale_k + shift_k > 0  instead
    of reading z (valid when z = relu(that sum), i.e. no residual tensor input)."""

    def __init__(self, mask, ys, affine=None):
        assert 1 <= len(ys) <= 2
        assert affine is None or (mask is None and len(affine) == len(ys))
        self.mask = mask
        self.ys = list(ys)
        self.affine = list(affine) if affine is not None else None


def wt_flip_transpose(w: torch.Tensor) -> torch.Tensor:
    """[Co, KH, KW, Ci] filter -> [Ci, KH, KW, Co] with the taps flipped: the filter of the
    stride-1 forward conv that computes this conv's input gradient (csrc/kernels/wtrans.hip)."""
    return w.flip(1, 2).permute(3, 1, 2, 0).contiguous()


def dgrad_as_fwd_conv(KH, KW, stride, pad, dil) -> bool:
    """Shapes whose input gradient is a stride-1 forward conv of dy over the transposed
    filter (the others use the parity-class GEMMs, with the transposed filter as well)."""
    return stride == 1 and pad <= dil * (KH - 1) and dil * (KH - 1) - pad == dil * (KW - 1) - pad


class WtTable:
    """The transposed, flipped bf16 copies ``wt`` of a model's stride-1 conv filters, one
    buffer, refreshed from the bf16 weight mirrors by one batched kernel launch per step
    (``refresh``, after the forward pass: the weights cannot change before backward).  The
    dgrad GEMMs then read both operands K-contiguous (``mlc_conv_dgrad_t``)."""

    def __init__(self):
        self.slots = []      # arena slots of [Co, KH, KW, Ci] filters
        self.views = []
        self.buf = None
        self.desc = None
        self.blocks = 0
        self._srcs = None

    def add(self, slot) -> int:
        self.slots.append(slot)
        return len(self.slots) - 1

    def __getitem__(self, i) -> torch.Tensor:
        return self.views[i]

    @staticmethod
    def _dims(shape):
        """(Co, KH, KW, Ci) of a conv filter, or of a [out, in] dense weight (1x1 taps)."""
        return tuple(shape) if len(shape) == 4 else (shape[0], 1, 1, shape[1])

    def finalize(self, device):
        if not self.slots:
            return
        total = sum((s.numel + 63) // 64 * 64 for s in self.slots)
        self.buf = torch.zeros(total, device=device, dtype=torch.bfloat16)
        off = 0
        for s in self.slots:
            Co, KH, KW, Ci = self._dims(s.shape)
            v = self.buf[off:off + s.numel]
            self.views.append(v.view(Ci, KH, KW, Co) if len(s.shape) == 4 else v.view(Ci, Co))
            off += (s.numel + 63) // 64 * 64
        if self.buf.is_cuda:
            self._build()    # outside any stream capture (the table is an H2D copy)

    def _build(self):
        rows, blk = [], 0
        for s, v in zip(self.slots, self.views):
            Co, KH, KW, Ci = self._dims(s.shape)
            rows.append([s.bf16.data_ptr(), v.data_ptr(), Co, KH * KW, Ci, blk])
            blk += KH * KW * ((Co + 63) // 64) * ((Ci + 63) // 64)
        self.desc = torch.tensor(rows, dtype=torch.int64).to(self.buf.device)
        self.blocks = blk
        self._srcs = [r[0] for r in rows]

    def refresh(self):
        if self.buf is None:
            return
        if not self.buf.is_cuda:
            for s, v in zip(self.slots, self.views):
                v.copy_(wt_flip_transpose(s.bf16) if s.bf16.dim() == 4 else s.bf16.t())
            return
        if self._srcs != [s.bf16.data_ptr() for s in self.slots]:
            self._build()    # first call, or a weight mirror was re-allocated
        _lib.call('mlc_wt_transpose', _lib.ptr(self.desc), len(self.slots), self.blocks, _lib.stream())


def conv2d_dgrad(dy: torch.Tensor, w: torch.Tensor, x_shape, stride=1, pad=0, dil=1,
                 addend: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                 bn: Optional[BnBwdSpec] = None, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx = conv_transpose(dy, w) [+ addend] (the addend fuses the gradient sum of a
    residual branch point into the epilogue; ``out`` may alias ``addend``).  With ``bn``
    the epilogue also masks dx by ``bn.mask > 0`` and accumulates the BN-backward sums.
    ``wt`` (= :func:`wt_flip_transpose` of ``w``): read the filter operand K-contiguous
    from it (stride 1: the equivalent forward conv, :func:`dgrad_as_fwd_conv`)."""
    N, H, W, C = x_shape
    Co, KH, KW, Ci = w.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dx = out if out is not None else torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        b = [None] * 11
        if bn is not None:
            b[0] = bn.mask
            for k, (yk, mk, sk) in enumerate(bn.ys):
                b[1 + 3 * k:4 + 3 * k] = [yk, mk, sk]
            for k, (ak, hk) in enumerate(bn.affine or []):
                b[7 + 2 * k:9 + 2 * k] = [ak, hk]
        if wt is not None:
            assert tuple(wt.shape) == (Ci, KH, KW, Co), (wt.shape, w.shape)
            _lib.call('mlc_conv_dgrad_t', _lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), _lib.ptr(addend), N, H, W,
                      C, Co, KH, KW, stride, pack_pad(pad), dil, Ho, Wo, *[_lib.ptr(t) for t in b], _lib.stream())
            return dx
        _lib.call('mlc_conv_dgrad', _lib.ptr(dy), _lib.ptr(w), _lib.ptr(dx), _lib.ptr(addend), N, H, W, C,
                  Co, KH, KW, stride, pack_pad(pad), dil, Ho, Wo, *[_lib.ptr(t) for t in b], _lib.stream())
        return dx
    if wt is not None and isinstance(pad, int) and dgrad_as_fwd_conv(KH, KW, stride, pad, dil):   # fwd conv over wt
        dxf = F.conv2d(dy.permute(0, 3, 1, 2).float(), wt.permute(0, 3, 1, 2).float(), None, 1,
                       dil * (KH - 1) - pad, dil)
    else:
        if wt is not None:
            w = wt_flip_transpose(wt)     # the flip-transpose is its own inverse
        dxf = torch.nn.grad.conv2d_input((N, C, H, W), w.permute(0, 3, 1, 2).float(),
                                         dy.permute(0, 3, 1, 2).float(), stride, pad, dil)
    dxf = dxf.permute(0, 2, 3, 1)
    if addend is not None:
        dxf = dxf + addend.float()
    if bn is not None:
        if bn.mask is not None:
            dxf = dxf * (bn.mask.float() > 0)
        elif bn.affine is not None:
            q = sum(yk.float() * ak + hk for (yk, _, _), (ak, hk) in zip(bn.ys, bn.affine))
            dxf = dxf * (q > 0)
        d = dxf.to(torch.bfloat16).float().reshape(-1, C)
        for yk, mk, sk in bn.ys:
            sv = sk.view(NSTAT, 2, C)
            sv[0, 0] += d.sum(0)
            sv[0, 1] += (d * (yk.float().reshape(-1, C) - mk)).sum(0)
    dx = dxf.to(torch.bfloat16).contiguous()
    if out is not None:
        out.copy_(dx)
        return out
    return dx


_USE_SLAB = os.environ.get('MLC_WGRAD_SLAB', '1') != '0'
_SLAB = {}
_SLAB_OLD = []   # superseded buffers stay alive: a captured graph may still point at them


_ROLE = threading.local()


def register_side_stream(stream) -> None:
    """Kept for callers of the old API: the workspace role is now explicit (side_role)."""


@contextlib.contextmanager
def side_stream(stream):
    """``with torch.cuda.stream(stream)`` for work that runs CONCURRENTLY with the main
    stream (weight gradients, the shortcut branch): its split-K GEMMs get workspaces of
    their own.  The role is explicit, not derived from the stream id: pool stream ids are
    recycled, so the pool stream a graph warm-up or capture runs the main work on can carry
    the id of an earlier context's side stream - main and side GEMMs then shared one
    workspace while running concurrently."""
    prev = getattr(_ROLE, 'side', False)
    _ROLE.side = True
    try:
        with torch.cuda.stream(stream):
            yield
    finally:
        _ROLE.side = prev


class CounterLease:
    """The split-K tile-counter regions (``split_counters`` in igemm.hip) that the kernel
    library hands to launches captured under one owner id.  They are returned to the
    device's pool when the lease dies, i.e. with the capture store (and so the graph) that
    holds it: a re-capture (another model, a rebuilt step) reuses them instead of
    draining the pool."""
    _next = 0

    def __init__(self, device):
        CounterLease._next += 1
        self.owner = CounterLease._next
        self.device = torch.device(device)

    def release(self):
        if self.owner and torch.cuda.is_available():
            from . import _lib
            with torch.cuda.device(self.device):
                _lib.load().mlc_counters_release(self.owner)
        self.owner = 0

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


@contextlib.contextmanager
def capture_scope(store: dict):
    """Workspaces requested while a graph is being captured live in ``store`` (owned by the
    graph's owner) instead of the process-wide eager pool.  A captured graph bakes the
    workspace pointers in; eager work on another stream (a second model, a validation pass)
    must never write the slabs a replay may be using at the same time.  The kernel
    library does the same for its split-K tile counters: regions handed out during the
    capture are tagged with a :class:`CounterLease` kept in ``store`` and go back to the
    pool when ``store`` is dropped."""
    prev = getattr(_ROLE, 'capture', None)
    _ROLE.capture = store
    lease = None
    if torch.cuda.is_available():
        from . import _lib
        lease = store.setdefault('__counter_lease__', CounterLease(torch.cuda.current_device()))
        _lib.load().mlc_counters_owner(lease.owner)
    try:
        yield
    finally:
        _ROLE.capture = prev
        if lease is not None:
            _lib.load().mlc_counters_owner(0)


def workspace_key(device) -> str:
    device = torch.device(device)
    if device.type == 'cuda' and getattr(_ROLE, 'side', False):
        return f'{device}/side'
    return str(device)


def workspace_store(pool: dict) -> dict:
    """The dict a workspace lives in: the capture scope's own while capturing, else ``pool``."""
    cap = getattr(_ROLE, 'capture', None)
    if cap is not None and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return cap.setdefault(id(pool), {})
    return pool


def slab_workspace(device, n: int) -> torch.Tensor:
    """fp32 split-K slab workspace (no zeroing needed), grown on demand - first during
    eager warm-up.  One per stream role (workspace_key) and per capture scope."""
    key = workspace_key(device)
    store = workspace_store(_SLAB)
    buf = store.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None:
            _SLAB_OLD.append(buf)
        buf = torch.empty(max(n, 1 << 20), device=device, dtype=torch.float32)
        store[key] = buf
    return buf


def conv2d_wgrad(dy: torch.Tensor, x: torch.Tensor, w_shape, stride=1, pad=0, dil=1,
                 out: Optional[torch.Tensor] = None, accumulate=False, in_affine=None,
                 slab: Optional[bool] = None) -> torch.Tensor:
    """fp32 weight gradient in [Co, KH, KW, Ci] order (written into ``out`` if given).
    Split-K partial sums go through a slab workspace and one reduction pass (``slab``; None =
    MLC_WGRAD_SLAB, default on), or are added with fp32 atomics (``slab=False``).
    ``in_affine``: as in :func:`conv2d_fwd` (x is pre-BN, the input is relu(x*sc + sh))."""
    Co, KH, KW, Ci = w_shape
    N, H, W, C = x.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dw = out if out is not None else torch.empty(Co, KH, KW, Ci, device=dy.device, dtype=torch.float32)
        use = _USE_SLAB if slab is None else slab
        ws = slab_workspace(dy.device, min(32 * Co * KH * KW * Ci, 64 << 20)) if use else None
        sc, sh = in_affine if in_affine is not None else (None, None)
        _lib.call('mlc_conv_wgrad', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dw), N, H, W, C, Co, KH, KW,
                  stride, pack_pad(pad), dil, Ho, Wo, 0, int(accumulate), _lib.ptr(ws),
                  ws.numel() if ws is not None else 0, _lib.ptr(sc), _lib.ptr(sh), _lib.stream())
        return dw
    if in_affine is not None:
        x = bn_relu_input(x, in_affine)
    dwf = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (Co, Ci, KH, KW),
                                      dy.permute(0, 3, 1, 2).float(), stride, pad, dil)
    dwf = dwf.permute(0, 2, 3, 1)
    if out is not None:
        if accumulate:
            out.add_(dwf.reshape(out.shape))
        else:
            out.copy_(dwf.reshape(out.shape))
        return out
    return dwf.contiguous()


# ---------------------------------------------------------------- batch norm
# partial-sum copies of the per-channel reductions (conv-epilogue BN statistics, BN / LN
# backward sums, bias column sums): 32 (== mlc_bn_stat_copies()), or one per contributing
# block in deterministic mode (_lib.DET_COPIES, see mlc_set_deterministic)
NSTAT = _lib.DET_COPIES if _lib.DETERMINISTIC else 32


def stat_buffers(C, device):
    """Zeroed (sum, sumsq) buffers of NSTAT*C fp32 for conv2d_fwd(stats=...)."""
    b = torch.zeros(2, NSTAT * C, device=device, dtype=torch.float32)
    return b[0], b[1]


# finalize folded into the apply passes (batchnorm.hip bn_{fwd,bwd}_fused_kernel): one launch
# per BatchNorm each way instead of a per-channel finalize kernel + the elementwise pass
# (MLC_BN_FUSED=0: the two-launch form; ResNet-50 +0.9 %, 402 -> 302 dispatches per step,
# profiles/round6/bn_fused_ab.jsonl).  Not in deterministic mode, whose reductions keep one
# partial copy per contributing block.
BN_FUSED = os.environ.get('MLC_BN_FUSED', '1') == '1'


def _bn_fused_ok(C, ncopy):
    return BN_FUSED and not _lib.DETERMINISTIC and C % 8 == 0 and C >= 8 and 1 <= ncopy <= 64


def bn_fwd_apply(y, res, s1, s2, gamma, beta, save_mean, save_invstd, run_mean, run_var,
                 eps=1e-5, momentum=0.1, relu=True, out=None, scale=None, shift=None,
                 res_affine=None, apply=True):
    """z = act(BN_train(y) [+ res]) given the conv epilogue's partial sums s1/s2
    ([NSTAT*C] each).  Writes save_mean/save_invstd and updates running stats.
    ``res_affine=(rscale, rshift)`` applies a per-channel affine to the residual first (a
    downsample branch's BN folded into this pass).  ``apply=False`` only finalizes the
    statistics into ``scale``/``shift`` (required then) and returns None."""
    rows = y.numel() // y.shape[-1]
    C = y.shape[-1]
    ncopy = s1.numel() // C
    if _cuda(y):
        if scale is None:
            scale = torch.empty(2, C, device=y.device, dtype=torch.float32)
            scale, shift = scale[0], scale[1]
        if apply and _bn_fused_ok(C, ncopy):
            z = out if out is not None else torch.empty_like(y)
            rs, rh = res_affine if res_affine is not None else (None, None)
            _lib.call('mlc_bn_fwd_fused', _lib.ptr(y), _lib.ptr(res), _lib.ptr(z), _lib.ptr(s1), _lib.ptr(s2), ncopy,
                      _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(save_mean), _lib.ptr(save_invstd), _lib.ptr(scale),
                      _lib.ptr(shift), _lib.ptr(run_mean), _lib.ptr(run_var), _lib.ptr(rs), _lib.ptr(rh), rows, C,
                      float(eps), float(momentum), int(relu), _lib.stream())
            return z
        _lib.call('mlc_bn_finalize', _lib.ptr(s1), _lib.ptr(s2), ncopy, _lib.ptr(gamma), _lib.ptr(beta),
                  _lib.ptr(save_mean), _lib.ptr(save_invstd), _lib.ptr(scale), _lib.ptr(shift),
                  _lib.ptr(run_mean), _lib.ptr(run_var), rows, C, float(eps), float(momentum),
                  _lib.stream())
        if not apply:
            return None
        z = out if out is not None else torch.empty_like(y)
        rs, rh = res_affine if res_affine is not None else (None, None)
        _lib.call('mlc_bn_fwd_apply2', _lib.ptr(y), _lib.ptr(res), _lib.ptr(z), _lib.ptr(scale),
                  _lib.ptr(shift), _lib.ptr(rs), _lib.ptr(rh), rows, C, int(relu), _lib.stream())
        return z
    s1t = s1.reshape(ncopy, C).sum(0)
    s2t = s2.reshape(ncopy, C).sum(0)
    mean = s1t / rows
    var = (s2t / rows - mean * mean).clamp_min(0)
    inv = torch.rsqrt(var + eps)
    save_mean.copy_(mean)
    save_invstd.copy_(inv)
    if run_mean is not None:
        unb = var * rows / max(rows - 1, 1)
        run_mean.mul_(1 - momentum).add_(momentum * mean)
        run_var.mul_(1 - momentum).add_(momentum * unb)
    if scale is not None:
        scale.copy_(inv * gamma)
        shift.copy_(beta - mean * inv * gamma)
    if not apply:
        return None
    zf = (y.float() - mean) * (inv * gamma) + beta
    if res is not None:
        rf = res.float()
        if res_affine is not None:
            rf = rf * res_affine[0] + res_affine[1]
        zf = zf + rf
    if relu:
        zf = zf.clamp_min(0)
    z = zf.to(torch.bfloat16)
    if out is not None:
        out.copy_(z)
        return out
    return z


def bn_apply(y, res, scale, shift, relu=True, res_affine=None):
    """z = act(y*scale + shift [+ res (*rscale + rshift)]) with precomputed per-channel
    scale/shift (inference BatchNorm / frozen BN)."""
    rows = y.numel() // y.shape[-1]
    C = y.shape[-1]
    if _cuda(y):
        z = torch.empty_like(y)
        rs, rh = res_affine if res_affine is not None else (None, None)
        _lib.call('mlc_bn_fwd_apply2', _lib.ptr(y), _lib.ptr(res), _lib.ptr(z), _lib.ptr(scale),
                  _lib.ptr(shift), _lib.ptr(rs), _lib.ptr(rh), rows, C, int(relu), _lib.stream())
        return z
    zf = y.float() * scale + shift
    if res is not None:
        rf = res.float()
        if res_affine is not None:
            rf = rf * res_affine[0] + res_affine[1]
        zf = zf + rf
    if relu:
        zf = zf.clamp_min(0)
    return zf.to(torch.bfloat16)


def bn_bwd(dz, z, y, mean, invstd, gamma, want_dres=False, dgamma=None, dbeta=None, sums=None,
           zero_sums=True, coef=None, prereduced=False):
    """Backward of z = act(BN(y) [+res]).  ``z`` is the saved output (ReLU mask) or None
    when there is no ReLU.  Returns (dy, dres or None); writes dgamma/dbeta (fp32).
    ``sums`` is NSTAT*2*C fp32 scratch (must be zero on entry when ``zero_sums`` is
    False), ``coef`` 3*C fp32 scratch.  ``prereduced``: the producer of ``dz`` (a dgrad
    epilogue, :class:`BnBwdSpec`) already applied the ReLU mask and filled ``sums``; the
    residual-branch gradient is then ``dz`` itself."""
    rows = y.numel() // y.shape[-1]
    C = y.shape[-1]
    if prereduced:
        assert sums is not None
        z = None
    if _cuda(dz):
        if sums is None:
            sums = torch.zeros(NSTAT * 2 * C, device=dz.device, dtype=torch.float32)
        elif zero_sums and not prereduced:
            sums.zero_()
        if coef is None:
            coef = torch.empty(3 * C, device=dz.device, dtype=torch.float32)
        if not prereduced:
            _lib.call('mlc_bn_bwd_reduce', _lib.ptr(dz), _lib.ptr(z), _lib.ptr(y), _lib.ptr(mean),
                      _lib.ptr(sums), rows, C, _lib.stream())
        ncopy = NSTAT
        if _bn_fused_ok(C, ncopy):
            dy = torch.empty_like(y)
            dres = None
            if want_dres:
                dres = dz if prereduced else torch.empty_like(y)
            _lib.call('mlc_bn_bwd_fused', _lib.ptr(dz), _lib.ptr(z), _lib.ptr(y), _lib.ptr(mean), _lib.ptr(sums),
                      ncopy, _lib.ptr(invstd), _lib.ptr(gamma), _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(dy),
                      _lib.ptr(None if prereduced else dres), rows, C, _lib.stream())
            return dy, dres
        _lib.call('mlc_bn_bwd_finalize', _lib.ptr(sums), _lib.ptr(invstd), _lib.ptr(gamma), _lib.ptr(coef),
                  _lib.ptr(dgamma), _lib.ptr(dbeta), rows, C, _lib.stream())
        dy = torch.empty_like(y)
        dres = None
        if want_dres:
            dres = dz if prereduced else torch.empty_like(y)
        _lib.call('mlc_bn_bwd_apply', _lib.ptr(dz), _lib.ptr(z), _lib.ptr(y), _lib.ptr(mean),
                  _lib.ptr(coef), _lib.ptr(dy), _lib.ptr(None if prereduced else dres), rows, C,
                  _lib.stream())
        return dy, dres
    d = dz.float().reshape(rows, C)
    if z is not None:
        d = d * (z.reshape(rows, C).float() > 0)
    yc = y.float().reshape(rows, C) - mean
    if prereduced:
        sv = sums.view(NSTAT, 2, C).sum(0)
        S1, S2 = sv[0], sv[1]
    else:
        S1 = d.sum(0)
        S2 = (d * yc).sum(0)
    if dgamma is not None:
        dgamma.copy_(S2 * invstd)
        dbeta.copy_(S1)
    k1 = gamma * invstd
    dyf = k1 * d - k1 * S1 / rows - k1 * invstd * invstd * S2 / rows * yc
    dy = dyf.reshape(y.shape).to(torch.bfloat16)
    dres = None
    if want_dres:
        dres = dz if prereduced else d.reshape(y.shape).to(torch.bfloat16)
    return dy, dres


# ---------------------------------------------------------------- pooling
def pool_out_hw(H, W, k, s, p, ceil_mode=False):
    """nn.MaxPool2d's output size (ceil_mode: the last window may start in the right / bottom
    padding as long as it starts inside the input or its left padding)."""
    if not ceil_mode:
        return conv_out_hw(H, W, k, k, s, p, 1)

    def one(L):
        o = -(-(L + 2 * p - k) // s) + 1
        if (o - 1) * s >= L + p:
            o -= 1
        return o
    return one(H), one(W)


def maxpool_fwd(x, k=3, s=2, p=1, ceil_mode=False):
    N, H, W, C = x.shape
    Ho, Wo = pool_out_hw(H, W, k, s, p, ceil_mode)
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
        idx = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.uint8)
        _lib.call('mlc_maxpool_fwd', _lib.ptr(x), _lib.ptr(y), _lib.ptr(idx), N, H, W, C, Ho, Wo, k, s, p,
                  _lib.stream())
        return y, idx
    xf = x.permute(0, 3, 1, 2).float()
    yf, ind = F.max_pool2d(xf, k, s, p, ceil_mode=ceil_mode, return_indices=True)
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), ind


def maxpool_bwd(dy, idx, x_shape, k=3, s=2, p=1):
    N, H, W, C = x_shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_maxpool_bwd', _lib.ptr(dy), _lib.ptr(idx), _lib.ptr(dx), N, H, W, C, Ho, Wo, k, s,
                  p, _lib.stream())
        return dx
    dyf = dy.permute(0, 3, 1, 2).float().reshape(N, C, -1)
    dxf = torch.zeros(N, C, H * W).scatter_add_(2, idx.reshape(N, C, -1), dyf)
    return dxf.reshape(N, C, H, W).permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def stem_s2d(x, pad=3):
    """NHWC bf16 image (3 real channels, any channel stride) -> the 2x2 space-to-depth
    image of its ``pad``-padded version, [N, (H+2p)/2, (W+2p)/2, 16] with channel
    (dy*2+dx)*3+ci and channels 12..15 zero (csrc/kernels/stem.hip)."""
    N, H, W, Cs = x.shape
    Hb, Wb = (H + 2 * pad) // 2, (W + 2 * pad) // 2
    if _cuda(x):
        out = torch.empty(N, Hb, Wb, 16, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_stem_s2d', _lib.ptr(x.contiguous()), _lib.ptr(out), N, H, W, Cs, pad, _lib.stream())
        return out
    xp = F.pad(x[..., :3].float(), (0, 0, pad, pad, pad, pad))
    xp = xp.reshape(N, Hb, 2, Wb, 2, 3).permute(0, 1, 3, 2, 4, 5).reshape(N, Hb, Wb, 12)
    return F.pad(xp, (0, 4)).to(torch.bfloat16).contiguous()


_STEM_CONV = os.environ.get('MLC_STEM_CONV', '1') == '1'


def stem_conv_fwd(xs, w, stats=None):
    """The space-to-depth stem conv (4x4/1 over the [N, Hb, Wb, 16] image, w [64, 4, 4, 16])
    through the persistent register-resident-filter kernel (csrc/kernels/stemconv.hip);
    :func:`conv2d_fwd` on the CPU, in deterministic mode, with MLC_STEM_CONV=0 or for other
    shapes.  ``stats`` as in :func:`conv2d_fwd`."""
    if _cuda(xs) and _STEM_CONV and not _lib.DETERMINISTIC and tuple(w.shape) == (64, 4, 4, 16) \
            and xs.shape[-1] == 16 and xs.is_contiguous() and w.is_contiguous():
        N, Hb, Wb, _ = xs.shape
        y = torch.empty(N, Hb - 3, Wb - 3, 64, device=xs.device, dtype=torch.bfloat16)
        s1, s2 = stats if stats is not None else (None, None)
        _lib.call('mlc_stem_conv_fwd', _lib.ptr(xs), _lib.ptr(w), _lib.ptr(y), _lib.ptr(s1), _lib.ptr(s2),
                  N, Hb, Wb, _lib.stream())
        return y
    return conv2d_fwd(xs, w, 1, 0, 1, stats=stats)


def stem_s2d_to_nhwc(xs, pad=3):
    """Inverse of :func:`stem_s2d`: [N, Hb, Wb, 16] -> the [N, H, W, 3] image (float)."""
    N, Hb, Wb, _ = xs.shape
    x = xs[..., :12].float().reshape(N, Hb, Wb, 2, 2, 3).permute(0, 1, 3, 2, 4, 5)
    return x.reshape(N, 2 * Hb, 2 * Wb, 3)[:, pad:2 * Hb - pad, pad:2 * Wb - pad]


def stem_w_to_s2d(w):
    """[Co, Ci<=3, 7, 7] filter -> [Co, 4, 4, 16] space-to-depth filter (see stem_s2d)."""
    Co, Ci = w.shape[:2]
    w8 = F.pad(w.float(), (0, 1, 0, 1))                          # 8x8, tap 7 = 0
    w8 = F.pad(w8, (0, 0, 0, 0, 0, 3 - Ci)) if Ci < 3 else w8
    w2 = w8.reshape(Co, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1).reshape(Co, 4, 4, 12)
    return F.pad(w2, (0, 4))


def stem_w_from_s2d(w2, Ci=3):
    """Inverse of :func:`stem_w_to_s2d`: [Co, 4, 4, 16] -> [Co, Ci, 7, 7]."""
    Co = w2.shape[0]
    w8 = w2[..., :12].reshape(Co, 4, 4, 2, 2, 3).permute(0, 5, 1, 3, 2, 4).reshape(Co, 3, 8, 8)
    return w8[:, :Ci, :7, :7].contiguous()


def stem_pool_ok(C: int) -> bool:
    """Channel counts the fused stem kernels take: C/8 a power of two <= 64."""
    G = C // 8
    return C % 8 == 0 and 1 <= G <= 64 and G & (G - 1) == 0


_POOLED_REDUCE = os.environ.get('MLC_STEM_POOLED_REDUCE', '1') == '1'


def stem_pool_fwd(y, scale, shift):
    """ResNet stem tail: pooled = maxpool3x3/2(relu(y*scale + shift)) without
    materialising the activation (csrc/kernels/stem.hip).  Returns (pooled, idx); idx is
    the window argmax (uint8, 255 = ReLU inactive) on the GPU, an encoded int64 index
    (flat argmax * 2 + active) on the CPU."""
    N, H, W, C = y.shape
    Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    if _cuda(y):
        out = torch.empty(N, Ho, Wo, C, device=y.device, dtype=torch.bfloat16)
        # one buffer: the argmax bytes, then (MLC_STEM_POOLED_REDUCE=1, default) the pre-BN
        # value at the argmax, from which the backward's reduction runs over the pooled tensor
        n = N * Ho * Wo * C
        off = (n + 15) // 16 * 16          # 16-byte aligned ymax
        idx = torch.empty(off + 2 * n if _POOLED_REDUCE else n, device=y.device, dtype=torch.uint8)
        ymax = idx[off:].view(torch.bfloat16) if _POOLED_REDUCE else None
        _lib.call('mlc_stem_pool_fwd', _lib.ptr(y), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(out),
                  _lib.ptr(idx), _lib.ptr(ymax), N, H, W, C, _lib.stream())
        return out, idx
    a = (y.float() * scale + shift).permute(0, 3, 1, 2)
    m, ind = F.max_pool2d(a, 3, 2, 1, return_indices=True)
    active = (m > 0).long()
    out = m.clamp_min(0).permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
    return out, (ind * 2 + active).permute(0, 2, 3, 1).contiguous()


def stem_pool_bwd(dp, idx, y, mean, invstd, gamma, dgamma, dbeta, sums, coef):
    """Backward of :func:`stem_pool_fwd` through the BatchNorm: returns dy (bf16, the conv
    output gradient) and writes dgamma/dbeta.  ``sums`` (NSTAT*2*C fp32) must be zero on
    entry; ``coef`` is 3*C fp32 scratch."""
    N, H, W, C = y.shape
    rows = N * H * W
    if _cuda(dp):
        n = dp.numel()
        off = (n + 15) // 16 * 16
        if idx.numel() == off + 2 * n:   # pooled-side reduction (stem_pool_fwd kept ymax)
            _lib.call('mlc_stem_pool_bwd_reduce_pooled', _lib.ptr(dp), _lib.ptr(idx),
                      _lib.ptr(idx[off:].view(torch.bfloat16)), _lib.ptr(mean), _lib.ptr(sums), N, H, W, C,
                      _lib.stream())
        else:
            _lib.call('mlc_stem_pool_bwd_reduce', _lib.ptr(dp), _lib.ptr(idx), _lib.ptr(y), _lib.ptr(mean),
                      _lib.ptr(sums), N, H, W, C, _lib.stream())
        _lib.call('mlc_bn_bwd_finalize', _lib.ptr(sums), _lib.ptr(invstd), _lib.ptr(gamma), _lib.ptr(coef),
                  _lib.ptr(dgamma), _lib.ptr(dbeta), rows, C, _lib.stream())
        dy = torch.empty_like(y)
        _lib.call('mlc_stem_pool_bwd_apply', _lib.ptr(dp), _lib.ptr(idx), _lib.ptr(y), _lib.ptr(mean),
                  _lib.ptr(coef), _lib.ptr(dy), N, H, W, C, _lib.stream())
        return dy
    ind, active = idx.permute(0, 3, 1, 2) // 2, idx.permute(0, 3, 1, 2) % 2
    g = dp.permute(0, 3, 1, 2).float() * active
    du = torch.zeros(N, C, H * W).scatter_add_(2, ind.reshape(N, C, -1), g.reshape(N, C, -1))
    du = du.reshape(N, C, H, W).permute(0, 2, 3, 1).contiguous()
    dy, _ = bn_bwd(du, None, y, mean, invstd, gamma, dgamma=dgamma, dbeta=dbeta)
    return dy


def avgpool2d_fwd(x, k, s, p, count_include_pad=True):
    """KxK/s average pool (pad p, floor mode) of NHWC bf16 ``x`` (pool_loss.hip)."""
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_avgpool2d_fwd', _lib.ptr(x), _lib.ptr(y), N, H, W, C, Ho, Wo, k, s, p, int(count_include_pad),
                  _lib.stream())
        return y
    yf = F.avg_pool2d(_nchw(x), k, s, p, count_include_pad=count_include_pad)
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def avgpool2d_bwd(dy, x_shape, k, s, p, count_include_pad=True, addend=None):
    """Input gradient of :func:`avgpool2d_fwd` (+ ``addend``, NHWC bf16 of ``x_shape``: the other
    consumers' gradient of the pool's input, summed in the same pass)."""
    N, H, W, C = x_shape
    _, Ho, Wo, _ = dy.shape
    if addend is not None:
        assert tuple(addend.shape) == tuple(x_shape) and addend.is_contiguous(), (addend.shape, x_shape)
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_avgpool2d_bwd', _lib.ptr(dy.contiguous()), _lib.ptr(addend), _lib.ptr(dx), N, H, W, C, Ho,
                  Wo, k, s, p, int(count_include_pad), _lib.stream())
        return dx
    with torch.enable_grad():             # called from autograd backward (grad mode off)
        xf = torch.zeros(N, C, H, W, requires_grad=True)
        F.avg_pool2d(xf, k, s, p, count_include_pad=count_include_pad).backward(_nchw(dy))
    g = xf.grad.permute(0, 2, 3, 1)
    if addend is not None:
        g = g + addend.float()
    return g.to(torch.bfloat16).contiguous()


def adaptive_avg_fwd(x, Ho, Wo):
    """adaptive_avg_pool2d of NHWC bf16 ``x`` to (Ho, Wo) - PyTorch's (overlapping) bins, fp32
    sums, one bf16 rounding (pool_loss.hip; the GPU's stock channels_last bf16 kernel is
    ~3e-3 off its own CPU result on PSPNet's 3x3 / 6x6 bins, docs/numerics.md)."""
    N, H, W, C = x.shape
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_adaptive_avg_fwd', _lib.ptr(x.contiguous()), _lib.ptr(y), N, H, W, C, Ho, Wo, _lib.stream())
        return y
    yf = F.adaptive_avg_pool2d(x.permute(0, 3, 1, 2).float(), (Ho, Wo))
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def adaptive_avg_bwd(dy, x_shape):
    N, H, W, C = x_shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_adaptive_avg_bwd', _lib.ptr(dy.contiguous()), _lib.ptr(dx), N, H, W, C, Ho, Wo, _lib.stream())
        return dx
    with torch.enable_grad():             # called from autograd backward (grad mode off)
        xf = torch.zeros(N, C, H, W, requires_grad=True)
        F.adaptive_avg_pool2d(xf, (Ho, Wo)).backward(dy.permute(0, 3, 1, 2).float())
    return xf.grad.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


class AdaptiveAvgFn(torch.autograd.Function):
    """NHWC bf16 adaptive average pool with the native backward (:func:`adaptive_avg_fwd`)."""

    @staticmethod
    def forward(ctx, x, Ho, Wo):
        ctx.xshape = tuple(x.shape)
        return adaptive_avg_fwd(x, Ho, Wo)

    @staticmethod
    def backward(ctx, dy):
        return adaptive_avg_bwd(dy, ctx.xshape), None, None


def avgpool_fwd(x):
    N, H, W, C = x.shape
    if _cuda(x):
        y = torch.empty(N, C, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_avgpool_fwd', _lib.ptr(x), _lib.ptr(y), N, H * W, C, _lib.stream())
        return y
    return x.float().mean(dim=(1, 2)).to(torch.bfloat16)


def avgpool_bwd(dy, x_shape, addend=None):
    """Input gradient of the global average pool (+ ``addend``, NHWC bf16 of ``x_shape``)."""
    N, H, W, C = x_shape
    if addend is not None:
        assert tuple(addend.shape) == tuple(x_shape) and addend.is_contiguous(), (addend.shape, x_shape)
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_avgpool_bwd', _lib.ptr(dy), _lib.ptr(addend), _lib.ptr(dx), N, H * W, C, _lib.stream())
        return dx
    g = dy.float()[:, None, None, :] / (H * W)
    if addend is not None:
        g = g + addend.float()
    return g.expand(N, H, W, C).to(torch.bfloat16).contiguous()


# ---------------------------------------------------------------- linear
def linear_fwd(x, w, bias=None):
    """x [B, I] bf16, w [O, I] bf16 -> fp32 [B, O] (+bias)."""
    B, I = x.shape
    O = w.shape[0]
    if _cuda(x):
        out = torch.empty(B, O, device=x.device, dtype=torch.float32)
        _lib.call('mlc_gemm_f32out', _lib.ptr(x), _lib.ptr(w), _lib.ptr(out), _lib.ptr(bias), B, O, I,
                  I, I, O, 0, 1, 0, 0, 1, _lib.stream())
        return out
    out = x.float() @ w.float().t()
    return out + bias if bias is not None else out


def linear_dgrad(dout, w):
    """dout [B, O] bf16, w [O, I] bf16 -> dx [B, I] bf16."""
    B, O = dout.shape
    I = w.shape[1]
    if _cuda(dout):
        dx = torch.empty(B, I, device=dout.device, dtype=torch.bfloat16)
        _lib.call('mlc_gemm_bf16out', _lib.ptr(dout), _lib.ptr(w), _lib.ptr(dx), B, I, O, O, I, I, 0, 0,
                  _lib.stream())
        return dx
    return (dout.float() @ w.float()).to(torch.bfloat16)


def linear_wgrad(dout, x, out=None, accumulate=False):
    """dW [O, I] fp32 = dout^T x (+= into ``out`` when ``accumulate``).  Accumulation
    uses split-K with fp32 atomics, so small weight matrices (M x N tiles << CUs) still
    spread the long token reduction over the whole chip."""
    B, O = dout.shape
    I = x.shape[1]
    if _cuda(dout) and B % 8:
        # the GEMM reduces over the rows in 8-row chunks: zero rows add nothing (a batch of
        # 4 sequences in BERT's classifier head)
        pad = 8 - B % 8
        dout = torch.nn.functional.pad(dout, (0, 0, 0, pad))
        x = torch.nn.functional.pad(x, (0, 0, 0, pad))
        B += pad
    if _cuda(dout):
        dw = out if out is not None else torch.empty(O, I, device=dout.device, dtype=torch.float32)
        if accumulate:
            _lib.call('mlc_gemm_f32out', _lib.ptr(dout), _lib.ptr(x), _lib.ptr(dw), None, O, I, B, O, I, I,
                      1, 0, 1, 1, 0, _lib.stream())
        else:
            _lib.call('mlc_gemm_f32out', _lib.ptr(dout), _lib.ptr(x), _lib.ptr(dw), None, O, I, B, O, I, I,
                      1, 0, 0, 0, 1, _lib.stream())
        return dw
    g = dout.float().t() @ x.float()
    if out is not None:
        if accumulate:
            out.add_(g)
        else:
            out.copy_(g)
        return out
    return g


# Dense weight + bias gradients: split-K tiles written to fp32 slabs that a reduction pass
# sums (MLC_DENSE_WGRAD=slab, default) or added into dW with fp32 atomics (=atomic); the conv
# weight gradients' MLC_WGRAD_SLAB counterpart for dense layers.  Interleaved A/B on one
# MI355X (profiles/round6/dense_wgrad_ab.jsonl): BERT-base slab 5,711 / 5,708 seq/s vs atomic
# 5,568 / 5,563; ViT-B/16 5,136 / 5,151 vs 5,166 / 5,165 img/s.
DENSE_WGRAD_ATOMIC = os.environ.get('MLC_DENSE_WGRAD', 'slab') == 'atomic'


def linear_wgrad_bias(dout, x, dw, db):
    """dW [O, I] += dout^T x and db [O] += colsum(dout) in ONE GEMM: the bias gradient is
    summed from dout's tiles as the wgrad kernel stages them (``mlc_linear_wgrad_bias``)."""
    B, O = dout.shape
    I = x.shape[1]
    if _cuda(dout) and B % 8:
        # the GEMM reduces over the rows in 8-row chunks: zero rows add nothing (PSPNet's
        # 1x1 pyramid level has batch x 1 x 1 rows)
        pad = 8 - B % 8
        dout = torch.nn.functional.pad(dout, (0, 0, 0, pad))
        x = torch.nn.functional.pad(x, (0, 0, 0, pad))
        B += pad
    if _cuda(dout):
        assert dout.is_contiguous() and x.is_contiguous() and x.shape[0] == B
        assert tuple(dw.shape) == (O, I) and dw.is_contiguous() and db.numel() == O
        from .transformer import gemm_workspace
        if DENSE_WGRAD_ATOMIC:       # split-K partial tiles added straight into dW (fp32 atomics)
            ws, nws = None, 0
        else:                        # split-K slabs (<= 8 splits) + a reduction pass
            ws = gemm_workspace(dout.device, 8 * O * I)
            nws = ws.numel()
        _lib.call('mlc_linear_wgrad_bias', _lib.ptr(dout), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db), O, I, B, O, I, I,
                  0, _lib.ptr(ws), nws, _lib.stream())
        return dw, db
    dw.add_(dout.float().t() @ x.float())
    db.add_(dout.float().sum(0))
    return dw, db


def colsum(g, out):
    R, Cc = g.shape
    if _cuda(g):
        _lib.call('mlc_colsum', _lib.ptr(g), _lib.ptr(out), R, Cc, _lib.stream())
        return out
    out.copy_(g.float().sum(0))
    return out


# ---------------------------------------------------------------- loss
def softmax_ce(logits, labels, loss_sum, correct=None, scale=None, smoothing=0.0, want_grad=True,
               num_classes=None):
    """Fused softmax cross-entropy over the first ``num_classes`` columns of ``logits``
    ([B, ld], extra columns are padding).  Accumulates the summed loss (and #correct)
    into fp32 scalars; returns bf16 dlogits [B, ld] = (softmax - target) * scale
    (scale defaults to 1/B), zero in the padding columns."""
    B, ld = logits.shape
    V = num_classes or ld
    scale = (1.0 / B) if scale is None else scale
    if _cuda(logits):
        dl = torch.empty(B, ld, device=logits.device, dtype=torch.bfloat16) if want_grad else None
        _lib.call('mlc_softmax_ce', _lib.ptr(logits), _lib.ptr(labels), _lib.ptr(dl), _lib.ptr(loss_sum),
                  _lib.ptr(correct), B, V, ld, float(scale), float(smoothing), _lib.stream())
        return dl
    lf = logits.float()[:, :V]
    lse = torch.logsumexp(lf, 1)
    nll = lse - lf.gather(1, labels[:, None])[:, 0]
    sm = lse - lf.mean(1)
    loss_sum.add_(((1 - smoothing) * nll + smoothing * sm).sum())
    if correct is not None:
        correct.add_((lf.argmax(1) == labels).float().sum())
    if not want_grad:
        return None
    p = torch.softmax(lf, 1)
    tgt = torch.full_like(p, smoothing / V)
    tgt.scatter_add_(1, labels[:, None], torch.full((B, 1), 1 - smoothing, dtype=p.dtype))
    g = torch.zeros(B, ld)
    g[:, :V] = (p - tgt) * scale
    return g.to(torch.bfloat16)


# ---------------------------------------------------------------- layout helpers
def nchw_to_nhwc(x, pad_to=None):
    N, C, H, W = x.shape
    Cp = pad_to or C
    if _cuda(x) and x.dtype == torch.float32:
        y = torch.empty(N, H, W, Cp, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_nchw_to_nhwc', _lib.ptr(x.contiguous()), _lib.ptr(y), N, C, H * W, Cp, _lib.stream())
        return y
    y = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    if Cp != C:
        y = F.pad(y, (0, Cp - C))
    return y.contiguous()


# ---------------------------------------------------------------- optimizers
def sgd_step(p, g, m, pbf, hyper, ndecay, nbf, momentum=0.9, dampening=0.0, wd=0.0,
             nesterov=False, first=False):
    n = p.numel()
    if _cuda(p):
        _lib.call('mlc_sgd', _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(pbf), _lib.ptr(hyper), n,
                  ndecay, nbf, float(momentum), float(dampening), float(wd), int(nesterov), int(first),
                  _lib.stream())
        return
    lr, gs = float(hyper[0]), float(hyper[1])
    d = g * gs
    wdv = torch.zeros_like(p)
    wdv[:ndecay] = wd
    d = d + wdv * p
    if momentum:
        if first:
            m.copy_(d)
        else:
            m.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d + momentum * m if nesterov else m
    p.sub_(lr * d)
    if pbf is not None and nbf:
        pbf[:nbf].copy_(p[:nbf].to(torch.bfloat16))


def adam_step(p, g, m, v, pbf, hyper, ndecay, nbf, b1=0.9, b2=0.999, eps=1e-8, wd=0.0,
              decoupled=True):
    n = p.numel()
    if _cuda(p):
        _lib.call('mlc_adam', _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), _lib.ptr(pbf),
                  _lib.ptr(hyper), n, ndecay, nbf, float(b1), float(b2), float(eps), float(wd),
                  int(decoupled), _lib.stream())
        return
    lr, gs, bc1, bc2 = [float(h) for h in hyper[:4]]
    d = g * gs
    wdv = torch.zeros_like(p)
    wdv[:ndecay] = wd
    if not decoupled:
        d = d + wdv * p
    m.mul_(b1).add_((1 - b1) * d)
    v.mul_(b2).add_((1 - b2) * d * d)
    # torch.optim.Adam(W)'s form (csrc/kernels/optim.hip adam_kernel computes the same)
    upd = m / (v.sqrt() / math.sqrt(bc2) + eps)
    if decoupled:
        p.sub_(lr * wdv * p)
    p.sub_((lr / bc1) * upd)
    if pbf is not None and nbf:
        pbf[:nbf].copy_(p[:nbf].to(torch.bfloat16))


def sqnorm(x, out, scale=1.0):
    if _cuda(x):
        _lib.call('mlc_sqnorm', _lib.ptr(x), x.numel(), _lib.ptr(out), float(scale), _lib.stream())
        return out
    out.add_(((x * scale) ** 2).sum())
    return out


# ---------------------------------------------------------------- generic engine ops
# Activation codes of csrc/kernels/normact.hip (and the dense GEMM epilogue's ReLU = 3)
ACT = {'identity': 0, 'relu': 1, 'relu6': 2, 'silu': 3, 'sigmoid': 4, 'tanh': 5, 'hardswish': 6,
       'leaky_relu': 7, 'gelu': 8, 'elu': 9, 'hardsigmoid': 10}


def act_ref(a: torch.Tensor, act: int, alpha: float = 0.0) -> torch.Tensor:
    """fp32 reference of the activation codes (the CPU path of the native ops)."""
    if act == 1:
        return a.clamp_min(0)
    if act == 2:
        return a.clamp(0, 6)
    if act == 3:
        return a * torch.sigmoid(a)
    if act == 4:
        return torch.sigmoid(a)
    if act == 5:
        return torch.tanh(a)
    if act == 6:
        return F.hardswish(a)
    if act == 7:
        return torch.where(a > 0, a, alpha * a)
    if act == 8:
        return F.gelu(a)
    if act == 9:
        return torch.where(a > 0, a, alpha * (torch.exp(a) - 1))
    if act == 10:
        return F.hardsigmoid(a)
    return a


def act_grad_ref(a: torch.Tensor, act: int, alpha: float = 0.0) -> torch.Tensor:
    """d act / d a (torch's conventions at the kinks: ReLU'(0) = 0, as normact.hip)."""
    if act == 0:
        return torch.ones_like(a)
    if act == 1:
        return (a > 0).float()
    if act == 2:
        return ((a > 0) & (a < 6)).float()
    if act == 7:
        return torch.where(a > 0, torch.ones_like(a), torch.full_like(a, alpha))
    if act == 9:
        return torch.where(a > 0, torch.ones_like(a), alpha * torch.exp(a))
    if act == 10:
        return ((a > -3) & (a < 3)).float() / 6
    if act == 6:
        return torch.where(a < -3, torch.zeros_like(a), torch.where(a <= 3, (2 * a + 3) / 6, torch.ones_like(a)))
    with torch.enable_grad():
        x = a.detach().requires_grad_()
        (g,) = torch.autograd.grad(act_ref(x, act, alpha).sum(), x)
    return g


def _nchw(x):
    return x.permute(0, 3, 1, 2).float()


def gconv_block_kb(Cout: int, Cog: int, Cg: int) -> int:
    """K-side channels per tap of the grouped-conv kernels (csrc/kernels/gconv.hip block_kb):
    the widest 8-aligned K-side span of a 16-channel output block, rounded up to 16."""
    kb = 16
    for oc0 in range(0, Cout, 16):
        last = min(oc0 + 15, Cout - 1) // Cog
        lo = (oc0 // Cog) * Cg & ~7
        kb = max(kb, (((last + 1) * Cg + 7) & ~7) - lo)
    return (kb + 15) // 16 * 16


def gconv_ok(C: int, Co: int, groups: int) -> bool:
    """Shapes the grouped-conv kernels take (any group widths; channels % 8; bounded waste)."""
    if groups < 2 or C % groups or Co % groups or C % 8 or Co % 8:
        return False
    return gconv_block_kb(Co, Co // groups, C // groups) <= 256 and gconv_block_kb(C, C // groups, Co // groups) <= 256


def gconv_fwd(x, w, groups, stride=1, pad=0, dil=1, stats=None):
    """Grouped conv (groups > 1, C/groups == Co/groups): x [N,H,W,C] bf16, w [Co,KH,KW,Cg] bf16
    -> y [N,Ho,Wo,Co] bf16 on the 16x16x32 MFMA kernel (gconv.hip); ``stats`` as conv2d_fwd."""
    N, H, W, C = x.shape
    Co, KH, KW, Cg = w.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, pad, dil)
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.bfloat16)
        wb = torch.empty(int(_lib.load().mlc_gconv_wb_elems(C, Co, KH, KW, groups, 0)), device=x.device,
                         dtype=torch.bfloat16)
        s1, s2 = stats if stats is not None else (None, None)
        _lib.call('mlc_gconv_fwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(wb), _lib.ptr(y), _lib.ptr(s1), _lib.ptr(s2),
                  N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo, groups, _lib.stream())
        return y
    yf = F.conv2d(_nchw(x), w.permute(0, 3, 1, 2).float(), None, stride, pad, dil, groups)
    if stats is not None:
        stats[0][:Co].add_(yf.sum(dim=(0, 2, 3)))
        stats[1][:Co].add_((yf * yf).sum(dim=(0, 2, 3)))
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def gconv_dgrad(dy, w, x_shape, groups, stride=1, pad=0, dil=1):
    N, H, W, C = x_shape
    Co, KH, KW, Cg = w.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        wb = torch.empty(int(_lib.load().mlc_gconv_wb_elems(C, Co, KH, KW, groups, 1)), device=dy.device,
                         dtype=torch.bfloat16)
        _lib.call('mlc_gconv_dgrad', _lib.ptr(dy), _lib.ptr(w), _lib.ptr(wb), _lib.ptr(dx), N, H, W, C, Co, KH, KW,
                  stride, pad, dil, Ho, Wo, groups, _lib.stream())
        return dx
    dxf = torch.nn.grad.conv2d_input((N, C, H, W), w.permute(0, 3, 1, 2).float(), _nchw(dy), stride, pad, dil,
                                     groups)
    return dxf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def gconv_wgrad(dy, x, w_shape, groups, stride=1, pad=0, dil=1, out=None, accumulate=False):
    """fp32 [Co, KH, KW, Cg] weight gradient (written into / added to ``out``)."""
    Co, KH, KW, Cg = w_shape
    N, H, W, C = x.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dw = out if out is not None else torch.empty(Co, KH, KW, Cg, device=dy.device, dtype=torch.float32)
        _lib.call('mlc_gconv_wgrad', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dw), N, H, W, C, Co, KH, KW, stride, pad,
                  dil, Ho, Wo, groups, int(accumulate), _lib.stream())
        return dw
    g = torch.nn.grad.conv2d_weight(_nchw(x), (Co, Cg, KH, KW), _nchw(dy), stride, pad, dil, groups)
    g = g.permute(0, 2, 3, 1)
    if out is None:
        return g.contiguous()
    if accumulate:
        out.add_(g.reshape(out.shape))
    else:
        out.copy_(g.reshape(out.shape))
    return out


def dwconv_fwd(x, w, stride=1, pad=0, dil=1, stats=None):
    """Depthwise conv: x [N,H,W,C] bf16, w [KH,KW,C] bf16 (tap-major) -> y [N,Ho,Wo,C]."""
    N, H, W, C = x.shape
    KH, KW, _ = w.shape
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, pad, dil)
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.bfloat16)
        s1, s2 = stats if stats is not None else (None, None)
        _lib.call('mlc_dwconv_fwd', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(s1), _lib.ptr(s2), N, H, W, C,
                  KH, KW, stride, pad, dil, Ho, Wo, _lib.stream())
        return y
    yf = F.conv2d(_nchw(x), w.permute(2, 0, 1)[:, None].float(), None, stride, pad, dil, C)
    if stats is not None:
        stats[0][:C].add_(yf.sum(dim=(0, 2, 3)))
        stats[1][:C].add_((yf * yf).sum(dim=(0, 2, 3)))
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def dwconv_dgrad(dy, w, x_shape, stride=1, pad=0, dil=1):
    N, H, W, C = x_shape
    KH, KW, _ = w.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dx = torch.empty(N, H, W, C, device=dy.device, dtype=torch.bfloat16)
        _lib.call('mlc_dwconv_dgrad', _lib.ptr(dy), _lib.ptr(w), _lib.ptr(dx), N, H, W, C, KH, KW, stride, pad, dil,
                  Ho, Wo, _lib.stream())
        return dx
    dxf = torch.nn.grad.conv2d_input((N, C, H, W), w.permute(2, 0, 1)[:, None].float(), _nchw(dy), stride, pad,
                                     dil, C)
    return dxf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def dwconv_wgrad(dy, x, w_shape, stride=1, pad=0, dil=1, out=None, accumulate=False):
    """fp32 [KH, KW, C] depthwise weight gradient."""
    KH, KW, C = w_shape
    N, H, W, _ = x.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dw = out if out is not None else torch.empty(KH, KW, C, device=dy.device, dtype=torch.float32)
        ws = slab_workspace(dy.device, 32 * KH * KW * C)
        _lib.call('mlc_dwconv_wgrad', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(ws), N, H, W, C, KH, KW,
                  stride, pad, dil, Ho, Wo, int(accumulate), _lib.stream())
        return dw
    g = torch.nn.grad.conv2d_weight(_nchw(x), (C, 1, KH, KW), _nchw(dy), stride, pad, dil, C)
    g = g[:, 0].permute(1, 2, 0)
    if out is None:
        return g.contiguous()
    if accumulate:
        out.add_(g)
    else:
        out.copy_(g)
    return out


def conv2d_fwd_ex(x, w, bias=None, act=0, stride=1, pad=0, dil=1):
    """y = act(conv(x, w) + bias) (dense epilogue; act 0 or 3 = ReLU); groups == 1."""
    N, H, W, C = x.shape
    Co, KH, KW, Ci = w.shape
    assert Ci == C, (w.shape, x.shape)
    Ho, Wo = conv_out_hw(H, W, KH, KW, stride, pad, dil)
    if _cuda(x):
        y = torch.empty(N, Ho, Wo, Co, device=x.device, dtype=torch.bfloat16)
        _lib.call('mlc_conv_fwd_ex', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(bias), int(act), N, H, W, C, Co,
                  KH, KW, stride, pack_pad(pad), dil, Ho, Wo, _lib.stream())
        return y
    yf = F.conv2d(_nchw(x), w.permute(0, 3, 1, 2).float(), bias, stride, pad, dil)
    if act == 3:
        yf = yf.clamp_min(0)
    return yf.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()


def conv2d_wgrad_bias(dy, x, w_shape, dbias, stride=1, pad=0, dil=1, out=None, accumulate=False, slab=None):
    """fp32 weight gradient [Co, KH, KW, Ci] and dbias[Co] += colsum(dy), one GEMM."""
    Co, KH, KW, Ci = w_shape
    N, H, W, C = x.shape
    _, Ho, Wo, _ = dy.shape
    if _cuda(dy):
        dw = out if out is not None else torch.empty(Co, KH, KW, Ci, device=dy.device, dtype=torch.float32)
        use = _USE_SLAB if slab is None else slab
        ws = slab_workspace(dy.device, min(32 * Co * KH * KW * Ci, 64 << 20)) if use else None
        _lib.call('mlc_conv_wgrad_bias', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(dbias), N, H, W, C, Co,
                  KH, KW, stride, pack_pad(pad), dil, Ho, Wo, int(accumulate), _lib.ptr(ws), ws.numel() if ws is not None else 0,
                  _lib.stream())
        return dw
    dbias.add_(dy.float().sum(dim=(0, 1, 2)))
    return conv2d_wgrad(dy, x, w_shape, stride, pad, dil, out=out, accumulate=accumulate)


def zero_many(tensors):
    """Zero contiguous fp32 tensors, up to four per launch (a step's workspace and gradient
    arenas in one dispatch instead of one memset each)."""
    ts = [t for t in tensors if t is not None and t.numel()]
    if not ts:
        return
    if not _cuda(ts[0]) or any(t.dtype != torch.float32 or not t.is_contiguous() for t in ts):
        for t in ts:
            t.zero_()
        return
    for i in range(0, len(ts), 4):
        chunk = ts[i:i + 4] + [None] * (4 - len(ts[i:i + 4]))
        args = []
        for t in chunk:
            args += [_lib.ptr(t), t.numel() if t is not None else 0]
        _lib.call('mlc_zero4', *args, _lib.stream())


def rows_ld(t):
    """Row stride of an ``[..., C]`` tensor stored as rows of C contiguous elements at one fixed
    stride: C when dense, > C for the leading channels of wider rows (a DenseNet concat buffer's
    view); None for any other layout."""
    C = t.shape[-1]
    if t.dim() < 2 or t.stride(-1) != 1:
        return C if t.dim() == 1 and t.stride(-1) == 1 else None
    ld = t.stride(-2)
    want = ld
    for d in range(t.dim() - 2, -1, -1):
        if t.shape[d] != 1 and t.stride(d) != want:
            return None
        want *= t.shape[d]
    return ld if ld >= C else None


def dense_rows(t):
    """``t`` itself when its rows are dense, else a contiguous copy (for passes that read dense rows)."""
    return t if rows_ld(t) == t.shape[-1] else t.contiguous()


def bn_stats(x, s1, s2, ld=None):
    """Per-channel sum / sum of squares of NHWC x into (s1, s2) ([NSTAT*C] fp32 each, added);
    ``ld``: the copies' row stride (>= C; s1 / s2 then point at a channel offset of wider
    statistics buffers).  x may be the channel slice of wider rows (:func:`rows_ld`)."""
    C = x.shape[-1]
    rows = x.numel() // C
    if _cuda(x):
        x_ld = rows_ld(x)
        if x_ld is None:
            x, x_ld = x.contiguous(), C
        if ld is None and x_ld == C:
            _lib.call('mlc_bn_stats', _lib.ptr(x), _lib.ptr(s1), _lib.ptr(s2), rows, C, _lib.stream())
        else:
            _lib.call('mlc_bn_stats_ld', _lib.ptr(x), _lib.ptr(s1), _lib.ptr(s2), rows, C, ld or C, x_ld,
                      _lib.stream())
        return
    xf = x.float().reshape(rows, C)
    t1, t2 = (s1[0], s2[0]) if s1.dim() == 2 else (s1, s2)     # copy 0 of a strided slice
    t1[:C].add_(xf.sum(0))
    t2[:C].add_((xf * xf).sum(0))


def bn_finalize(s1, s2, rows, gamma, beta, save_mean, save_invstd, scale, shift, run_mean=None, run_var=None,
                eps=1e-5, momentum=0.1):
    """Batch statistics -> mean / invstd, the fused affine (scale, shift) and running stats."""
    C = gamma.numel()
    ncopy = s1.numel() // C
    if _cuda(s1):
        _lib.call('mlc_bn_finalize', _lib.ptr(s1), _lib.ptr(s2), ncopy, _lib.ptr(gamma), _lib.ptr(beta),
                  _lib.ptr(save_mean), _lib.ptr(save_invstd), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(run_mean),
                  _lib.ptr(run_var), rows, C, float(eps), float(momentum), _lib.stream())
        return
    mean = s1.reshape(ncopy, C).sum(0) / rows
    var = (s2.reshape(ncopy, C).sum(0) / rows - mean * mean).clamp_min(0)
    inv = torch.rsqrt(var + eps)
    save_mean.copy_(mean)
    save_invstd.copy_(inv)
    scale.copy_(inv * gamma)
    shift.copy_(beta - mean * inv * gamma)
    if run_mean is not None:
        run_mean.mul_(1 - momentum).add_(momentum * mean)
        run_var.mul_(1 - momentum).add_(momentum * var * rows / max(rows - 1, 1))


def bnact_apply(y, res, scale, shift, act=0, alpha=0.0, res_affine=None, row_scale=None):
    """z = act(y*scale + shift [* row_scale[n]] [+ res (*rscale + rshift)]) (NHWC bf16 [N, H, W, C]);
    ``row_scale`` [N] fp32: a per-sample factor of the BN output (a block's drop-path mask /
    keep), identity activation only."""
    C = y.shape[-1]
    rows = y.numel() // C
    hw = rows // y.shape[0]
    if _cuda(y):
        y = dense_rows(y)
        z = torch.empty_like(y)
        rs, rh = res_affine if res_affine is not None else (None, None)
        _lib.call('mlc_bnact_apply', _lib.ptr(y), _lib.ptr(res), _lib.ptr(z), _lib.ptr(scale), _lib.ptr(shift),
                  _lib.ptr(rs), _lib.ptr(rh), rows, C, int(act), float(alpha), _lib.ptr(row_scale), hw, _lib.stream())
        return z
    a = y.float() * scale + shift
    if row_scale is not None:
        a = a * row_scale.view(-1, *([1] * (y.dim() - 1)))
    if res is not None:
        r = res.float()
        if res_affine is not None:
            r = r * res_affine[0] + res_affine[1]
        a = a + r
    return act_ref(a, act, alpha).to(torch.bfloat16)


def bnact_fused(y, res, s1, s2, gamma, beta, mean, invstd, scale, shift, run_mean, run_var, eps, momentum, act=0,
                alpha=0.0, res_affine=None, row_scale=None, prev_tot=None, prev_c=0, tot_out=None):
    """:func:`bn_finalize` + :func:`bnact_apply` in one launch (normact.hip apply_fused_kernel):
    fills mean / invstd / scale / shift (and the running statistics) from the partial copies
    ``s1`` / ``s2`` and returns z; None when the shape does not fit (use the two calls).
    ``prev_tot`` ([2, prev_c] fp32): per-channel totals of the first ``prev_c`` channels, added
    to the copies' sums there (a DenseNet concat's older segment); ``tot_out`` ([2, C]): this
    BN's per-channel totals, published for the next BN of such a chain.  ``y`` may be the
    leading channels of wider rows (:func:`rows_ld`); z is dense."""
    C = y.shape[-1]
    ncopy = s1.numel() // C
    if not (_cuda(y) and _bn_fused_ok(C, ncopy)):
        return None
    rows = y.numel() // C
    y_ld = rows_ld(y)
    if y_ld is None:
        y, y_ld = y.contiguous(), C
    z = torch.empty(y.shape, device=y.device, dtype=y.dtype)
    rs, rh = res_affine if res_affine is not None else (None, None)
    _lib.call('mlc_bnact_fused', _lib.ptr(y), _lib.ptr(res), _lib.ptr(z), _lib.ptr(s1), _lib.ptr(s2), ncopy,
              _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(mean), _lib.ptr(invstd), _lib.ptr(scale), _lib.ptr(shift),
              _lib.ptr(run_mean), _lib.ptr(run_var), _lib.ptr(rs), _lib.ptr(rh), rows, C, float(eps), float(momentum),
              int(act), float(alpha), _lib.ptr(row_scale), rows // y.shape[0], _lib.ptr(prev_tot), int(prev_c),
              _lib.ptr(tot_out), y_ld, _lib.stream())
    return z


def bnact_bwd(dz, z, y, res, mean, scale, shift, invstd, gamma, act=0, alpha=0.0, dgamma=None, dbeta=None,
              sums=None, coef=None, want_dres=False, res_affine=None, row_scale=None, addend=None, split=None):
    """Backward of z = act(BN(y) [* row_scale[n]] [+ res (*rscale + rshift)]) with the forward's
    (scale, shift): returns (dy, dres or None) and writes dgamma / dbeta; dres is the gradient
    of the residual term (before ``res_affine``, i.e. of a folded shortcut BN's output).
    ``sums`` (NSTAT*2*C fp32) must be zero on entry.  ``addend``: another consumer's gradient of
    y added to dy in the apply pass - an NHWC tensor whose last dim may be a channel slice of
    wider rows (a DenseNet concat's gradient, row stride ``addend.stride(-2)``).  ``y`` may be
    such a slice as well (a DenseNet concat buffer's leading channels); dy / dres are dense.
    ``split`` (a multiple of 8 in (0, C)): dy comes back as two dense tensors, channels [0, split)
    and [split, C) - the gradients of a DenseNet concatenation's two operands, stored apart by
    the apply pass."""
    C = y.shape[-1]
    rows = y.numel() // C
    hw = rows // y.shape[0]
    rs, rh = res_affine if res_affine is not None else (None, None)
    add_ld = 0
    if addend is not None:
        # rows of C channels at a row stride >= C (the channel slice of a contiguous NHWC tensor)
        add_ld = rows_ld(addend)
        assert addend.shape == y.shape and add_ld is not None, (addend.shape, addend.stride())
    if _cuda(dz):
        y_ld = rows_ld(y)
        if y_ld is None:
            y, y_ld = y.contiguous(), C
        if coef is None:
            coef = torch.empty(3 * C, device=dz.device, dtype=torch.float32)
        zz = z if act in (4, 5) else None        # sigmoid / tanh read their derivative off z
        if C <= 2048:          # (fixed summation order: deterministic as well)
            # one call: reduce to per-block partial rows (no float atomics), finalize, apply
            part = slab_workspace(dz.device, 2048 * 2 * C)    # the kernel caps the blocks (MLC_NORMACT_CAP)
            dy, dy2 = _bwd_out(y, split)
            dres = torch.empty(y.shape, device=y.device, dtype=y.dtype) if want_dres else None
            _lib.call('mlc_bnact_bwd', _lib.ptr(dz), _lib.ptr(zz), _lib.ptr(y), _lib.ptr(res), _lib.ptr(mean),
                      _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(rs), _lib.ptr(rh), _lib.ptr(invstd), _lib.ptr(gamma),
                      _lib.ptr(part), part.numel(), _lib.ptr(coef), _lib.ptr(dgamma), _lib.ptr(dbeta), _lib.ptr(dy),
                      _lib.ptr(dres), rows, C, int(act), float(alpha), _lib.ptr(row_scale), hw, _lib.ptr(addend),
                      add_ld, y_ld, _lib.ptr(dy2), int(split or 0), _lib.stream())
            return (dy, dy2) if split else dy, dres
        if sums is None:
            sums = torch.zeros(NSTAT * 2 * C, device=dz.device, dtype=torch.float32)
        _lib.call('mlc_bnact_bwd_reduce', _lib.ptr(dz), _lib.ptr(zz), _lib.ptr(y), _lib.ptr(res), _lib.ptr(mean),
                  _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(rs), _lib.ptr(rh), _lib.ptr(sums), rows, C, int(act),
                  float(alpha), _lib.ptr(row_scale), hw, y_ld, _lib.stream())
        _lib.call('mlc_bn_bwd_finalize', _lib.ptr(sums), _lib.ptr(invstd), _lib.ptr(gamma), _lib.ptr(coef),
                  _lib.ptr(dgamma), _lib.ptr(dbeta), rows, C, _lib.stream())
        dy, dy2 = _bwd_out(y, split)
        dres = torch.empty(y.shape, device=y.device, dtype=y.dtype) if want_dres else None
        _lib.call('mlc_bnact_bwd_apply', _lib.ptr(dz), _lib.ptr(zz), _lib.ptr(y), _lib.ptr(res), _lib.ptr(mean),
                  _lib.ptr(coef), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(rs), _lib.ptr(rh), _lib.ptr(dy),
                  _lib.ptr(dres), rows, C, int(act), float(alpha), _lib.ptr(row_scale), hw, _lib.ptr(addend), add_ld,
                  y_ld, _lib.ptr(dy2), int(split or 0), _lib.stream())
        return (dy, dy2) if split else dy, dres
    rsc = row_scale.repeat_interleave(hw)[:, None] if row_scale is not None else None
    a = y.float().reshape(rows, C) * scale + shift
    if rsc is not None:
        a = a * rsc
    if res is not None:
        r = res.float().reshape(rows, C)
        a = a + (r * rs + rh if rs is not None else r)
    d = dz.float().reshape(rows, C)
    if act:
        if act in (4, 5):
            zf = z.float().reshape(rows, C)
            d = d * (zf * (1 - zf) if act == 4 else 1 - zf * zf)
        else:
            d = d * act_grad_ref(a, act, alpha)
    dres = d.reshape(y.shape).to(torch.bfloat16) if want_dres else None
    if rsc is not None:
        d = d * rsc
    yc = y.float().reshape(rows, C) - mean
    S1, S2 = d.sum(0), (d * yc).sum(0)
    if dgamma is not None:
        dgamma.copy_(S2 * invstd)
        dbeta.copy_(S1)
    k1 = gamma * invstd
    dyf = k1 * d - k1 * S1 / rows - k1 * invstd * invstd * S2 / rows * yc
    if addend is not None:
        dyf = dyf + addend.float().reshape(rows, C)
    dy = dyf.reshape(y.shape).to(torch.bfloat16)
    if split:
        return (dy[..., :split].contiguous(), dy[..., split:].contiguous()), dres
    return dy, dres


def _bwd_out(y, split):
    """dy of :func:`bnact_bwd`: one dense tensor, or two split at channel ``split``."""
    if not split:
        return torch.empty(y.shape, device=y.device, dtype=y.dtype), None
    C = y.shape[-1]
    assert 0 < split < C and split % 8 == 0, (split, C)
    lead = tuple(y.shape[:-1])
    return (torch.empty(*lead, split, device=y.device, dtype=y.dtype),
            torch.empty(*lead, C - split, device=y.device, dtype=y.dtype))


def act_fwd(x, act, alpha=0.0):
    if _cuda(x) and x.numel() % 8 == 0:
        y = torch.empty_like(x)
        _lib.call('mlc_act_fwd', _lib.ptr(x), _lib.ptr(y), x.numel(), int(act), float(alpha), _lib.stream())
        return y
    return act_ref(x.float(), act, alpha).to(torch.bfloat16)


def chscale_fwd(y, g, res=None, relu=False):
    """Channel gate (squeeze-excitation): act(y * g [+ res]) with y [N, H, W, C] NHWC bf16, g
    [N, C] per image and channel, an optional residual of y's shape and an optional ReLU."""
    N, H, W, C = y.shape
    if _cuda(y) and C % 8 == 0:
        out = torch.empty_like(y)
        _lib.call('mlc_chscale_fwd', _lib.ptr(y), _lib.ptr(g.contiguous()), _lib.ptr(res), _lib.ptr(out), N, H * W, C,
                  int(relu), _lib.stream())
        return out
    a = y.float() * g.float().view(N, 1, 1, C)
    if res is not None:
        a = a + res.float()
    if relu:
        a = a.clamp_min(0)
    return a.to(torch.bfloat16)


def chscale_bwd(dout, y, g, z=None, want_dres=False, addend=None):
    """(dy, dg, dres) of :func:`chscale_fwd`: the ReLU mask from its output ``z`` (if it had a
    ReLU), dres = the masked gradient (if it had a residual), dy = that * g, dg [N, C] (fp32)
    = its sum over pixels times y - one pass (float atomics per channel; deterministic mode
    sums in torch)."""
    N, H, W, C = y.shape
    if addend is not None:
        assert tuple(addend.shape) == tuple(y.shape) and addend.is_contiguous(), (addend.shape, y.shape)
    if _cuda(y) and C % 8 == 0 and not _lib.DETERMINISTIC:
        dy = torch.empty_like(y)
        dres = torch.empty_like(y) if want_dres else None
        dg = torch.zeros(N, C, device=y.device, dtype=torch.float32)
        _lib.call('mlc_chscale_bwd', _lib.ptr(dout.contiguous()), _lib.ptr(y), _lib.ptr(g.contiguous()), _lib.ptr(z),
                  _lib.ptr(addend), _lib.ptr(dy), _lib.ptr(dres), _lib.ptr(dg), N, H * W, C, _lib.stream())
        return dy, dg, dres
    d = dout.float()
    if z is not None:
        d = d * (z.float() > 0)
    dres = d.to(torch.bfloat16) if want_dres else None
    dyf = d * g.float().view(N, 1, 1, C)
    if addend is not None:
        dyf = dyf + addend.float()
    return dyf.to(torch.bfloat16), (d * y.float()).sum((1, 2)), dres


def act_bwd(dy, x, y, act, alpha=0.0):
    if _cuda(dy) and dy.numel() % 8 == 0:
        dx = torch.empty_like(dy)
        _lib.call('mlc_act_bwd', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(y), _lib.ptr(dx), dy.numel(), int(act),
                  float(alpha), _lib.stream())
        return dx
    if act in (4, 5):
        yf = y.float()
        g = yf * (1 - yf) if act == 4 else 1 - yf * yf
    else:
        g = act_grad_ref(x.float(), act, alpha)
    return (dy.float() * g).to(torch.bfloat16)
