"""Transformer sites of the generic native engine (:mod:`mlcomp_amd.models.native_generic`).

The reference trains whatever model the experiment returns
(`mlcomp/worker/executors/catalyst_/catalyst_.py:365-372`), including any ``timm`` model
(`mlcomp/contrib/model/timm.py:8-10`: ViT, DeiT, Swin ...).  The hand BERT engine
(:mod:`mlcomp_amd.models.native_bert`) reaches the transformer kernels for one architecture;
these sites reach them from a torch.fx graph of ANY model:

* ``nn.LayerNorm`` [after a residual add]      -> :class:`LayerNormSite`: ``transformer.hip``
  LayerNorm forward / backward (the residual add fused into the normalisation pass);
* ``nn.MultiheadAttention`` (self-attention)   -> :class:`MHASite`: packed in-projection GEMM,
  the fused flash attention (``flash_attn.hip``, any S, head dim <= 128, key-padding
  mask as a key bias), out-projection GEMM;
* ``nn.TransformerEncoderLayer`` / ``nn.TransformerEncoder`` -> :class:`EncoderSite`: the
  whole layer as one autograd node (post-norm or pre-norm, ReLU or exact GELU, all three
  dropouts on the kernels' counter-hash masks), scheduled like the hand BERT engine:
  dropout + residual fused into the LayerNorm passes, GELU'(pre-activation) stored by the
  FFN GEMM epilogue and multiplied in the next input-gradient epilogue, weight gradients
  on the side stream;
* ``F.scaled_dot_product_attention`` (no mask, not causal) -> :class:`SDPASite`: q/k/v packed
  into the kernel's [B*S, 3*H*D] layout, flash attention forward / backward;
* ``Linear -> GELU`` -> a dense GEMM with the GELU in its epilogue (:class:`LinearGelu`).

Every GEMM is the framework's own MFMA kernel (``igemm.hip`` dense epilogues): no hipBLASLt,
rocBLAS or MIOpen call.  Each site has the fp32 PyTorch path of its ops on CPU (the
:mod:`~mlcomp_amd.ops.transformer` references), which the CPU tests compare with torch
autograd.
"""
from __future__ import annotations

import math
from types import SimpleNamespace
from typing import List, Optional

import torch
import torch.nn as nn

from . import functional as Fn
from . import transformer as Tx
from .glayers import Site, _freeze, _run, _Uses
from .layers import NativeContext


def _seed(ctx):
    return getattr(ctx, 'seed', None)


def next_salt(ctx) -> int:
    """A dropout-mask salt no other site of this model uses (the kernels' masks are a hash
    of (seed, salt, element index); the seed advances every training step)."""
    s = getattr(ctx, '_salt', 1000)
    ctx._salt = s + 8
    return s


# ---------------------------------------------------------------------------- parameters
class DenseSet:
    """A dense layer's weight [O, I] (bf16 mirror in the decay arena) and optional bias [O]:
    an ``nn.Linear`` or MultiheadAttention's packed in-projection.  ``backward`` is the hand
    BERT engine's schedule: input gradient first, weight + bias gradient (one GEMM) forked to
    the side stream."""

    def __init__(self, ctx: NativeContext, name: str, weight: torch.Tensor, bias: Optional[torch.Tensor]):
        self.ctx, self.name = ctx, name
        self.src = SimpleNamespace(weight=weight, bias=bias)
        self.O, self.I = int(weight.shape[0]), int(weight[0].numel())     # conv filters flatten to [O, C*k*k]
        self.w = ctx.arena.weight(f'{name}.weight', (self.O, self.I))
        self.b = ctx.arena.vector(f'{name}.bias', (self.O,)) if bias is not None else None
        _freeze(self.w, weight)
        _freeze(self.b, bias)
        self.uses = _Uses()

    def load_from_torch(self):
        dev = self.ctx.device
        self.w.master.copy_(self.src.weight.detach().float().reshape(self.O, self.I).to(dev))
        if self.b is not None:
            self.b.master.copy_(self.src.bias.detach().float().to(dev))

    def export_to_torch(self):
        w = self.src.weight
        w.data.copy_(self.w.master.view(w.shape).to(w.device, w.dtype))
        if self.b is not None:
            b = self.src.bias
            b.data.copy_(self.b.master.to(b.device, b.dtype))

    def mark_ready(self):
        self.ctx.arena.mark_ready(self.w)
        if self.b is not None:
            self.ctx.arena.mark_ready(self.b)

    def fwd(self, x, act=0, want_preact=False):
        return Tx.dense_fwd(x, self.w.bf16, self.b.master if self.b is not None else None, act, want_preact)

    def backward(self, dy, x, dact_u=None, addend=None, dact_is_deriv=False, need_dx=True):
        """dx = dy @ W [* dact_u] [+ addend] (returned); dW += dy^T x, db += colsum(dy)."""
        dx = dense_backward(self.ctx, self.w, self.b, dy, x, dact_u=dact_u, addend=addend,
                            dact_is_deriv=dact_is_deriv, need_dx=need_dx)
        if self.uses.bwd_done():
            self.mark_ready()
        return dx


def _wgrad(w, b, dy, x):
    if b is not None and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0:
        Fn.linear_wgrad_bias(dy, x, w.grad, b.grad)
    else:
        Fn.linear_wgrad(dy, x, out=w.grad, accumulate=True)
        if b is not None:
            Tx.colsum_acc(dy, b.grad) if dy.shape[1] % 8 == 0 else b.grad.add_(dy.float().sum(0))


def dense_backward(ctx, w, b, dy, x, dact_u=None, addend=None, dact_is_deriv=False, need_dx=True):
    """A dense layer's backward with the hand BERT engine's schedule: the input gradient
    dx = dy @ W [* dact_u] [+ addend] on the main stream first, the weight + bias gradient
    (one GEMM) forked onto the side stream from the point before it (unjoined with
    ``ctx.wgrad_defer``: one free-running chain joined before the optimizer)."""
    side = ctx.wgrad_stream
    dx = None
    if side is None:
        if need_dx:
            dx = Tx.dense_dgrad(dy, w.bf16, dact_u=dact_u, addend=addend, dact_is_deriv=dact_is_deriv)
        _wgrad(w, b, dy, x)
        return dx
    main = torch.cuda.current_stream(ctx.device)
    fork = torch.cuda.Event()
    fork.record(main)
    if need_dx:
        dx = Tx.dense_dgrad(dy, w.bf16, dact_u=dact_u, addend=addend, dact_is_deriv=dact_is_deriv)
    side.wait_event(fork)
    with Fn.side_stream(side):
        _wgrad(w, b, dy, x)
    dy.record_stream(side)
    x.record_stream(side)
    if not ctx.wgrad_defer:
        main.wait_stream(side)
    return dx


class LNParams:
    """``nn.LayerNorm`` over the last dimension (affine, with bias) -> gamma / beta slots."""

    def __init__(self, ctx: NativeContext, name: str, ln: nn.LayerNorm):
        self.ctx, self.name, self.src = ctx, name, ln
        self.H = int(ln.normalized_shape[-1])
        self.eps = float(ln.eps)
        self.g = ctx.arena.vector(f'{name}.weight', (self.H,))
        self.b = ctx.arena.vector(f'{name}.bias', (self.H,))
        _freeze(self.g, ln.weight)
        _freeze(self.b, ln.bias)
        self.uses = _Uses()

    @staticmethod
    def supported(ln) -> Optional[str]:
        if not isinstance(ln, nn.LayerNorm) or len(ln.normalized_shape) != 1:
            return 'LayerNorm over more than the last dimension'
        if not ln.elementwise_affine or ln.bias is None:
            return 'LayerNorm without affine weight and bias'
        if ln.normalized_shape[0] % 8:
            return f'LayerNorm width {ln.normalized_shape[0]} (native: a multiple of 8)'
        return None

    def load_from_torch(self):
        dev = self.ctx.device
        self.g.master.copy_(self.src.weight.detach().float().to(dev))
        self.b.master.copy_(self.src.bias.detach().float().to(dev))

    def export_to_torch(self):
        ln = self.src
        ln.weight.data.copy_(self.g.master.to(ln.weight.device, ln.weight.dtype))
        ln.bias.data.copy_(self.b.master.to(ln.bias.device, ln.bias.dtype))

    def mark_ready(self):
        self.ctx.arena.mark_ready(self.g)
        self.ctx.arena.mark_ready(self.b)

    def fwd(self, x, r=None, p_in=0.0, salt_in=0):
        return Tx.ln_fwd(x, r, self.g.master, self.b.master, self.eps, p_in=p_in, seed=_seed(self.ctx),
                         salt_in=salt_in)

    def bwd(self, dy, s, mean, rstd, sums, want_dr=False, p_in=0.0, salt_in=0):
        out = Tx.ln_bwd(dy, s, mean, rstd, self.g.master, self.g.grad, self.b.grad, sums, p_in=p_in,
                        seed=_seed(self.ctx), salt_in=salt_in, want_dr=want_dr)
        if self.uses.bwd_done():
            self.mark_ready()
        return out


def _rows(x: torch.Tensor) -> torch.Tensor:
    """[..., H] -> contiguous bf16 [T, H]."""
    x2 = x.reshape(-1, x.shape[-1])
    if x2.dtype != torch.bfloat16:
        x2 = x2.to(torch.bfloat16)
    return x2.contiguous()


# ---------------------------------------------------------------------------- LayerNorm
class LayerNormSite(Site):
    """``LN(x [+ r])`` over the last dimension; with ``r`` the residual add is fused into
    the normalisation pass and both inputs get the same gradient."""

    def __init__(self, ctx, ln: LNParams, residual: bool = False):
        super().__init__(ctx)
        object.__setattr__(self, 'ln', ln)
        self.residual = residual
        self.k_sums = ctx.ws.request(f'{ln.name}@{id(self)}.sums', Fn.NSTAT * 2 * ln.H)

    def params(self):
        return [self.ln]

    def forward(self, x, r=None):
        return _run(self, x, r) if r is not None else _run(self, x)

    def fwd(self, x, r=None):
        shape = x.shape if r is None else torch.broadcast_shapes(x.shape, r.shape)
        x2 = _rows(x.expand(shape))
        r2 = _rows(r.expand(shape)) if r is not None else None
        y, s, mean, rstd = self.ln.fwd(x2, r2)
        return y.view(shape), [s, mean, rstd], (shape, x.dtype, None if r is None else (r.shape, r.dtype))

    def bwd(self, dout, saved, keep, needs):
        s, mean, rstd = saved
        shape, xdt, rkeep = keep
        ds, _ = self.ln.bwd(_rows(dout), s, mean, rstd, self.ctx.ws[self.k_sums])
        ds = ds.view(shape)
        out = [_reduce_to(ds, shape, xdt) if needs[0] else None]
        if rkeep is not None:
            out.append(_reduce_to(ds, rkeep[0], rkeep[1]) if needs[1] else None)
        return out


def _reduce_to(g: torch.Tensor, shape, dtype) -> torch.Tensor:
    """A broadcast input's gradient: sum over the broadcast dimensions."""
    if tuple(g.shape) != tuple(shape):
        lead = g.dim() - len(shape)
        dims = [i for i in range(g.dim()) if i < lead or (shape[i - lead] == 1 and g.shape[i] != 1)]
        g = g.float().sum(dims, keepdim=True)
        g = g.reshape(shape)
    return g.to(dtype)


# ---------------------------------------------------------------------------- attention core
class _Attn:
    """The attention math shared by the MHA / encoder sites: qkv [B*S, 3*E] (q | k | v,
    head h at columns h*D) -> context [B*S, E]."""

    def __init__(self, ctx, heads: int, E: int, p: float):
        self.ctx, self.H, self.E, self.p = ctx, heads, E, float(p)
        self.D = E // heads
        self.scale = 1.0 / math.sqrt(self.D)
        self.salt = next_salt(ctx)

    def p_now(self):
        return self.p if self.ctx.training else 0.0

    def fwd(self, qkv, kb, B, S):
        return Tx.attn_fwd(qkv, kb, B, S, self.H, self.scale, self.p_now(), _seed(self.ctx), self.salt,
                           head_dim=self.D)

    def bwd(self, qkv, kb, dctx, lse, ctx2, B, S):
        return Tx.attn_bwd(qkv, kb, dctx.contiguous(), lse, B, S, self.H, self.scale, self.p_now(),
                           _seed(self.ctx), self.salt, head_dim=self.D, ctx=ctx2)


def key_bias_of(mask: Optional[torch.Tensor], B: int, S: int) -> Optional[torch.Tensor]:
    """``key_padding_mask`` ([B, S]; True / nonzero = padding, or an additive float mask) ->
    the kernels' fp32 key bias (0 / -inf)."""
    if mask is None:
        return None
    if mask.dtype == torch.bool:
        kb = torch.zeros(B, S, device=mask.device, dtype=torch.float32).masked_fill(mask, float('-inf'))
    else:
        kb = mask.float()
    return kb.contiguous()


def mha_supported(m: nn.MultiheadAttention) -> Optional[str]:
    if not m._qkv_same_embed_dim or m.bias_k is not None or m.bias_v is not None or m.add_zero_attn:
        return 'MultiheadAttention with separate k/v dims, bias_k/bias_v or add_zero_attn'
    E, H = m.embed_dim, m.num_heads
    if E % 8:
        return f'MultiheadAttention embed_dim {E} (native: a multiple of 8)'
    if not Tx.attn_supported(1, E // H):
        return f'MultiheadAttention head dim {E // H} (the fused attention takes <= 128)'
    return None


class MHAParams:
    """nn.MultiheadAttention -> in-projection [3E, E] and out-projection [E, E] dense sets
    (``dense(name, weight, bias)`` makes / shares them: the net's parameter registry)."""

    def __init__(self, dense, name: str, m: nn.MultiheadAttention):
        self.src = m
        self.inp = dense(f'{name}.in_proj', m.in_proj_weight, m.in_proj_bias)
        self.out = dense(f'{name}.out_proj', m.out_proj.weight, m.out_proj.bias)
        self.E, self.heads, self.p = m.embed_dim, m.num_heads, float(m.dropout)
        self.batch_first = bool(m.batch_first)

    def parts(self):
        return [self.inp, self.out]


class MHASite(Site):
    """Self-attention ``mha(x, x, x, key_padding_mask=...)[0]``: in-projection GEMM, flash
    attention, out-projection GEMM.  Sequence-first inputs ([S, B, E]) are transposed to
    batch-first rows on the way in and viewed back on the way out."""

    def __init__(self, ctx, mp: MHAParams):
        super().__init__(ctx)
        object.__setattr__(self, 'mp', mp)
        object.__setattr__(self, 'attn', _Attn(ctx, mp.heads, mp.E, mp.p))

    def params(self):
        return [self.mp.inp, self.mp.out]

    def forward(self, x, kpm=None):
        return _run(self, x, kpm) if kpm is not None else _run(self, x)

    def fwd(self, x, kpm=None):
        mp = self.mp
        if mp.batch_first:
            B, S, E = x.shape
            x2 = _rows(x)
        else:
            S, B, E = x.shape
            x2 = _rows(x.transpose(0, 1))
        kb = key_bias_of(kpm, B, S)
        qkv, _ = mp.inp.fwd(x2)
        ctx2, lse = self.attn.fwd(qkv, kb, B, S)
        out, _ = mp.out.fwd(ctx2)
        y = out.view(B, S, E)
        if not mp.batch_first:
            y = y.transpose(0, 1)
        saved = [x2, qkv, lse, ctx2] + ([kb] if kb is not None else [])
        return y, saved, (B, S, x.dtype, kb is not None)

    def bwd(self, dout, saved, keep, needs):
        mp = self.mp
        B, S, xdt, has_kb = keep
        x2, qkv, lse, ctx2 = saved[:4]
        kb = saved[4] if has_kb else None
        d = dout if mp.batch_first else dout.transpose(0, 1)
        dctx = mp.out.backward(_rows(d), ctx2)
        dqkv = self.attn.bwd(qkv, kb, dctx, lse, ctx2, B, S)
        dx = mp.inp.backward(dqkv, x2, need_dx=needs[0])
        out = [None]
        if dx is not None:
            dx = dx.view(B, S, -1)
            out[0] = (dx if mp.batch_first else dx.transpose(0, 1)).to(xdt)
        if len(needs) > 1:
            out.append(None)
        return out


# ---------------------------------------------------------------------------- encoder layers
def encoder_layer_supported(layer: nn.TransformerEncoderLayer) -> Optional[str]:
    why = mha_supported(layer.self_attn)
    if why:
        return why
    act = getattr(layer, 'activation_relu_or_gelu', 0)
    if act not in (1, 2):
        return f'TransformerEncoderLayer activation {layer.activation!r} (native: relu / exact gelu)'
    if act == 2 and isinstance(layer.activation, nn.GELU) and layer.activation.approximate != 'none':
        return 'TransformerEncoderLayer tanh-approximate GELU'
    for ln in (layer.norm1, layer.norm2):
        why = LNParams.supported(ln)
        if why:
            return why
    if layer.linear1.bias is None or layer.linear2.bias is None:
        return 'TransformerEncoderLayer without biases'
    if layer.linear1.out_features % 8:
        return f'TransformerEncoderLayer dim_feedforward {layer.linear1.out_features} (native: a multiple of 8)'
    return None


class EncoderLayerParams:
    def __init__(self, dense, lnp, name: str, layer: nn.TransformerEncoderLayer):
        self.src = layer
        self.mha = MHAParams(dense, f'{name}.self_attn', layer.self_attn)
        self.ffn1 = dense(f'{name}.linear1', layer.linear1.weight, layer.linear1.bias)
        self.ffn2 = dense(f'{name}.linear2', layer.linear2.weight, layer.linear2.bias)
        self.ln1 = lnp(f'{name}.norm1', layer.norm1)
        self.ln2 = lnp(f'{name}.norm2', layer.norm2)
        self.norm_first = bool(layer.norm_first)
        self.gelu = layer.activation_relu_or_gelu == 2
        self.p_ff, self.p1, self.p2 = float(layer.dropout.p), float(layer.dropout1.p), float(layer.dropout2.p)
        self.batch_first = bool(layer.self_attn.batch_first)

    def parts(self):
        return self.mha.parts() + [self.ffn1, self.ffn2, self.ln1, self.ln2]


class NativeEncoderLayer:
    """One nn.TransformerEncoderLayer on the kernels (rows [B*S, E] bf16 in and out)."""

    def __init__(self, ctx, lp: EncoderLayerParams):
        self.ctx, self.lp = ctx, lp
        self.attn = _Attn(ctx, lp.mha.heads, lp.mha.E, lp.mha.p)
        self.salt = next_salt(ctx)       # +0 dropout1, +1 ffn dropout, +2 dropout2
        self.k1 = ctx.ws.request(f'{lp.ln1.name}@{id(self)}.sums', Fn.NSTAT * 2 * lp.ln1.H)
        self.k2 = ctx.ws.request(f'{lp.ln2.name}@{id(self)}.sums', Fn.NSTAT * 2 * lp.ln2.H)

    def _p(self, p):
        return p if self.ctx.training else 0.0

    def _ffn_fwd(self, h):
        """FFN up-projection + activation + dropout: (g_dropped, multiplier) where the
        backward's input gradient of the down-projection is multiplied by ``multiplier``
        (gelu'(pre-activation) or the ReLU mask, times the dropout mask) in its epilogue."""
        lp = self.lp
        if lp.gelu:
            g, m = lp.ffn1.fwd(h, act=2, want_preact=True)      # m = gelu'(pre-activation)
        else:
            z, _ = lp.ffn1.fwd(h)
            g = torch.relu(z)
            m = (z > 0).to(torch.bfloat16)
        p = self._p(lp.p_ff)
        if p > 0:
            seed = _seed(self.ctx)
            g = Tx.dropout(g, p, seed, self.salt + 1)
            m = Tx.dropout(m, p, seed, self.salt + 1)          # same mask and scale
        return g, m

    def fwd(self, x, kb, B, S):
        lp, ctx = self.lp, self.ctx
        seed = _seed(ctx)
        p1, p2 = self._p(lp.p1), self._p(lp.p2)
        if not lp.norm_first:
            qkv, _ = lp.mha.inp.fwd(x)
            ctx2, lse = self.attn.fwd(qkv, kb, B, S)
            ao, _ = lp.mha.out.fwd(ctx2)
            h1, s1, m1, r1 = lp.ln1.fwd(x, ao, p_in=p1, salt_in=self.salt)
            g, m = self._ffn_fwd(h1)
            f, _ = lp.ffn2.fwd(g)
            h2, s2, m2, r2 = lp.ln2.fwd(h1, f, p_in=p2, salt_in=self.salt + 2)
            return h2, [x, qkv, lse, ctx2, s1, m1, r1, h1, g, m, s2, m2, r2]
        n1, _, m1, r1 = lp.ln1.fwd(x)
        qkv, _ = lp.mha.inp.fwd(n1)
        ctx2, lse = self.attn.fwd(qkv, kb, B, S)
        ao, _ = lp.mha.out.fwd(ctx2)
        x1 = (x.float() + Tx.dropout(ao, p1, seed, self.salt).float()).to(torch.bfloat16)
        n2, _, m2, r2 = lp.ln2.fwd(x1)
        g, m = self._ffn_fwd(n2)
        f, _ = lp.ffn2.fwd(g)
        x2 = (x1.float() + Tx.dropout(f, p2, seed, self.salt + 2).float()).to(torch.bfloat16)
        return x2, [x, n1, m1, r1, qkv, lse, ctx2, x1, n2, m2, r2, g, m]

    def bwd(self, dy, saved, kb, B, S):
        lp, ctx = self.lp, self.ctx
        seed = _seed(ctx)
        p1, p2 = self._p(lp.p1), self._p(lp.p2)
        if not lp.norm_first:
            x, qkv, lse, ctx2, s1, m1, r1, h1, g, m, s2, m2, r2 = saved
            ds2, df = lp.ln2.bwd(dy, s2, m2, r2, ctx.ws[self.k2], want_dr=True, p_in=p2, salt_in=self.salt + 2)
            du = lp.ffn2.backward(df, g, dact_u=m, dact_is_deriv=True)
            dh1 = lp.ffn1.backward(du, h1, addend=ds2)
            ds1, dao = lp.ln1.bwd(dh1, s1, m1, r1, ctx.ws[self.k1], want_dr=True, p_in=p1, salt_in=self.salt)
            dctx = lp.mha.out.backward(dao, ctx2)
            dqkv = self.attn.bwd(qkv, kb, dctx, lse, ctx2, B, S)
            return lp.mha.inp.backward(dqkv, x, addend=ds1)
        x, n1, m1, r1, qkv, lse, ctx2, x1, n2, m2, r2, g, m = saved
        df = Tx.dropout(dy, p2, seed, self.salt + 2)
        du = lp.ffn2.backward(df, g, dact_u=m, dact_is_deriv=True)
        dn2 = lp.ffn1.backward(du, n2)
        dx1n, _ = lp.ln2.bwd(dn2, x1, m2, r2, ctx.ws[self.k2])
        dx1 = (dy.float() + dx1n.float()).to(torch.bfloat16)
        dao = Tx.dropout(dx1, p1, seed, self.salt)
        dctx = lp.mha.out.backward(dao, ctx2)
        dqkv = self.attn.bwd(qkv, kb, dctx, lse, ctx2, B, S)
        dn1 = lp.mha.inp.backward(dqkv, n1)
        dxn, _ = lp.ln1.bwd(dn1, x, m1, r1, ctx.ws[self.k1])
        return (dx1.float() + dxn.float()).to(torch.bfloat16)


class _EncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, kb, layer: NativeEncoderLayer, B, S):
        y, saved = layer.fwd(x, kb, B, S)
        ctx.layer, ctx.kb, ctx.B, ctx.S = layer, kb, B, S
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = ctx.layer.bwd(dy.contiguous(), ctx.saved_tensors, ctx.kb, ctx.B, ctx.S)
        return dx, None, None, None, None, None


class _LNFn(torch.autograd.Function):
    """A LayerNorm over rows inside an encoder stack (the stack's final norm)."""

    @staticmethod
    def forward(ctx, x, anchor, ln: LNParams, k_sums, ws):
        y, s, m, r = ln.fwd(x)
        ctx.ln, ctx.k, ctx.ws = ln, k_sums, ws
        ctx.save_for_backward(s, m, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        s, m, r = ctx.saved_tensors
        ds, _ = ctx.ln.bwd(dy.contiguous(), s, m, r, ctx.ws[ctx.k])
        return ds, None, None, None, None


class EncoderSite(nn.Module):
    """``nn.TransformerEncoderLayer`` or ``nn.TransformerEncoder`` (its layers + optional
    final norm) as native layers: ``forward(src, src_key_padding_mask=None)``."""

    def __init__(self, ctx, layers: List[EncoderLayerParams], final_norm: Optional[LNParams] = None):
        super().__init__()
        object.__setattr__(self, 'ctx', ctx)
        object.__setattr__(self, 'layers', [NativeEncoderLayer(ctx, lp) for lp in layers])
        object.__setattr__(self, 'norm', final_norm)
        self.k_norm = ctx.ws.request(f'{final_norm.name}@{id(self)}.sums', Fn.NSTAT * 2 * final_norm.H) \
            if final_norm is not None else None
        self.batch_first = layers[0].batch_first

    def forward(self, x, kpm=None):
        if self.batch_first:
            B, S, E = x.shape
            h = _rows(x)
        else:
            S, B, E = x.shape
            h = _rows(x.transpose(0, 1))
        kb = key_bias_of(kpm, B, S)
        ctx = self.ctx
        train = torch.is_grad_enabled() and ctx.training
        for layer in self.layers:
            if train:
                for p in layer.lp.parts():      # backward marks a slot after its last use
                    p.uses.fwd()
                h = _EncoderFn.apply(h, ctx.anchor, kb, layer, B, S)
            else:
                with torch.no_grad():
                    h = layer.fwd(h, kb, B, S)[0]
        if self.norm is not None:
            if train:
                self.norm.uses.fwd()
                h = _LNFn.apply(h, ctx.anchor, self.norm, self.k_norm, ctx.ws)
            else:
                with torch.no_grad():
                    h = self.norm.fwd(h)[0]
        y = h.view(B, S, E)
        return y if self.batch_first else y.transpose(0, 1)


# ---------------------------------------------------------------------------- SDPA, dense + GELU
class SDPASite(Site):
    """``F.scaled_dot_product_attention(q, k, v, dropout_p=p, scale=s)`` (no mask, not causal)
    on the flash kernels; the output is a [B, H, S, D] view of the kernel's [B*S, H*D]
    context rows (so a following ``transpose(1, 2).reshape(B, S, H*D)`` is free).

    ``heads`` set (the lowering matched timm's ``qkv(x).reshape(B, N, 3, H, D).permute(2, 0,
    3, 1, 4)`` split): the single input is the projection output [B, N, 3*H*D], which already
    is the kernel's packed layout - no copy forward, and the packed gradient is the
    projection's output gradient - no copy backward.  Otherwise q / k / v [B, H, S, D] are
    packed with one copy."""

    def __init__(self, ctx, p: float = 0.0, scale: Optional[float] = None, heads: Optional[int] = None):
        super().__init__(ctx)
        self.p, self.scale, self.heads = float(p), scale, heads
        self.salt = next_salt(ctx)

    def params(self):
        return []

    def forward(self, *qkv):
        return _run(self, *qkv)

    def fwd(self, *inputs):
        if self.heads is not None:
            (L,) = inputs
            B, S, E3 = L.shape
            H = self.heads
            D = E3 // (3 * H)
            qkv = _rows(L)
            dt = L.dtype
        else:
            q, k, v = inputs
            B, H, S, D = q.shape
            if tuple(k.shape) != (B, H, S, D) or tuple(v.shape) != (B, H, S, D):
                raise ValueError(f'SDPA site: q {tuple(q.shape)} k {tuple(k.shape)} v {tuple(v.shape)} '
                                 '(self-attention shapes expected)')
            qkv = torch.stack([t.to(torch.bfloat16) for t in (q, k, v)], 2)    # [B, H, 3, S, D]
            qkv = qkv.permute(0, 3, 2, 1, 4).reshape(B * S, 3 * H * D).contiguous()
            dt = q.dtype
        scale = self.scale if self.scale is not None else 1.0 / math.sqrt(D)
        p = self.p if self.ctx.training else 0.0
        ctx2, lse = Tx.attn_fwd(qkv, None, B, S, H, scale, p, _seed(self.ctx), self.salt, head_dim=D)
        out = ctx2.view(B, S, H, D).transpose(1, 2)
        return out, [qkv, lse, ctx2], (B, H, S, D, scale, p, dt)

    def bwd(self, dout, saved, keep, needs):
        qkv, lse, ctx2 = saved
        B, H, S, D, scale, p, dt = keep
        dctx = dout.transpose(1, 2).reshape(B * S, H * D)
        if dctx.dtype != torch.bfloat16:
            dctx = dctx.to(torch.bfloat16)
        dqkv = Tx.attn_bwd(qkv, None, dctx.contiguous(), lse, B, S, H, scale, p, _seed(self.ctx), self.salt,
                           head_dim=D, ctx=ctx2)
        if self.heads is not None:
            return [dqkv.view(B, S, 3 * H * D).to(dt) if needs[0] else None]
        d = dqkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)                   # [3, B, H, S, D]
        return [d[i].to(dt) if needs[i] else None for i in range(3)]


class PatchEmbed(Site):
    """A conv whose stride equals its kernel and that has no padding (a ViT patch
    embedding, kernels of any size): the non-overlapping patches are one GEMM with the bias
    in its epilogue.  The patch gather is a reshape / permute copy of the input image."""

    def __init__(self, ctx, dense: DenseSet, k: int, C: int):
        super().__init__(ctx)
        object.__setattr__(self, 'dense', dense)
        self.k, self.C = int(k), int(C)

    def params(self):
        return [self.dense]

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        N, C, H, W = x.shape
        k = self.k
        Hp, Wp = H // k, W // k
        xc = x[:, :, :Hp * k, :Wp * k]
        pt = xc.reshape(N, C, Hp, k, Wp, k).permute(0, 2, 4, 1, 3, 5).reshape(N * Hp * Wp, C * k * k)
        pt = _rows(pt)
        y, _ = self.dense.fwd(pt)
        out = y.view(N, Hp, Wp, -1).permute(0, 3, 1, 2)        # logical NCHW, channels_last strides
        return out, [pt], (N, C, H, W, Hp, Wp, x.dtype)

    def bwd(self, dout, saved, keep, needs):
        (pt,) = saved
        N, C, H, W, Hp, Wp, dt = keep
        k = self.k
        d = _rows(dout.permute(0, 2, 3, 1))
        dpt = self.dense.backward(d, pt, need_dx=needs[0])
        if dpt is None:
            return [None]
        dx = dpt.view(N, Hp, Wp, C, k, k).permute(0, 3, 1, 4, 2, 5).reshape(N, C, Hp * k, Wp * k)
        if Hp * k != H or Wp * k != W:
            dx = torch.nn.functional.pad(dx, (0, W - Wp * k, 0, H - Hp * k))
        return [dx.to(dt)]


class MlpSite(Site):
    """``fc2(gelu(fc1(x))) [+ r]`` (exact GELU; a transformer MLP, timm's ``Mlp``): fc1's
    epilogue adds the bias, applies the GELU and stores gelu'(pre-activation); fc2's adds its
    bias and the residual ``r``; backward multiplies by gelu' inside fc2's input-gradient
    epilogue, so no elementwise pass is left.  Weight gradients on the side stream."""

    def __init__(self, ctx, fc1, fc2, residual: bool = False):
        super().__init__(ctx)
        object.__setattr__(self, 'fc1', fc1)          # glayers.LinearParams, unpadded
        object.__setattr__(self, 'fc2', fc2)
        self.residual = residual

    def params(self):
        return [self.fc1, self.fc2]

    def forward(self, x, r=None):
        return _run(self, x, r) if r is not None else _run(self, x)

    def fwd(self, x, r=None):
        p1, p2 = self.fc1, self.fc2
        lead = x.shape[:-1]
        x2 = _rows(x)
        g, m = Tx.dense_fwd(x2, p1.w.bf16, p1.b.master if p1.b is not None else None, act=2, want_preact=True)
        r2 = _rows(r.expand(*lead, p2.O)) if r is not None else None
        y, _ = Tx.dense_fwd(g, p2.w.bf16, p2.b.master if p2.b is not None else None, addend=r2)
        keep = (x.dtype, None if r is None else (r.shape, r.dtype))
        return y.view(*lead, p2.O), [x2, g, m], keep

    def bwd(self, dout, saved, keep, needs):
        _db = dense_backward
        p1, p2 = self.fc1, self.fc2
        x2, g, m = saved
        xdt, rkeep = keep
        d = _rows(dout)
        du = _db(self.ctx, p2.w, p2.b, d, g, dact_u=m, dact_is_deriv=True)
        if p2.uses.bwd_done():
            p2.mark_ready()
        dx = _db(self.ctx, p1.w, p1.b, du, x2, need_dx=needs[0])
        if p1.uses.bwd_done():
            p1.mark_ready()
        out = [dx.view(*dout.shape[:-1], p1.I).to(xdt) if dx is not None else None]
        if rkeep is not None:
            out.append(_reduce_to(dout, rkeep[0], rkeep[1]) if needs[1] else None)
        return out


class LinearGelu(Site):
    """``gelu(x W^T + b)`` (exact erf GELU) in one GEMM epilogue that also stores
    gelu'(pre-activation), so the backward is one multiply before the GEMMs."""

    def __init__(self, ctx, lin):
        super().__init__(ctx)
        object.__setattr__(self, 'lin', lin)     # a glayers.LinearParams (shared with LinearAct)

    def forward(self, x):
        return _run(self, x)

    def fwd(self, x):
        p = self.lin
        lead = x.shape[:-1]
        x2 = _rows(x)
        if p.Ip != p.I:
            x2 = torch.nn.functional.pad(x2, (0, p.Ip - p.I)).contiguous()
        y, u = Tx.dense_fwd(x2, p.w.bf16, p.b.master if p.b is not None else None, act=2, want_preact=True)
        out = y[:, :p.O] if p.Op != p.O else y
        return out.reshape(*lead, p.O), [x2, u], None

    def bwd(self, dout, saved, keep, needs):
        p = self.lin
        x2, u = saved
        d = dout.reshape(-1, p.O)
        if p.Op != p.O:
            d = torch.nn.functional.pad(d, (0, p.Op - p.O))
        d = (d.float() * u.float()).to(torch.bfloat16).contiguous()
        if p.b is not None and d.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0:
            Fn.linear_wgrad_bias(d, x2, p.w.grad, p.b.grad)
        else:
            Fn.linear_wgrad(d, x2, out=p.w.grad, accumulate=True)
            if p.b is not None:
                p.b.grad.add_(d.float().sum(0))
        dx = Fn.linear_dgrad(d, p.w.bf16) if needs[0] else None
        if p.uses.bwd_done():
            p.mark_ready()
        if dx is not None:
            if p.Ip != p.I:
                dx = dx[:, :p.I]
            dx = dx.reshape(*dout.shape[:-1], p.I)
        return [dx]


__all__ = ['DenseSet', 'LNParams', 'LayerNormSite', 'MHAParams', 'MHASite', 'EncoderLayerParams', 'EncoderSite',
           'SDPASite', 'LinearGelu', 'PatchEmbed', 'MlpSite', 'dense_backward', 'encoder_layer_supported', 'mha_supported', 'key_bias_of', 'next_salt']
