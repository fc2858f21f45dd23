"""BERT on the native kernels: every dense layer is the MFMA GEMM with a fused
bias / exact-GELU epilogue (pre-activation kept for backward), the GELU derivative and
the residual-gradient sum are fused into the dgrad epilogues, LayerNorm is one kernel
fused with the residual add and hidden dropout, and attention (QK^T, scale + key mask,
softmax, attention dropout, PV; backward recomputing P from the saved log-sum-exp) is one
MFMA kernel per direction that reads Q/K/V in place from the QKV projection and writes
dQ/dK/dV straight into its gradient (``Tx.attn_fwd`` / ``Tx.attn_bwd``: whole-tile kernels
for head dim 64 with S in {64, 128}, streaming flash kernels for head dim 64 / 128 and any
S that is a multiple of 64); other shapes fall back to library batched GEMMs around the
softmax kernel.

Parameters live in the flat arenas (``ops.arena``): matmul weights and embedding tables
in the decay arena (bf16 mirror for the kernels), biases and LayerNorm affine in the
no-decay arena - so AdamW is one fused launch per arena and the RCCL bucketer all-reduces
arena slices as gradients complete during backward.

Activations are token-major [T = B*S, H] bf16.  Dropout masks come from a hash of
(step seed, site salt, element): the seed is a device scalar the step advances, so a
captured HIP graph draws fresh masks every replay and backward regenerates them.
"""
from __future__ import annotations

import math
from typing import List

import os

import torch

from mlcomp_amd.ops import _lib
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops import transformer as Tx
from mlcomp_amd.ops.layers import NativeContext
from .bert import BertForSequenceClassification
from mlcomp_amd.train.native_spec import NativeUnsupported

# MLC_GELU_DERIV=1 (default): the FFN's first GEMM stores gelu'(pre-activation) instead of
# the pre-activation, so the input-gradient GEMM of the second only multiplies by it (no erf
# / exp in that epilogue); 0 keeps the pre-activation and recomputes the derivative.
GELU_DERIV = os.environ.get('MLC_GELU_DERIV', '1') == '1'
# MLC_LN_DEFER=1 (default): the LayerNorm backward kernels leave their dgamma/dbeta partial
# sums in the workspace and ONE launch at the end of backward (Tx.LnFinalizer) adds all 25 of
# them into the gradient arena, instead of a finalize launch after each LayerNorm backward;
# the LayerNorm slots are marked ready for the bucketer then.
LN_DEFER = os.environ.get('MLC_LN_DEFER', '1') == '1'


class _Dense:
    def __init__(self, ctx: NativeContext, name: str, lin: torch.nn.Linear):
        self.ctx = ctx
        self.lin = lin
        self.w = ctx.arena.weight(f'{name}.weight', tuple(lin.weight.shape))
        self.b = ctx.arena.vector(f'{name}.bias', tuple(lin.bias.shape))
        # MLC_DENSE_WT=1: a transposed weight copy for the input-gradient GEMM, so it reads
        # both operands K-contiguous (LDS-DMA loop); refreshed after the forward pass.
        # Measured -0.8 % on BERT-base (profiles/round2_ab/README.md), so off by default
        self.wt_idx = None
        if ctx.wt is not None and os.environ.get('MLC_DENSE_WT', '0') == '1':
            self.wt_idx = ctx.wt.add(self.w)

    def load(self):
        self.w.master.copy_(self.lin.weight.detach().float())
        self.b.master.copy_(self.lin.bias.detach().float())

    def export(self):
        self.lin.weight.data.copy_(self.w.master.to(self.lin.weight.device))
        self.lin.bias.data.copy_(self.b.master.to(self.lin.bias.device))

    def fwd(self, x, act=0, want_preact=False):
        self.ctx.wt_stale = True
        return Tx.dense_fwd(x, self.w.bf16, self.b.master, act, want_preact)

    def dgrad(self, dy, dact_u=None, addend=None, dact_is_deriv=False):
        """dx = dy @ W [* gelu'(dact_u)] [+ addend] (``dact_is_deriv``: dact_u = gelu'(u))."""
        wt = None
        if self.wt_idx is not None:
            if self.ctx.wt_stale:
                raise RuntimeError('transposed weights are stale: refresh_wt() must follow the forward pass')
            wt = self.ctx.wt[self.wt_idx]
        return Tx.dense_dgrad(dy, self.w.bf16, dact_u=dact_u, addend=addend, wt=wt, dact_is_deriv=dact_is_deriv)

    def bwd_params(self, dy, x):
        """dW += dy^T x, db += colsum(dy) (straight into the grad arena); the caller calls
        :meth:`mark` after the layer's dgrad, the last backward reader of W."""
        if dy.shape[0] % 8 == 0 and dy.shape[1] % 8 == 0 and x.shape[1] % 8 == 0:
            Fn.linear_wgrad_bias(dy, x, self.w.grad, self.b.grad)
        else:
            Fn.linear_wgrad(dy, x, out=self.w.grad, accumulate=True)
            Tx.colsum_acc(dy, self.b.grad)

    def mark(self):
        self.ctx.arena.mark_ready(self.w)
        self.ctx.arena.mark_ready(self.b)

    def bwd_params_async(self, dy, x, fork=None):
        """:meth:`bwd_params` on the context's weight-gradient stream (when there is one),
        forked from event ``fork`` (default: now); returns a join callable for after the
        layer's dgrad."""
        side = self.ctx.wgrad_stream
        if side is None:
            self.bwd_params(dy, x)
            return lambda: None
        main = torch.cuda.current_stream(self.ctx.device)
        if fork is None:
            side.wait_stream(main)
        else:
            side.wait_event(fork)
        with Fn.side_stream(side):
            self.bwd_params(dy, x)
        if self.ctx.wgrad_defer:
            # no per-layer join: the chain joins in flush_wgrad; keep dy / x alive for it
            dy.record_stream(side)
            x.record_stream(side)
            return lambda: None
        return lambda: main.wait_stream(side)

    def backward(self, dy, x, **dgrad_kw):
        """Input gradient (returned) + weight/bias gradients (side stream), then mark the
        slots.  With ``ctx.dgrad_first`` the dgrad is captured first and the wgrad
        forked from the point before it, so graph replay keeps the dgrad chain on one
        hardware queue (see mlcomp_amd.ops.layers)."""
        if self.ctx.dgrad_first and self.ctx.wgrad_stream is not None:
            fork = torch.cuda.Event()
            fork.record(torch.cuda.current_stream(self.ctx.device))
            dx = self.dgrad(dy, **dgrad_kw)
            join = self.bwd_params_async(dy, x, fork)
        else:
            join = self.bwd_params_async(dy, x)
            dx = self.dgrad(dy, **dgrad_kw)
        side = self.ctx.wgrad_stream
        if side is not None and self.ctx.wgrad_lag and not self.ctx.wgrad_defer:
            # lagged join (MLC_WGRAD_LAG=1): this weight gradient is joined after the NEXT
            # dense layer's input gradient, so the main stream never waits on a wgrad that
            # just started; holding dy / x until then keeps their memory from being reused
            ev = torch.cuda.Event()
            ev.record(side)
            self.ctx.lag_wgrad(ev, (dy, x), (self.w, self.b))
            return dx
        join()
        self.mark()
        return dx


class _LN:
    def __init__(self, ctx: NativeContext, name: str, ln: torch.nn.LayerNorm):
        self.ctx = ctx
        self.ln = ln
        self.g = ctx.arena.vector(f'{name}.weight', tuple(ln.weight.shape))
        self.b = ctx.arena.vector(f'{name}.bias', tuple(ln.bias.shape))
        self.k_sums = ctx.ws.request(f'{name}.sums', Fn.NSTAT * 2 * ln.weight.numel())

    def load(self):
        self.g.master.copy_(self.ln.weight.detach().float())
        self.b.master.copy_(self.ln.bias.detach().float())

    def export(self):
        self.ln.weight.data.copy_(self.g.master.to(self.ln.weight.device))
        self.ln.bias.data.copy_(self.b.master.to(self.ln.bias.device))

    def mark(self):
        self.ctx.arena.mark_ready(self.g)
        self.ctx.arena.mark_ready(self.b)

    def bwd(self, dy, s, mean, rstd, **kw):
        """Tx.ln_bwd into this LayerNorm's slots; with LN_DEFER the finalize (and the
        mark) waits for the model's LnFinalizer."""
        out = Tx.ln_bwd(dy, s, mean, rstd, self.g.master, self.g.grad, self.b.grad, self.ctx.ws[self.k_sums],
                        defer_finalize=LN_DEFER, **kw)
        if not LN_DEFER:
            self.mark()
        return out


class NativeBertLayer:
    def __init__(self, net: 'NativeBert', idx: int, layer):
        ctx = net.ctx
        self.net, self.idx = net, idx
        n = f'layers.{idx}'
        self.qkv = _Dense(ctx, f'{n}.qkv', layer.qkv)
        self.out = _Dense(ctx, f'{n}.out', layer.out)
        self.ln1 = _LN(ctx, f'{n}.ln1', layer.ln1)
        self.ffn1 = _Dense(ctx, f'{n}.ffn1', layer.ffn1)
        self.ffn2 = _Dense(ctx, f'{n}.ffn2', layer.ffn2)
        self.ln2 = _LN(ctx, f'{n}.ln2', layer.ln2)
        self.salt = 16 + 8 * idx     # dropout sites: +0 attn probs, +1 attn-out, +2 ffn-out

    def parts(self):
        return [self.qkv, self.out, self.ln1, self.ffn1, self.ffn2, self.ln2]

    def __call__(self, x, key_bias):
        return _BertLayerFn.apply(x, self.net.ctx.anchor, key_bias, self)

    # -------------------------------------------------------------- forward / backward
    def fwd(self, x, key_bias):
        net = self.net
        B, S, nh, dh = net.B, net.S, net.c.heads, net.c.head_dim
        pa, ph = net.p_attn, net.p_hidden
        qkv, _ = self.qkv.fwd(x)
        # fused attention (any S, head dim <= 128): reads q/k/v in place, writes the
        # merged-head context
        ctx2, lse = Tx.attn_fwd(qkv, key_bias, B, S, nh, 1.0 / math.sqrt(dh), pa, net.seed, self.salt,
                                head_dim=dh)
        att = (qkv, lse)
        ao, _ = self.out.fwd(ctx2)
        h1, s1, m1, r1 = Tx.ln_fwd(x, ao, self.ln1.g.master, self.ln1.b.master, net.c.eps, p_in=ph,
                                   seed=net.seed, salt_in=self.salt + 1)
        # act 2: the GEMM epilogue stores gelu'(pre-activation) for the backward (not u)
        g, u = self.ffn1.fwd(h1, act=2 if GELU_DERIV else 1, want_preact=True)
        f, _ = self.ffn2.fwd(g)
        h2, s2, m2, r2 = Tx.ln_fwd(h1, f, self.ln2.g.master, self.ln2.b.master, net.c.eps, p_in=ph,
                                   seed=net.seed, salt_in=self.salt + 2)
        return h2, (x, *att, ctx2, s1, m1, r1, h1, u, g, s2, m2, r2)

    def bwd(self, dh2, saved, key_bias):
        net = self.net
        B, S, nh, dh = net.B, net.S, net.c.heads, net.c.head_dim
        pa, ph = net.p_attn, net.p_hidden
        x, att = saved[0], saved[1:3]
        ctx2, s1, m1, r1, h1, u, g, s2, m2, r2 = saved[3:]
        ds2, df = self.ln2.bwd(dh2, s2, m2, r2, p_in=ph, seed=net.seed, salt_in=self.salt + 2, want_dr=True)
        du = self.ffn2.backward(df, g, dact_u=u, dact_is_deriv=GELU_DERIV)   # grad of the GELU input
        dh1 = self.ffn1.backward(du, h1, addend=ds2)      # + residual branch
        ds1, dao = self.ln1.bwd(dh1, s1, m1, r1, p_in=ph, seed=net.seed, salt_in=self.salt + 1, want_dr=True)
        dctx2 = self.out.backward(dao, ctx2)
        qkv, lse = att
        dqkv = Tx.attn_bwd(qkv, key_bias, dctx2, lse, B, S, nh, 1.0 / math.sqrt(dh), pa, net.seed, self.salt,
                           head_dim=dh, ctx=ctx2)
        return self.qkv.backward(dqkv, x, addend=ds1)


class _BertLayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, key_bias, layer: NativeBertLayer):
        h, saved = layer.fwd(x, key_bias)
        ctx.layer = layer
        ctx.kb = key_bias
        ctx.save_for_backward(*saved)
        return h

    @staticmethod
    def backward(ctx, dh):
        return ctx.layer.bwd(dh.contiguous(), ctx.saved_tensors, ctx.kb), None, None, None


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, anchor, net: 'NativeBert'):
        B, S = ids.shape
        e = (net.word.bf16[ids].float() + net.pos.bf16[:S][None].float() + net.tok_type.bf16[tt].float())
        e = e.to(torch.bfloat16).view(B * S, -1)
        y, s, m, r = Tx.ln_fwd(e, None, net.ln.g.master, net.ln.b.master, net.c.eps, p_out=net.p_hidden,
                               seed=net.seed, salt_out=1)
        ctx.net = net
        ctx.save_for_backward(ids, tt, s, m, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        net = ctx.net
        ids, tt, s, m, r = ctx.saved_tensors
        ds, _ = net.ln.bwd(dy.contiguous(), s, m, r, p_out=net.p_hidden, seed=net.seed, salt_out=1)
        if LN_DEFER:   # the last LayerNorm backward of the step: finalize all of them at once
            net.ln_fin.run()
            for ln in net.all_lns():
                ln.mark()
        B, S = ids.shape
        if not _lib.DETERMINISTIC and net.tok_type.grad.shape[0] <= 4:
            # one kernel: word atomics, per-position and per-type sums (Tx.embed_bwd)
            Tx.embed_bwd(ds, ids, tt, net.word.grad, net.pos.grad, net.tok_type.grad)
            for sl in (net.word, net.pos, net.tok_type):
                net.ctx.arena.mark_ready(sl)
            return None, None, None, None
        d = ds.float().view(B, S, -1)
        if _lib.DETERMINISTIC:
            # index_add_ races float atomics on repeated ids: a stable sort groups the rows
            # of each id in token order and segment_reduce sums every group sequentially
            # (no atomics, no one-hot GEMM), then the ids - now unique - are added once each
            dd = d.reshape(B * S, -1)
            for tbl, ix in ((net.word, ids), (net.tok_type, tt)):
                tbl.grad.add_(_segment_sums(ix.reshape(-1), dd, tbl.grad.shape[0]))
        else:
            net.word.grad.index_add_(0, ids.reshape(-1), d.reshape(B * S, -1))
            net.tok_type.grad.index_add_(0, tt.reshape(-1), d.reshape(B * S, -1))
        net.pos.grad[:S].add_(d.sum(0))
        for sl in (net.word, net.pos, net.tok_type):
            net.ctx.arena.mark_ready(sl)
        return None, None, None, None


def _segment_sums(ix: torch.Tensor, rows: torch.Tensor, V: int) -> torch.Tensor:
    """[V, H] per-id sums of ``rows`` in a fixed order, with static shapes (graph-capturable:
    no host sync): a stable sort groups the rows of each id in token order, integer counts
    give the segment lengths, and torch.segment_reduce sums every segment sequentially."""
    order = torch.sort(ix, stable=True)[1]
    counts = torch.zeros(V, dtype=torch.long, device=ix.device).scatter_add_(0, ix, torch.ones_like(ix))
    return torch.segment_reduce(rows[order], 'sum', lengths=counts, axis=0, unsafe=True)


class _HeadFn(torch.autograd.Function):
    """[CLS] -> tanh pooler -> (dropout) -> classifier -> fused softmax-CE (sum reduced)."""

    @staticmethod
    def forward(ctx, h, anchor, labels, net: 'NativeBert'):
        B, S = net.B, net.S
        cls = h.view(B, S, -1)[:, 0].contiguous()
        z, _ = net.pooler.fwd(cls)
        net.ctx.refresh_wt()    # every dense layer has run its forward: transposed copies for backward
        pooled = torch.tanh(z.float()).to(torch.bfloat16)
        pd = Tx.dropout(pooled, net.p_hidden, net.seed, 2)
        logits = Fn.linear_fwd(pd, net.cls_w.bf16, net.cls_b.master)
        dl = Fn.softmax_ce(logits, labels, net.loss_sum(), net.correct(), scale=1.0 / B,
                           num_classes=net.c.num_labels)
        ctx.net = net
        ctx.save_for_backward(cls, pooled, pd, dl)
        net._logits = logits
        return (net.loss_sum() / B).sum()

    @staticmethod
    def backward(ctx, g):
        net = ctx.net
        cls, pooled, pd, dl = ctx.saved_tensors
        a = net.ctx.arena
        Fn.linear_wgrad(dl, pd, out=net.cls_w.grad, accumulate=True)
        Tx.colsum_acc(dl, net.cls_b.grad) if dl.shape[1] % 8 == 0 else net.cls_b.grad.add_(dl.float().sum(0))
        dpd = Fn.linear_dgrad(dl, net.cls_w.bf16)
        a.mark_ready(net.cls_w)
        a.mark_ready(net.cls_b)
        dpooled = Tx.dropout(dpd, net.p_hidden, net.seed, 2)   # same mask, same scale
        dz = (dpooled.float() * (1 - pooled.float() ** 2)).to(torch.bfloat16)
        net.pooler.bwd_params(dz, cls)
        dcls = net.pooler.dgrad(dz)
        net.pooler.mark()
        dh = torch.zeros(net.B, net.S, dcls.shape[1], device=dcls.device, dtype=torch.bfloat16)
        dh[:, 0] = dcls
        return dh.view(net.B * net.S, -1), None, None, None


def native_bert_unsupported(c, seq_len: int = 1):
    """Why the native BERT engine cannot train config ``c`` (None when it can): GEMM rows
    in 16-byte chunks (hidden / intermediate % 8) and the fused attention's head dims
    (<= 128, :func:`mlcomp_amd.ops.transformer.attn_supported`)."""
    if c.hidden % 8 or c.intermediate % 8:
        return f'hidden {c.hidden} / intermediate {c.intermediate}: the native GEMMs need multiples of 8'
    if c.hidden % c.heads:
        return f'hidden {c.hidden} is not a multiple of heads {c.heads}'
    if seq_len < 1 or not Tx.attn_supported(seq_len, c.head_dim):
        return f'head_dim {c.head_dim} (seq_len {seq_len}): the fused attention takes head dims <= 128'
    return None


class NativeBert:
    def __init__(self, model: BertForSequenceClassification, device, batch: int, seq_len: int):
        c = model.config
        unsupported = native_bert_unsupported(c, seq_len)
        if unsupported:
            raise NativeUnsupported(unsupported)
        self.model, self.c = model, c
        self.B, self.S = batch, seq_len
        self.p_hidden, self.p_attn = c.hidden_dropout, c.attention_dropout
        ctx = self.ctx = NativeContext()
        a = ctx.arena
        # registration order == forward order (the arena lays slots out backward-first)
        self.word = a.weight('word', tuple(model.word.weight.shape))
        self.pos = a.weight('pos', tuple(model.pos.weight.shape))
        self.tok_type = a.weight('tok_type', tuple(model.tok_type.weight.shape))
        self.ln = _LN(ctx, 'ln', model.ln)
        self.layers: List[NativeBertLayer] = [NativeBertLayer(self, i, l) for i, l in enumerate(model.layers)]
        self.pooler = _Dense(ctx, 'pooler', model.pooler)
        self.Lp = (c.num_labels + 7) // 8 * 8   # classifier rows padded for 16 B MFMA chunks
        self.cls_w = a.weight('classifier.weight', (self.Lp, c.hidden))
        self.cls_b = a.vector('classifier.bias', (self.Lp,))
        self.k_loss = ctx.ws.request('loss', 1)
        self.k_correct = ctx.ws.request('correct', 1)
        ctx.finalize(device)
        # weight gradients: captured after each dense layer's input gradient and forked from
        # the point before it (dgrad_first), never joined per layer (one free-running side
        # chain, joined before the optimizer).  Interleaved A/B on one MI355X (bench.py,
        # 2 rounds): per-layer join 5,139 / 5,155 seq/s, lagged join by 1 / 3 layers 5,348 /
        # 5,556, this 5,612 / 5,610 (profiles/round5/bert_wgrad_join_ab.txt); round 4's
        # deferral without dgrad_first lost 3-6 %.  MLC_WGRAD_DEFER / MLC_DGRAD_FIRST override.
        ctx.default_wgrad_defer(True)
        ctx.default_dgrad_first(True)
        self.device = ctx.device
        self.seed = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.ln_fin = Tx.LnFinalizer()
        for ln in self.all_lns():
            self.ln_fin.add(ctx.ws[ln.k_sums], ln.g.grad, ln.b.grad)
        self.ln_fin.build()
        self.load_from_torch()

    def all_lns(self):
        yield self.ln
        for l in self.layers:
            yield l.ln1
            yield l.ln2

    # ------------------------------------------------------------------ weights
    def _dense_parts(self):
        for l in self.layers:
            yield from l.parts()
        yield self.pooler
        yield self.ln

    def load_from_torch(self):
        m = self.model
        with torch.no_grad():
            self.word.master.copy_(m.word.weight.float())
            self.pos.master.copy_(m.pos.weight.float())
            self.tok_type.master.copy_(m.tok_type.weight.float())
            for p in self._dense_parts():
                p.load()
            self.cls_w.master.zero_()
            self.cls_b.master.zero_()
            self.cls_w.master[:self.c.num_labels].copy_(m.classifier.weight.float())
            self.cls_b.master[:self.c.num_labels].copy_(m.classifier.bias.float())
        self.ctx.arena.decay.refresh_mirror()

    def export_to_torch(self):
        m = self.model
        with torch.no_grad():
            m.word.weight.copy_(self.word.master.to(m.word.weight.device))
            m.pos.weight.copy_(self.pos.master.to(m.pos.weight.device))
            m.tok_type.weight.copy_(self.tok_type.master.to(m.tok_type.weight.device))
            for p in self._dense_parts():
                p.export()
            m.classifier.weight.copy_(self.cls_w.master[:self.c.num_labels].to(m.classifier.weight.device))
            m.classifier.bias.copy_(self.cls_b.master[:self.c.num_labels].to(m.classifier.bias.device))

    @property
    def arena(self):
        return self.ctx.arena

    def loss_sum(self):
        return self.ctx.ws[self.k_loss]

    def correct(self):
        return self.ctx.ws[self.k_correct]

    def train(self, mode=True):
        self.ctx.training = mode
        self.p_hidden = self.c.hidden_dropout if mode else 0.0
        self.p_attn = self.c.attention_dropout if mode else 0.0

    def eval(self):
        self.train(False)

    # ------------------------------------------------------------------ graph
    def loss(self, ids, tt, key_bias, labels):
        h = _EmbedFn.apply(ids, tt, self.ctx.anchor, self)
        for layer in self.layers:
            h = layer(h, key_bias)
        return _HeadFn.apply(h, self.ctx.anchor, labels, self)

    def logits(self):
        return self._logits[:, :self.c.num_labels]

    def predict(self, ids, tt, key_bias=None):
        """Inference forward on the native kernels (no dropout, no autograd, no loss
        accumulators touched): fp32 logits [B, num_labels].  Any batch size / sequence
        length the kernels take (the eval loader's last batch may be short)."""
        B, S = ids.shape
        saved = (self.B, self.S, self.ctx.training)
        self.B, self.S = B, S
        self.train(False)
        try:
            with torch.no_grad():
                e = (self.word.bf16[ids].float() + self.pos.bf16[:S][None].float()
                     + self.tok_type.bf16[tt].float()).to(torch.bfloat16).view(B * S, -1)
                h = Tx.ln_fwd(e, None, self.ln.g.master, self.ln.b.master, self.c.eps, p_out=0.0,
                              seed=self.seed, salt_out=1)[0]
                for layer in self.layers:
                    h, _ = layer.fwd(h, key_bias)
                cls = h.view(B, S, -1)[:, 0].contiguous()
                z, _ = self.pooler.fwd(cls)
                pooled = torch.tanh(z.float()).to(torch.bfloat16)
                logits = Fn.linear_fwd(pooled, self.cls_w.bf16, self.cls_b.master)
            return logits[:, :self.c.num_labels].float()
        finally:
            self.B, self.S = saved[0], saved[1]
            self.train(saved[2])


__all__ = ['NativeBert']
