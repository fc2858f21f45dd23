"""Python entry points of the transformer kernels (``csrc/kernels/transformer.hip`` and the
dense-layer GEMM epilogue of ``igemm.hip``), each with an fp32 PyTorch reference used on
CPU (and by the numerics tests).  Dropout uses the kernels' counter-based hash, which the
CPU path reproduces bit-exactly, so masks agree between the two."""
from __future__ import annotations

import math
import os
from typing import Optional, Tuple

import torch

from . import _lib
from .functional import NSTAT, _cuda

_M32 = 0xFFFFFFFF


def _hash(seed: int, salt: int, idx: torch.Tensor) -> torch.Tensor:
    x = (idx * 0x9E3779B9) & _M32
    x = x ^ ((seed * 0x85EBCA6B + salt * 0xC2B2AE35) & _M32)
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def keep_mask(shape, p: float, seed: int, salt: int, device=None) -> torch.Tensor:
    """Same keep decisions as the kernels for a contiguous tensor of ``shape``."""
    n = 1
    for s in shape:
        n *= s
    idx = torch.arange(n, dtype=torch.int64, device=device)
    thr = int(p * 16777216.0)
    return ((_hash(seed, salt, idx) >> 8) >= thr).reshape(shape)


def _seed_val(seed) -> int:
    return int(seed.item()) if torch.is_tensor(seed) else int(seed or 0)


# ---------------------------------------------------------------------------- LayerNorm
def ln_fwd(x, r, gamma, beta, eps=1e-12, p_in=0.0, p_out=0.0, seed=None, salt_in=0, salt_out=0):
    """y = dropout_out(LN(x + dropout_in(r))).  Returns (y, s, mean, rstd) where s is the
    normalised input (``x`` itself when there is no ``r``)."""
    T, H = x.shape
    if _cuda(x):
        y = torch.empty_like(x)
        s = torch.empty_like(x) if r is not None else x
        mean = torch.empty(T, device=x.device, dtype=torch.float32)
        rstd = torch.empty(T, device=x.device, dtype=torch.float32)
        _lib.call('mlc_ln_fwd', _lib.ptr(x), _lib.ptr(r), _lib.ptr(s if r is not None else None), _lib.ptr(y),
                  _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(gamma), _lib.ptr(beta), T, H, float(eps), float(p_in),
                  float(p_out), _lib.ptr(seed), salt_in, salt_out, _lib.stream())
        return y, s, mean, rstd
    sd = _seed_val(seed)
    v = x.float()
    if r is not None:
        rr = r.float()
        if p_in > 0:
            rr = torch.where(keep_mask((T, H), p_in, sd, salt_in), rr / (1 - p_in), torch.zeros_like(rr))
        v = v + rr
    s = v.to(torch.bfloat16) if r is not None else x
    mean = v.mean(1)
    var = ((v - mean[:, None]) ** 2).mean(1)
    rstd = torch.rsqrt(var + eps)
    y = (v - mean[:, None]) * rstd[:, None] * gamma + beta
    if p_out > 0:
        y = torch.where(keep_mask((T, H), p_out, sd, salt_out), y / (1 - p_out), torch.zeros_like(y))
    return y.to(torch.bfloat16), s, mean, rstd


def ln_bwd(dy, s, mean, rstd, gamma, dgamma, dbeta, sums=None, p_in=0.0, p_out=0.0, seed=None, salt_in=0,
           salt_out=0, want_dr=False, defer_finalize=False):
    """Returns (ds, dr): ds = dLoss/ds, dr = dropout_in'(ds) (None unless ``want_dr``).
    dgamma / dbeta are ACCUMULATED (+=).  ``defer_finalize`` (GPU): leave the per-copy
    partial sums in ``sums`` for a later :class:`LnFinalizer` launch (dgamma/dbeta untouched
    until then)."""
    T, H = dy.shape
    if _cuda(dy):
        ds = torch.empty_like(dy)
        dr = torch.empty_like(dy) if want_dr else None
        if sums is None:
            assert not defer_finalize, 'a deferred finalize needs a persistent sums scratch'
            sums = torch.zeros(NSTAT * 2 * H, device=dy.device, dtype=torch.float32)
        dg, db = (None, None) if defer_finalize else (dgamma, dbeta)
        _lib.call('mlc_ln_bwd', _lib.ptr(dy), _lib.ptr(s), _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(gamma),
                  _lib.ptr(ds), _lib.ptr(dr), _lib.ptr(sums), _lib.ptr(dg), _lib.ptr(db), T, H, float(p_in),
                  float(p_out), _lib.ptr(seed), salt_in, salt_out, _lib.stream())
        return ds, dr
    sd = _seed_val(seed)
    d = dy.float()
    if p_out > 0:
        d = torch.where(keep_mask((T, H), p_out, sd, salt_out), d / (1 - p_out), torch.zeros_like(d))
    xh = (s.float() - mean[:, None]) * rstd[:, None]
    dgamma.add_((d * xh).sum(0))
    dbeta.add_(d.sum(0))
    g = d * gamma
    a = g.mean(1, keepdim=True)
    b = (g * xh).mean(1, keepdim=True)
    dsf = rstd[:, None] * (g - a - xh * b)
    ds = dsf.to(torch.bfloat16)
    dr = None
    if want_dr:
        drf = dsf
        if p_in > 0:
            drf = torch.where(keep_mask((T, H), p_in, sd, salt_in), dsf / (1 - p_in), torch.zeros_like(dsf))
        dr = drf.to(torch.bfloat16)
    return ds, dr


_EMB_SCRATCH = {}


def embed_bwd(ds, ids, tt, word_grad, pos_grad, tok_grad):
    """Embedding gradients from ds [B*S, H] (bf16): word_grad[ids] += ds, pos_grad[s] +=
    sum over the batch, tok_grad[tt] += ds (all fp32, accumulated).  ids / tt int64 [B, S]."""
    B, S = ids.shape
    H = ds.shape[-1]
    if _cuda(ds):
        ntypes = tok_grad.shape[0] if tok_grad is not None else 1
        from .functional import workspace_key, workspace_store
        key = (workspace_key(ds.device), S * ntypes * H)
        store = workspace_store(_EMB_SCRATCH)
        pt = store.get(key)
        if pt is None:    # [S][ntypes][H] partial sums, left zeroed by the kernel
            pt = store[key] = torch.zeros(S * ntypes * H, device=ds.device, dtype=torch.float32)
        # contiguous copies bound to names: a temporary freed while the argument list is
        # still being built could hand its block to the next copy before the kernel runs
        dsc, idc = ds.contiguous(), ids.contiguous()
        ttc = tt.contiguous() if tok_grad is not None else None
        _lib.call('mlc_embed_bwd', _lib.ptr(dsc), _lib.ptr(idc), _lib.ptr(ttc), _lib.ptr(word_grad),
                  _lib.ptr(pos_grad), _lib.ptr(tok_grad), _lib.ptr(pt), B, S, H, ntypes, _lib.stream())
        return
    d = ds.float().reshape(B * S, H)
    word_grad.index_add_(0, ids.reshape(-1), d)
    if tok_grad is not None:
        tok_grad.index_add_(0, tt.reshape(-1), d)
    pos_grad[:S].add_(d.view(B, S, H).sum(0))


class LnFinalizer:
    """Finalizes the dgamma / dbeta of many LayerNorms in ONE launch
    (``mlc_ln_finalize_many``): each entry's ``ln_bwd(..., defer_finalize=True)`` left its
    partial sums in a persistent NSTAT-copy scratch; ``run()`` adds every sum into its grad
    slots.  The descriptor table is built once (pointers must stay put), outside capture."""

    def __init__(self):
        self.entries = []        # (sums [NSTAT*2*H], dgamma [H], dbeta [H])
        self.desc = None
        self.max_h = 0

    def add(self, sums, dgamma, dbeta):
        self.entries.append((sums, dgamma, dbeta))

    def build(self):
        if not self.entries or not self.entries[0][0].is_cuda:
            return
        rows = [[s.data_ptr(), g.data_ptr(), b.data_ptr(), g.numel()] for s, g, b in self.entries]
        self.desc = torch.tensor(rows, dtype=torch.int64).to(self.entries[0][0].device)
        self.max_h = max(g.numel() for _, g, _ in self.entries)

    def run(self):
        if not self.entries or not self.entries[0][0].is_cuda:
            return       # the CPU path of ln_bwd accumulates immediately
        if self.desc is None:
            self.build()
        _lib.call('mlc_ln_finalize_many', _lib.ptr(self.desc), len(self.entries), self.max_h, _lib.stream())


# ---------------------------------------------------------------------------- softmax
def softmax_fwd(S, key_bias, rows_per_batch, scale, p=0.0, seed=None, salt=0):
    """S [R, L] bf16 scores; key_bias [B, L] fp32 (0 / -inf) or None.  Returns (P, Pd)."""
    R, L = S.shape
    if _cuda(S):
        P = torch.empty_like(S)
        Pd = torch.empty_like(S) if p > 0 else P
        _lib.call('mlc_softmax_fwd', _lib.ptr(S), _lib.ptr(key_bias), _lib.ptr(P),
                  _lib.ptr(Pd if p > 0 else None), R, L, rows_per_batch, float(scale), float(p), _lib.ptr(seed),
                  salt, _lib.stream())
        return P, Pd
    v = S.float() * scale
    if key_bias is not None:
        v = v + key_bias.repeat_interleave(rows_per_batch, 0)
    Pf = torch.softmax(v, 1).nan_to_num(0.0)
    P = Pf.to(torch.bfloat16)
    if p > 0:
        m = keep_mask((R, L), p, _seed_val(seed), salt)
        Pd = torch.where(m, Pf / (1 - p), torch.zeros_like(Pf)).to(torch.bfloat16)
    else:
        Pd = P
    return P, Pd


def softmax_bwd(P, dPd, scale, p=0.0, seed=None, salt=0):
    R, L = P.shape
    if _cuda(P):
        dS = torch.empty_like(P)
        _lib.call('mlc_softmax_bwd', _lib.ptr(P), _lib.ptr(dPd), _lib.ptr(dS), R, L, float(scale), float(p),
                  _lib.ptr(seed), salt, _lib.stream())
        return dS
    d = dPd.float()
    if p > 0:
        d = torch.where(keep_mask((R, L), p, _seed_val(seed), salt), d / (1 - p), torch.zeros_like(d))
    Pf = P.float()
    dot = (Pf * d).sum(1, keepdim=True)
    return (scale * Pf * (d - dot)).to(torch.bfloat16)


# ---------------------------------------------------------------------------- fused attention
# The streaming kernels measured faster than the whole-tile ones on every shape both take
# (profiles/flash_attn/); MLC_ATTN_KERNEL=tile routes head dim 64, S in {64, 128} back to them.
_FLASH_ONLY = os.environ.get('MLC_ATTN_KERNEL', 'flash') != 'tile'


def _attn_small(S: int, head_dim: int) -> bool:
    """Shapes of the whole-tile kernels ``mlc_attn_fwd`` / ``mlc_attn_bwd`` (transformer.hip)."""
    return head_dim == 64 and S in (64, 128) and not _FLASH_ONLY


def _attn_flash(S: int, head_dim: int) -> bool:
    """Shapes of the streaming kernels ``mlc_flash_fwd`` / ``mlc_flash_bwd`` (flash_attn.hip):
    any S (a partial last 64-key tile is masked in the kernel), head dim 64 or 128."""
    return head_dim in (64, 128) and S >= 1


def _pad_dim(head_dim: int) -> int:
    """The kernel head dim a head dim of ``head_dim`` runs at (zero-padded columns change
    neither the scores nor the kept output columns)."""
    return 64 if head_dim <= 64 else 128


def attn_supported(S: int, head_dim: int) -> bool:
    """Shapes the fused attention path takes: every S >= 1 and head dim <= 128 (head dims
    other than 64 / 128 run zero-padded to the next of the two)."""
    return S >= 1 and 1 <= head_dim <= 128


def _pad_heads(t, rows, groups, H, D, Dp):
    """[rows, groups*H*D] -> [rows, groups*H*Dp] with zero columns after each head."""
    out = torch.zeros(rows, groups, H, Dp, device=t.device, dtype=t.dtype)
    out[..., :D] = t.view(rows, groups, H, D)
    return out.view(rows, groups * H * Dp)


def _unpad_heads(t, rows, groups, H, D, Dp):
    return t.view(rows, groups, H, Dp)[..., :D].reshape(rows, groups * H * D)


def _attn_ref_probs(qkv, key_bias, B, S, H, scale, D=64):
    E = H * D
    q, k, v = qkv.float().view(B, S, 3, H, D).permute(2, 0, 3, 1, 4).unbind(0)   # [B, H, S, D]
    x = torch.matmul(q, k.transpose(-1, -2)) * scale
    if key_bias is not None:
        x = x + key_bias.float()[:, None, None, :]
    P = torch.softmax(x, -1).nan_to_num(0.0)
    return q, k, v, P, E


def attn_fwd(qkv, key_bias, B, S, H, scale, p=0.0, seed=None, salt=0, head_dim: int = 64):
    """Fused multi-head attention over the QKV projection output ``qkv`` [B*S, 3*H*D]
    (columns q | k | v, head h at h*D).  Returns (ctx [B*S, H*D] bf16, lse [B*H*S] fp32).
    Attention-probability dropout uses the softmax kernel's mask indexing
    (((b*H + h)*S + q)*S + key), so every path drops the same elements."""
    D = head_dim
    if _cuda(qkv) and D not in (64, 128):
        assert attn_supported(S, D), (S, D)
        Dp = _pad_dim(D)
        ctx, lse = attn_fwd(_pad_heads(qkv, B * S, 3, H, D, Dp), key_bias, B, S, H, scale, p, seed, salt, Dp)
        return _unpad_heads(ctx, B * S, 1, H, D, Dp), lse
    if _cuda(qkv):
        assert attn_supported(S, D) and qkv.is_contiguous() and tuple(qkv.shape) == (B * S, 3 * H * D)
        assert key_bias is None or (key_bias.is_contiguous() and tuple(key_bias.shape) == (B, S))
        ctx = torch.empty(B * S, H * D, device=qkv.device, dtype=torch.bfloat16)
        lse = torch.empty(B * H * S, device=qkv.device, dtype=torch.float32)
        if _attn_small(S, D):
            _lib.call('mlc_attn_fwd', _lib.ptr(qkv), _lib.ptr(key_bias), _lib.ptr(ctx), _lib.ptr(lse), B, S, H,
                      float(scale), float(p), _lib.ptr(seed), salt, _lib.stream())
        else:
            _lib.call('mlc_flash_fwd', _lib.ptr(qkv), _lib.ptr(key_bias), _lib.ptr(ctx), _lib.ptr(lse), B, S, H, D,
                      float(scale), float(p), _lib.ptr(seed), salt, _lib.stream())
        return ctx, lse
    q, k, v, P, E = _attn_ref_probs(qkv, key_bias, B, S, H, scale, D)
    Pd = P
    if p > 0:
        m = keep_mask((B, H, S, S), p, _seed_val(seed), salt)
        Pd = torch.where(m, P / (1 - p), torch.zeros_like(P))
    ctx = torch.matmul(Pd, v).permute(0, 2, 1, 3).reshape(B * S, E)
    x = torch.matmul(q, k.transpose(-1, -2)) * scale
    if key_bias is not None:
        x = x + key_bias.float()[:, None, None, :]
    lse = torch.logsumexp(x, -1).reshape(-1)
    return ctx.to(torch.bfloat16), lse


def attn_bwd(qkv, key_bias, dctx, lse, B, S, H, scale, p=0.0, seed=None, salt=0, head_dim: int = 64, ctx=None):
    """Gradient of :func:`attn_fwd` wrt ``qkv``: returns dqkv [B*S, 3*H*D] bf16.  ``ctx``
    (the forward output) is needed by the streaming kernels (rowsum(dO * O))."""
    D = head_dim
    if _cuda(qkv) and D not in (64, 128):
        assert attn_supported(S, D) and ctx is not None, (S, D)
        Dp = _pad_dim(D)
        dq = attn_bwd(_pad_heads(qkv, B * S, 3, H, D, Dp), key_bias, _pad_heads(dctx, B * S, 1, H, D, Dp), lse,
                      B, S, H, scale, p, seed, salt, Dp, ctx=_pad_heads(ctx, B * S, 1, H, D, Dp))
        return _unpad_heads(dq, B * S, 3, H, D, Dp)
    if _cuda(qkv):
        assert attn_supported(S, D) and qkv.is_contiguous() and tuple(qkv.shape) == (B * S, 3 * H * D)
        assert dctx.is_contiguous() and tuple(dctx.shape) == (B * S, H * D) and lse.numel() == B * H * S
        assert key_bias is None or (key_bias.is_contiguous() and tuple(key_bias.shape) == (B, S))
        dqkv = torch.empty_like(qkv)
        if _attn_small(S, D):
            _lib.call('mlc_attn_bwd', _lib.ptr(qkv), _lib.ptr(key_bias), _lib.ptr(dctx), _lib.ptr(lse),
                      _lib.ptr(dqkv), B, S, H, float(scale), float(p), _lib.ptr(seed), salt, _lib.stream())
        else:
            assert ctx is not None and ctx.is_contiguous() and ctx.shape == dctx.shape
            dot = torch.empty(B * H * S, device=qkv.device, dtype=torch.float32)
            _lib.call('mlc_flash_bwd', _lib.ptr(qkv), _lib.ptr(key_bias), _lib.ptr(ctx), _lib.ptr(dctx),
                      _lib.ptr(lse), _lib.ptr(dot), _lib.ptr(dqkv), B, S, H, D, float(scale), float(p),
                      _lib.ptr(seed), salt, _lib.stream())
        return dqkv
    q, k, v, P, E = _attn_ref_probs(qkv, key_bias, B, S, H, scale, D)
    do = dctx.float().view(B, S, H, D).permute(0, 2, 1, 3)
    m = keep_mask((B, H, S, S), p, _seed_val(seed), salt) if p > 0 else None
    Pd = torch.where(m, P / (1 - p), torch.zeros_like(P)) if m is not None else P
    dv = torch.matmul(Pd.transpose(-1, -2), do)
    dPd = torch.matmul(do, v.transpose(-1, -2))
    dP = torch.where(m, dPd / (1 - p), torch.zeros_like(dPd)) if m is not None else dPd
    dS = scale * P * (dP - (P * dP).sum(-1, keepdim=True))
    dq = torch.matmul(dS, k)
    dk = torch.matmul(dS.transpose(-1, -2), q)
    dqkv = torch.stack([dq, dk, dv]).permute(1, 3, 0, 2, 4).reshape(B * S, 3 * E)
    return dqkv.to(torch.bfloat16)


# ---------------------------------------------------------------------------- dense layers
_WS = {}
_WS_OLD = []   # superseded buffers stay alive: a captured graph may still point at them


def gemm_workspace(device, n: int) -> torch.Tensor:
    """fp32 split-K slab workspace per device (``splits`` x M x N partial sums, fully
    overwritten by each split-K GEMM), grown on demand - first during eager warm-up, so
    graph capture reuses it."""
    from .functional import workspace_key, workspace_store
    key = workspace_key(device)
    store = workspace_store(_WS)
    buf = store.get(key)
    if buf is None or buf.numel() < n:
        if buf is not None:
            _WS_OLD.append(buf)
        buf = torch.empty(max(n, 1 << 20), device=device, dtype=torch.float32)
        store[key] = buf
    return buf


def _gelu(u):
    return 0.5 * u * (1.0 + torch.erf(u / math.sqrt(2.0)))


def _dgelu(u):
    return 0.5 * (1.0 + torch.erf(u / math.sqrt(2.0))) + u * torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi)


def dense_fwd(x, w, bias=None, act: int = 0, want_preact: bool = False, addend=None):
    """y = act(x @ w^T + bias) [+ addend]: x [M, K] bf16, w [N, K] bf16, bias fp32 [N],
    addend bf16 [M, N] (a residual summed in the epilogue).  Returns (y, u) with u the bf16
    pre-activation (when ``want_preact``).  ``act`` 1 = exact-erf GELU; 2 = GELU returning
    u = gelu'(pre-activation) instead, for ``dense_dgrad(..., dact_is_deriv=True)`` (the
    backward epilogue then only multiplies)."""
    M, K = x.shape
    N = w.shape[0]
    if _cuda(x):
        y = torch.empty(M, N, device=x.device, dtype=torch.bfloat16)
        u = torch.empty_like(y) if want_preact else None
        if addend is not None:
            assert addend.dtype == torch.bfloat16 and addend.is_contiguous() and tuple(addend.shape) == (M, N)
        _lib.call('mlc_gemm_bf16_ex', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), M, N, K, K, K, N, 0, 1,
                  _lib.ptr(bias), act, _lib.ptr(u), _lib.ptr(addend), None,
                  _lib.ptr(gemm_workspace(x.device, 4 * M * N)), 4 * M * N, _lib.stream())
        return y, u
    z = x.float() @ w.float().t()
    if bias is not None:
        z = z + bias
    if act == 2:
        u = _dgelu(z).to(torch.bfloat16) if want_preact else None
    else:
        u = z.to(torch.bfloat16) if want_preact else None
    if act in (1, 2):
        z = _gelu(z)
    if addend is not None:
        z = z + addend.float()
    return z.to(torch.bfloat16), u


def dense_dgrad(dy, w, dact_u=None, addend=None, wt=None, dact_is_deriv=False):
    """dx = (dy @ w) [* gelu'(dact_u)] [+ addend]: dy [M, N], w [N, K] -> [M, K] bf16.
    ``dact_is_deriv``: ``dact_u`` already holds gelu'(u) (``dense_fwd(act=2)``), multiply.
    ``wt`` = w^T ([K, N], e.g. a ``Fn.WtTable`` view): the GEMM reads both operands
    K-contiguous (the LDS-DMA main loop) instead of w as an MN-contiguous tile."""
    M, N = dy.shape
    K = w.shape[1]
    if _cuda(dy):
        dx = torch.empty(M, K, device=dy.device, dtype=torch.bfloat16)
        b, ldb, tb = (wt, N, 1) if wt is not None else (w, K, 0)
        if wt is not None:
            assert tuple(wt.shape) == (K, N), (wt.shape, w.shape)
        _lib.call('mlc_gemm_bf16_ex', _lib.ptr(dy), _lib.ptr(b), _lib.ptr(dx), M, K, N, N, ldb, K, 0, tb, None,
                  4 if (dact_u is not None and dact_is_deriv) else 0,
                  None, _lib.ptr(addend), _lib.ptr(dact_u), _lib.ptr(gemm_workspace(dy.device, 4 * M * K)),
                  4 * M * K, _lib.stream())
        return dx
    if wt is not None:
        w = wt.t()
    z = dy.float() @ w.float()
    z = z.to(torch.bfloat16).float()
    if dact_u is not None:
        z = z * (dact_u.float() if dact_is_deriv else _dgelu(dact_u.float()))
    if addend is not None:
        z = z + addend.float()
    return z.to(torch.bfloat16)


def dact_gelu(dy, u):
    """dy * gelu'(u) as a standalone op (used when the GEMM producing dy cannot fuse it)."""
    return (dy.float() * _dgelu(u.float())).to(torch.bfloat16)


_SCRATCH = {}


def colsum_scratch(device, C: int) -> torch.Tensor:
    """A zeroed NSTAT*C fp32 buffer per device, grown on demand; the kernel leaves it
    zeroed, so every call of a step (and a captured graph) can share it."""
    from .functional import workspace_key, workspace_store
    # per stream role and capture scope, like the split-K slabs: the kernel relies on the
    # buffer being zero on entry, so two colsums that overlap must never share one
    key = workspace_key(device)
    store = workspace_store(_SCRATCH)
    buf = store.get(key)
    if buf is None or buf.numel() < NSTAT * C:
        if buf is not None:
            _WS_OLD.append(buf)
        buf = torch.zeros(NSTAT * max(C, 4096), device=device, dtype=torch.float32)
        store[key] = buf
    return buf


def colsum_acc(g, out, scratch=None):
    """out += column sums of g [R, C] bf16."""
    R, C = g.shape
    if _cuda(g):
        sc = scratch if scratch is not None else colsum_scratch(g.device, C)
        _lib.call('mlc_colsum_acc', _lib.ptr(g), _lib.ptr(out), _lib.ptr(sc), R, C, _lib.stream())
        return out
    out.add_(g.float().sum(0))
    return out


def dropout(x, p, seed, salt):
    if p <= 0:
        return x
    if _cuda(x):
        y = torch.empty_like(x)
        _lib.call('mlc_dropout', _lib.ptr(x), _lib.ptr(y), x.numel(), float(p), _lib.ptr(seed), salt, _lib.stream())
        return y
    m = keep_mask(tuple(x.shape), p, _seed_val(seed), salt)
    return torch.where(m, x.float() / (1 - p), torch.zeros_like(x, dtype=torch.float32)).to(x.dtype)


__all__ = ['ln_fwd', 'ln_bwd', 'LnFinalizer', 'embed_bwd', 'softmax_fwd', 'softmax_bwd', 'dense_fwd', 'dense_dgrad', 'dact_gelu', 'colsum_acc',
           'dropout', 'keep_mask']
