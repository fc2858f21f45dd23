"""BERT-base (32 x 128 tokens) step parts on one GPU, graph-timed: attention forward /
backward (whole-tile and streaming kernels) and LayerNorm forward / backward with and
without dropout, and the fused Adam update over a BERT-base-sized arena.  Shows what the
counter-hash dropout masks cost and how far the memory-bound parts are from HBM speed.

    python scripts/bench_bert_parts.py
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_1x1 import graph_time  # noqa: E402
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def main():
    dev = 'cuda'
    B, S, H, D = 32, 128, 12, 64
    T, E = B * S, H * D
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = (torch.randn(T, 3 * E, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    dctx = torch.randn(T, E, device=dev, generator=g).to(torch.bfloat16)
    kb = torch.zeros(B, S, device=dev)
    seed = torch.zeros(1, device=dev, dtype=torch.int32)
    scale = 1 / math.sqrt(D)
    fns = {}
    res = {}
    lib = _lib.load()
    for b128 in (0, 1):      # S = 128 fused backward off / on (flash path)
        Tx._FLASH_ONLY = True
        ctx, lse = Tx.attn_fwd(qkv, kb, B, S, H, scale, 0.1, seed, 7)

        def f(b128=b128, c=ctx, l=lse):
            lib.mlc_flash_bwd128(b128)
            Tx._FLASH_ONLY = True
            return Tx.attn_bwd(qkv, kb, dctx, l, B, S, H, scale, 0.1, seed, 7, ctx=c)
        fns[f'attn_bwd_flash_p0.1_b128_{b128}'] = ({}, f)

        def ff(b128=b128):
            lib.mlc_flash_bwd128(b128)
            Tx._FLASH_ONLY = True
            return Tx.attn_fwd(qkv, kb, B, S, H, scale, 0.1, seed, 7)
        fns[f'attn_fwd_flash_p0.1_b128_{b128}'] = ({}, ff)
    for kern in ('tile', 'flash'):
        Tx._FLASH_ONLY = kern == 'flash'
        for p in (0.0, 0.1):
            ctx, lse = Tx.attn_fwd(qkv, kb, B, S, H, scale, p, seed, 7)
            res[(kern, p)] = (ctx, lse)
            fl = Tx._FLASH_ONLY
            fns[f'attn_fwd_{kern}_p{p}'] = ({}, lambda p=p, fl=fl: (setattr(Tx, '_FLASH_ONLY', fl),
                                                                      Tx.attn_fwd(qkv, kb, B, S, H, scale, p, seed, 7)))
            fns[f'attn_bwd_{kern}_p{p}'] = ({}, lambda p=p, fl=fl, c=ctx, l=lse: (
                setattr(Tx, '_FLASH_ONLY', fl),
                Tx.attn_bwd(qkv, kb, dctx, l, B, S, H, scale, p, seed, 7, ctx=c)))
    x = torch.randn(T, E, device=dev).to(torch.bfloat16)
    r = torch.randn(T, E, device=dev).to(torch.bfloat16)
    gamma = torch.ones(E, device=dev)
    beta = torch.zeros(E, device=dev)
    for p in (0.0, 0.1):
        fns[f'ln_fwd_p{p}'] = ({}, lambda p=p: Tx.ln_fwd(x, r, gamma, beta, p_in=p, seed=seed, salt_in=3))
    y, s, mean, rstd = Tx.ln_fwd(x, r, gamma, beta, p_in=0.1, seed=seed, salt_in=3)
    dg = torch.zeros(E, device=dev)
    db = torch.zeros(E, device=dev)
    for p in (0.0, 0.1):
        fns[f'ln_bwd_p{p}'] = ({}, lambda p=p: Tx.ln_bwd(dctx, s, mean, rstd, gamma, dg, db, want_dr=True,
                                                         p_in=p, seed=seed, salt_in=3))
    n = 110_000_000
    pa = torch.randn(n, device=dev)
    gr = torch.randn(n, device=dev) * 1e-3
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
    hyper = torch.tensor([1e-4, 1.0, 0.1, 0.001], device=dev)
    for var in (0, 1, 2):    # Adam kernel variants (mlc_opt_config key 0)
        def adam(var=var):
            _lib.load().mlc_opt_config(0, var)
            _lib.call('mlc_adam', _lib.ptr(pa), _lib.ptr(gr), _lib.ptr(m), _lib.ptr(v), _lib.ptr(pbf),
                      _lib.ptr(hyper), n, n - 1_000_000, n - 1_000_000, 0.9, 0.999, 1e-8, 0.01, 1, _lib.stream())
        fns[f'adam_110M_v{var}'] = ({}, adam)
    t = graph_time(fns, rounds=5, iters=10)
    for var in (0, 1, 2):
        t[f'adam_110M_v{var}_TBps'] = round(n * 30 / (t[f'adam_110M_v{var}'] * 1e-6) / 1e12, 2)
    print(json.dumps(t), flush=True)


if __name__ == '__main__':
    main()
