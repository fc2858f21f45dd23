"""Per-shape native vs hipBLASLt selection (csrc/bench/blaslt.hip; run with
MLC_KERNEL_LIB=mlcomp_amd/_native/libmlcomp_kernels_blaslt.so) on BERT-base's dense
GEMMs: every form (bias forward, residual-addend input gradient, plain input gradient,
weight + bias gradient) is checked against an fp32 reference under both forced modes,
then the auto mode's timed choice is printed per shape as one JSON line.

    python scripts/bench_blaslt_select.py
"""
import ctypes
import json
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def r(*s):
    return torch.rand(*s, device='cuda').sub(0.5).to(torch.bfloat16)


def choices():
    lib = _lib.load()
    buf = (ctypes.c_int * 2560)()
    n = lib.mlc_blaslt_choices(buf, 256)
    rows = [list(buf[10 * i:10 * i + 10]) for i in range(n)]
    return [{'kind': ['bf16', 'wgrad'][k], 'MNK': [M, N, K], 'ta': ta, 'tb': tb, 'epi': e,
             'pick': 'native' if p < 0 else f'hipblaslt#{p}', 'native_us': tn / 1e3, 'lib_us': tl / 1e3}
            for k, M, N, K, ta, tb, e, p, tn, tl in rows]


def main():
    lib = _lib.load()
    M = 4096
    cases = [('qkv fwd', 'fwd', 2304, 768), ('out fwd', 'fwd', 768, 768), ('ffn2 fwd', 'fwd', 768, 3072),
             ('ffn1 fwd gelu', 'gelu', 3072, 768),
             ('qkv dgrad +res', 'dgrad_add', 2304, 768), ('out dgrad', 'dgrad', 768, 768),
             ('ffn1 dgrad +res', 'dgrad_add', 3072, 768), ('ffn2 dgrad dgelu', 'dgrad_dact', 768, 3072),
             ('qkv wgrad', 'wgrad', 2304, 768), ('out wgrad', 'wgrad', 768, 768),
             ('ffn1 wgrad', 'wgrad', 3072, 768), ('ffn2 wgrad', 'wgrad', 768, 3072)]
    bad = []
    for tag, kind, N, K in cases:
        x, w = r(M, K), r(N, K)
        b = torch.randn(N, device='cuda') * 0.1
        dy = r(M, N)
        add = r(M, K)
        u = r(M, K)

        def run():
            if kind == 'fwd':
                return Tx.dense_fwd(x, w, b)[0].float()
            if kind == 'gelu':
                return Tx.dense_fwd(x, w, b, act=1)[0].float()
            if kind == 'dgrad_add':
                return Tx.dense_dgrad(dy, w, addend=add).float()
            if kind == 'dgrad':
                return Tx.dense_dgrad(dy, w).float()
            if kind == 'dgrad_dact':
                return Tx.dense_dgrad(dy, w, dact_u=u, dact_is_deriv=True).float()
            dw = torch.ones(N, K, device='cuda')
            db = torch.ones(N, device='cuda')
            Fn.linear_wgrad_bias(dy, x, dw, db)
            return torch.cat([dw.flatten(), db])

        if kind in ('fwd', 'gelu'):
            ref = x.float() @ w.float().t() + b
            if kind == 'gelu':
                ref = 0.5 * ref * (1 + torch.erf(ref * 0.7071067811865476))
        elif kind.startswith('dgrad'):
            ref = dy.float() @ w.float()
            if kind == 'dgrad_add':
                ref = ref.bfloat16().float() + add.float()
            if kind == 'dgrad_dact':
                ref = ref.bfloat16().float() * u.float()
        else:
            ref = torch.cat([(dy.float().t() @ x.float() + 1).flatten(), dy.float().sum(0) + 1])
        errs = {}
        for mode in (0, 1):
            lib.mlc_blaslt_mode(mode)
            got = run()
            torch.cuda.synchronize()
            errs[mode] = float((got - ref).abs().max() / ref.abs().max())
            if not errs[mode] < 2e-2:
                bad.append((tag, mode, errs[mode]))
        lib.mlc_blaslt_mode(2)
        run()
        torch.cuda.synchronize()
        ch = choices()
        print(json.dumps({'shape': tag, 'M': M, 'N': N, 'K': K, 'err_native': round(errs[0], 5),
                          'err_forced_lib': round(errs[1], 5), 'choices': ch}), flush=True)
    if bad:
        print('NUMERICS FAILED', bad)
        sys.exit(1)


if __name__ == '__main__':
    main()
