"""Persistent short-K GEMM (igemm.hip gemm_persist_kernel, knob 14) vs the per-tile LDS-DMA
kernel on ResNet-50's forward 1x1 convs (batch 512, BN-statistics epilogue) and the dense
forward GEMMs of BERT-base / ViT-B/16, timed in graphs; one JSON line per shape with us per
variant and the achieved GB/s of the minimal operand bytes.

    python scripts/bench_persist.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402
from bench_expand_1x1 import timeit  # noqa: E402


def variants(lib, run):
    out = {}
    for name, (p, nb) in {'tile': (0, 3), 'persist3': (1, 3), 'persist2': (1, 2)}.items():
        def f(p=p, nb=nb):
            lib.mlc_gemm_get_set(14, p)
            lib.mlc_gemm_get_set(15, nb)
            run()
        out[name] = f
    return out


def main():
    lib = _lib.load()
    N = int(os.environ.get('BATCH', 512))
    rows = []
    for H, C, Co, S in [(56, 64, 256, 1), (56, 256, 64, 1), (56, 256, 128, 1), (28, 128, 512, 1), (28, 512, 128, 1),
                        (14, 256, 1024, 1), (14, 1024, 256, 1), (7, 512, 2048, 1), (7, 2048, 512, 1),
                        (56, 256, 512, 2), (28, 512, 1024, 2)]:
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, C, device='cuda') * C ** -0.5).to(torch.bfloat16)
        Ho = H // S
        y = torch.empty(N, Ho, Ho, Co, device='cuda', dtype=torch.bfloat16)
        st = torch.zeros(2, Fn.NSTAT * Co, device='cuda')
        ref = Fn.conv2d_fwd(x, w, S, 0, 1).float()
        fns = variants(lib, lambda: Fn.conv2d_fwd(x, w, S, 0, 1, stats=(st[0], st[1]), out=y))
        t = timeit(fns)
        for k, f in fns.items():        # each variant's output equals the plain conv
            f()
            torch.cuda.synchronize()
            assert (y.float() - ref).abs().max() <= 1e-2 * ref.abs().max() + 1e-3, k
        byts = x.numel() * 2 + y.numel() * 2
        rows.append({'shape': f'conv1x1 {H}x{H} {C}>{Co} /{S}', 'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                     'GBps': {k: round(byts / (v * 1e-3) / 1e9) for k, v in t.items()}})
        print(json.dumps(rows[-1]), flush=True)
    for M, K, Nn in [(4096, 768, 2304), (4096, 768, 3072), (4096, 3072, 768), (25216, 768, 2304), (25216, 768, 3072)]:
        x = (torch.randn(M, K, device='cuda') * 0.5).to(torch.bfloat16)
        w = (torch.randn(Nn, K, device='cuda') * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(Nn, device='cuda') * 0.1
        fns = variants(lib, lambda: Tx.dense_fwd(x, w, None))
        t = timeit(fns)
        fl = 2 * M * K * Nn
        rows.append({'shape': f'dense {M}x{K}>{Nn}', 'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                     'TFs': {k: round(fl / (v * 1e-3) / 1e12) for k, v in t.items()}})
        print(json.dumps(rows[-1]), flush=True)
    lib.mlc_gemm_get_set(14, 0)


if __name__ == '__main__':
    main()
