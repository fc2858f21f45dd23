"""GEMM throughput of the native MFMA kernel (dense-layer entry point, with and without
split-K) vs the library GEMM behind torch.matmul (hipBLASLt), on BERT-base / ResNet
shapes.  python scripts/bench_gemm.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlcomp_amd.ops import _lib
from mlcomp_amd.ops import transformer as Tx

SHAPES = [  # (M, N, K, name)
    (4096, 2304, 768, 'bert qkv'), (4096, 768, 768, 'bert out'), (4096, 3072, 768, 'bert ffn1'),
    (4096, 768, 3072, 'bert ffn2'), (4096, 768, 2304, 'bert qkv dgrad'), (4096, 4096, 4096, 'square 4k'),
    (8192, 8192, 8192, 'square 8k'), (802816, 256, 64, 'r50 l1 1x1 64->256'), (200704, 512, 128, 'r50 l2 1x1'),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    for M, N, K, name in SHAPES:
        x = torch.randn(M, K, device='cuda').to(torch.bfloat16)
        w = (torch.randn(N, K, device='cuda') * K ** -0.5).to(torch.bfloat16)
        b = torch.zeros(N, device='cuda')
        fl = 2.0 * M * N * K
        t_lib = timeit(lambda: torch.matmul(x, w.t()))
        dy = torch.randn(M, N, device='cuda').to(torch.bfloat16)
        t_dgl = timeit(lambda: torch.matmul(dy, w))
        res = []
        lib = _lib.load()
        for big in (0, 1):
            old = lib.mlc_gemm_get_set(3, big)
            t_nat = timeit(lambda: Tx.dense_fwd(x, w, b))
            t_dg = timeit(lambda: Tx.dense_dgrad(dy, w))
            lib.mlc_gemm_get_set(3, old)
            res.append(f'big{big} fwd {fl / t_nat / 1e12:6.1f} dgrad {fl / t_dg / 1e12:6.1f}')
        print(f'{name:20s} M={M:7d} N={N:5d} K={K:5d} | lib fwd {fl / t_lib / 1e12:6.1f} dgrad '
              f'{fl / t_dgl / 1e12:6.1f} | ' + ' | '.join(res) + '  TF/s', flush=True)


if __name__ == '__main__':
    main()
