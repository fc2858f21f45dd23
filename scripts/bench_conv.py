"""Per-shape conv microbenchmark: mlcomp_amd HIP implicit-GEMM vs MIOpen (PyTorch).

For every distinct conv of ResNet-50 at the bench batch, times fwd / dgrad / wgrad of
both implementations (same bf16 NHWC data, interleaved in one process) and prints a
table with TFLOP/s.  Usage: python scripts/bench_conv.py [--batch 256] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import functional as Fn  # noqa: E402

# (H, C, Co, K, stride, count in resnet50) at input resolution H
SHAPES = [
    (224, 8, 64, 7, 2, 1),
    (56, 64, 64, 1, 1, 1), (56, 64, 64, 3, 1, 3), (56, 64, 256, 1, 1, 4), (56, 256, 64, 1, 1, 2),
    (56, 256, 128, 1, 1, 1), (56, 128, 128, 3, 2, 1), (56, 256, 512, 1, 2, 1),
    (28, 128, 512, 1, 1, 4), (28, 512, 128, 1, 1, 3), (28, 128, 128, 3, 1, 3),
    (28, 512, 256, 1, 1, 1), (28, 256, 256, 3, 2, 1), (28, 512, 1024, 1, 2, 1),
    (14, 256, 1024, 1, 1, 6), (14, 1024, 256, 1, 1, 5), (14, 256, 256, 3, 1, 5),
    (14, 1024, 512, 1, 1, 1), (14, 512, 512, 3, 2, 1), (14, 1024, 2048, 1, 2, 1),
    (7, 512, 2048, 1, 1, 3), (7, 2048, 512, 1, 1, 2), (7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--json', default=None)
    a = ap.parse_args()
    dev = 'cuda'
    N = a.batch
    rows = []
    tot = {'ours': 0.0, 'miopen': 0.0}
    print(f"{'shape':32s} {'op':6s} {'ours ms':>8s} {'TF':>6s} {'miopen ms':>9s} {'TF':>6s} {'x':>5s}")
    for (H, C, Co, K, s, cnt) in SHAPES:
        p = (K - 1) // 2
        Ho = (H + 2 * p - K) // s + 1
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, K, K, C, device=dev) * (K * K * C) ** -0.5).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, Co, device=dev).to(torch.bfloat16)
        s1, s2 = Fn.stat_buffers(Co, dev)
        dw = torch.empty(Co, K, K, C, device=dev)
        xt = x.permute(0, 3, 1, 2)  # NCHW view of NHWC memory == channels_last
        wt = w.permute(0, 3, 1, 2)
        dyt = dy.permute(0, 3, 1, 2)
        flops = 2.0 * N * Ho * Ho * Co * C * K * K
        ops = {
            'fwd': (lambda: Fn.conv2d_fwd(x, w, s, p, stats=(s1, s2)),
                    lambda: torch.nn.functional.conv2d(xt, wt, None, s, p)),
            'dgrad': (lambda: Fn.conv2d_dgrad(dy, w, x.shape, s, p),
                      lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, (s, s), (p, p), (1, 1),
                                                                  False, (0, 0), 1, (True, False, False))),
            'wgrad': (lambda: Fn.conv2d_wgrad(dy, x, w.shape, s, p, out=dw),
                      lambda: torch.ops.aten.convolution_backward(dyt, xt, wt, None, (s, s), (p, p), (1, 1),
                                                                  False, (0, 0), 1, (False, True, False))),
        }
        for op, (ours, ref) in ops.items():
            if op == 'dgrad' and C == 8:
                continue
            t_o = timeit(ours, a.iters)
            t_r = timeit(ref, a.iters)
            tot['ours'] += t_o * cnt
            tot['miopen'] += t_r * cnt
            name = f'{N}x{H}x{H}x{C}->{Co} k{K}s{s}'
            print(f"{name:32s} {op:6s} {t_o:8.3f} {flops / t_o / 1e9:6.0f} {t_r:9.3f} "
                  f"{flops / t_r / 1e9:6.0f} {t_r / t_o:5.2f}", flush=True)
            rows.append(dict(shape=name, op=op, count=cnt, ours_ms=t_o, miopen_ms=t_r,
                             ours_tflops=flops / t_o / 1e9, miopen_tflops=flops / t_r / 1e9))
    print(f"weighted total (x layer count): ours {tot['ours']:.2f} ms  miopen {tot['miopen']:.2f} ms")
    if a.json:
        with open(a.json, 'w') as f:
            json.dump({'rows': rows, 'total': tot, 'batch': N}, f, indent=1)


if __name__ == '__main__':
    main()
