"""Per-shape cost of every ResNet-50 convolution (batch 256, 224x224, NHWC bf16) on the
native implicit-GEMM kernels vs MIOpen (torch channels_last bf16), with the roofline
numbers (TF/s of the GEMM work, GB/s of the minimal operand bytes) and the per-step
total weighted by how often each shape occurs in the network.

    python scripts/bench_convs.py [--batch 256] [--iters 10]
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlcomp_amd.ops import functional as Fn  # noqa: E402

# (name, H, Cin, Cout, k, stride, count in ResNet-50)
SHAPES = [
    ('stem 7x7/2', 224, 8, 64, 7, 2, 1),
    ('l1 1x1 64>64', 56, 64, 64, 1, 1, 1),
    ('l1 3x3 64', 56, 64, 64, 3, 1, 3),
    ('l1 1x1 64>256', 56, 64, 256, 1, 1, 4),     # 3 expand + downsample
    ('l1 1x1 256>64', 56, 256, 64, 1, 1, 2),
    ('l2 1x1 256>128', 56, 256, 128, 1, 1, 1),
    ('l2 3x3/2 128', 56, 128, 128, 3, 2, 1),
    ('l2 1x1/2 256>512 ds', 56, 256, 512, 1, 2, 1),
    ('l2 1x1 128>512', 28, 128, 512, 1, 1, 4),
    ('l2 1x1 512>128', 28, 512, 128, 1, 1, 3),
    ('l2 3x3 128', 28, 128, 128, 3, 1, 3),
    ('l3 1x1 512>256', 28, 512, 256, 1, 1, 1),
    ('l3 3x3/2 256', 28, 256, 256, 3, 2, 1),
    ('l3 1x1/2 512>1024 ds', 28, 512, 1024, 1, 2, 1),
    ('l3 1x1 256>1024', 14, 256, 1024, 1, 1, 6),
    ('l3 1x1 1024>256', 14, 1024, 256, 1, 1, 5),
    ('l3 3x3 256', 14, 256, 256, 3, 1, 5),
    ('l4 1x1 1024>512', 14, 1024, 512, 1, 1, 1),
    ('l4 3x3/2 512', 14, 512, 512, 3, 2, 1),
    ('l4 1x1/2 1024>2048 ds', 14, 1024, 2048, 1, 2, 1),
    ('l4 1x1 512>2048', 7, 512, 2048, 1, 1, 3),
    ('l4 1x1 2048>512', 7, 2048, 512, 1, 1, 2),
    ('l4 3x3 512', 7, 512, 512, 3, 1, 2),
]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--torch', type=int, default=1)
    ap.add_argument('--split-targets', default='',
                    help='comma list: also time wgrad at these split-K block targets')
    a = ap.parse_args()
    targets = [int(t) for t in a.split_targets.split(',') if t]
    from mlcomp_amd.ops import _lib
    sweep = {t: 0.0 for t in targets}
    N = a.batch
    tot = {'nf': 0.0, 'nd': 0.0, 'nw': 0.0, 'tf': 0.0, 'td': 0.0, 'tw': 0.0}
    print(f'{"shape":24s} {"us fwd/dgrad/wgrad (native)":>30s} {"TF/s":>17s} {"GB/s fwd":>8s} | '
          f'{"us (MIOpen)":>22s}', flush=True)
    for name, H, C, Co, k, s, cnt in SHAPES:
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, k, k, C, device='cuda') * (k * k * C) ** -0.5).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, Co, device='cuda').to(torch.bfloat16)
        y = torch.empty(N, Ho, Ho, Co, device='cuda', dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        dw = torch.empty(Co, k, k, C, device='cuda', dtype=torch.float32)
        fl = 2.0 * N * Ho * Ho * Co * k * k * C
        tf = timeit(lambda: Fn.conv2d_fwd(x, w, s, p, out=y), a.iters)
        td = timeit(lambda: Fn.conv2d_dgrad(dy, w, x.shape, s, p, out=dx), a.iters) if name != 'stem 7x7/2' else 0.0
        tw = timeit(lambda: Fn.conv2d_wgrad(dy, x, w.shape, s, p, out=dw), a.iters)
        byts = x.numel() * 2 + y.numel() * 2 + w.numel() * 2
        tot['nf'] += cnt * tf
        tot['nd'] += cnt * td
        tot['nw'] += cnt * tw
        line = (f'{name:24s} {tf * 1e6:9.1f} {td * 1e6:9.1f} {tw * 1e6:9.1f}   '
                f'{fl / tf / 1e12:5.0f} {fl / td / 1e12 if td else 0:5.0f} {fl / tw / 1e12:5.0f} '
                f'{byts / tf / 1e9:8.0f}')
        if targets:
            parts = []
            for tg in targets:
                old = _lib.load().mlc_gemm_get_set(1, tg)
                tt = timeit(lambda: Fn.conv2d_wgrad(dy, x, w.shape, s, p, out=dw), a.iters)
                _lib.load().mlc_gemm_get_set(1, old)
                sweep[tg] += cnt * tt
                parts.append(f'{tg}:{tt * 1e6:.1f}')
            line += ' | wgrad@' + ' '.join(parts)
        if a.torch:
            xt = x.permute(0, 3, 1, 2)          # channels_last views
            wt = w.permute(0, 3, 1, 2)
            dyt = dy.permute(0, 3, 1, 2)
            t1 = timeit(lambda: F.conv2d(xt, wt, None, s, p), a.iters)
            t2 = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wt, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (True, False, False)), a.iters)
            t3 = timeit(lambda: torch.ops.aten.convolution_backward(
                dyt, xt, wt, None, (s, s), (p, p), (1, 1), False, (0, 0), 1, (False, True, False)), a.iters)
            tot['tf'] += cnt * t1
            tot['td'] += cnt * t2
            tot['tw'] += cnt * t3
            line += f' | {t1 * 1e6:7.1f} {t2 * 1e6:7.1f} {t3 * 1e6:7.1f}'
        print(line, flush=True)
        del x, w, dy, y, dx, dw
    print(f'weighted per step (ms): native fwd {tot["nf"] * 1e3:.2f} dgrad {tot["nd"] * 1e3:.2f} '
          f'wgrad {tot["nw"] * 1e3:.2f} | MIOpen fwd {tot["tf"] * 1e3:.2f} dgrad {tot["td"] * 1e3:.2f} '
          f'wgrad {tot["tw"] * 1e3:.2f}', flush=True)
    if targets:
        print('wgrad per step by split target (ms): ' + ' '.join(f'{t}:{v * 1e3:.2f}' for t, v in sweep.items()))


if __name__ == '__main__':
    main()
