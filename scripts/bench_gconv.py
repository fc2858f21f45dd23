"""ResNeXt-50 32x4d's grouped 3x3 convs (gconv.hip) at batch 128: forward (with BN stats),
input gradient and weight gradient per shape, timed in HIP graphs; prints one JSON line per
shape with the microseconds and the achieved bandwidth of the minimal operand bytes.

    python scripts/bench_gconv.py

Round 5 (profiles/round5/generic/gconv_resnext_b128.jsonl): ~1 TB/s of the minimal operand
bytes (the strided input gradients 0.4-0.8 TB/s), 4.9 ms per ResNeXt-50 step; four sub-tiles
per wave, a fully unrolled K loop and a one-iteration gather prefetch in the weight gradient
each measured within 2 % (not kept).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import functional as Fn  # noqa: E402


def timeit(fns, rounds=5, iters=10):
    graphs = {}
    for k, f in fns.items():
        f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                f()
        graphs[k] = g
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, g in graphs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def main():
    N = int(os.environ.get('BATCH', 128))
    tot = {'fwd': 0.0, 'dgrad': 0.0, 'wgrad': 0.0}
    for H, C, s, cnt in [(56, 128, 1, 3), (56, 256, 2, 1), (28, 256, 1, 3), (28, 512, 2, 1), (14, 512, 1, 5),
                         (14, 1024, 2, 1), (7, 1024, 1, 2)]:
        groups = 32
        Ho = (H + 2 - 3) // s + 1
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C // groups, device='cuda') * 0.1).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, C, device='cuda').to(torch.bfloat16)
        st = torch.zeros(2, Fn.NSTAT * C, device='cuda')
        dw = torch.zeros(C, 3, 3, C // groups, device='cuda')
        t = timeit({'fwd': lambda: Fn.gconv_fwd(x, w, groups, s, 1, 1, stats=(st[0], st[1])),
                    'dgrad': lambda: Fn.gconv_dgrad(dy, w, x.shape, groups, s, 1, 1),
                    'wgrad': lambda: Fn.gconv_wgrad(dy, x, w.shape, groups, s, 1, 1, out=dw, accumulate=True)})
        byts = (x.numel() + dy.numel()) * 2
        for k in tot:
            tot[k] += cnt * t[k]
        print(json.dumps({'shape': [N, H, C, s], 'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                          'GBps': {k: round(byts / v / 1e6) for k, v in t.items()}}), flush=True)
    print(json.dumps({'weighted_ms': {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == '__main__':
    main()
