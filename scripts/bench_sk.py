"""Stream-K A/B on every ResNet-50 forward conv (BN-statistics epilogue) and stride-1 input
gradient (transposed filter), batch 256: knob 13 = 0 (plain grid) vs stream-K thresholds.
Graph-timed, interleaved rounds in one process (scripts/bench_1x1.graph_time).

    python scripts/bench_sk.py [--thresholds 0,90,100]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_1x1 import graph_time  # noqa: E402
from bench_convs import SHAPES  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--thresholds', default='0,90,100')
    a = ap.parse_args()
    ths = [int(t) for t in a.thresholds.split(',')]
    N = 256
    tot = {}
    for name, H, C, Co, k, s, cnt in SHAPES:
        if name.startswith('stem'):
            continue
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, k, k, C, device='cuda') * (k * k * C) ** -0.5).to(torch.bfloat16)
        wt = Fn.wt_flip_transpose(w)
        dy = torch.randn(N, Ho, Ho, Co, device='cuda').to(torch.bfloat16)
        y = torch.empty(N, Ho, Ho, Co, device='cuda', dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        s1, s2 = Fn.stat_buffers(Co, x.device)
        fns = {}
        for th in ths:
            fns[f'fwd_{th}'] = ({13: th}, lambda: Fn.conv2d_fwd(x, w, s, p, stats=(s1, s2), out=y))
            fns[f'dgrad_{th}'] = ({13: th}, lambda: Fn.conv2d_dgrad(dy, w, x.shape, s, p, out=dx, wt=wt))
        t = graph_time(fns)
        fl = 2.0 * N * Ho * Ho * Co * k * k * C
        rec = {'shape': name, 'count': cnt, 'us': t,
               'tflops': {kk: round(fl / v / 1e6, 0) for kk, v in t.items()}}
        for kk, v in t.items():
            tot[kk] = tot.get(kk, 0.0) + cnt * v
        print(json.dumps(rec), flush=True)
        del x, w, wt, dy, y, dx
    print(json.dumps({'per_step_us': {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == '__main__':
    main()
