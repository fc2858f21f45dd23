"""Cost of the BN-statistics epilogue (per-column sum / sum-of-squares atomics) on the
ResNet-50 1x1 forward convs: the same conv with and without ``stats``, graph-timed in
interleaved rounds (scripts/bench_1x1.graph_time).

    python scripts/bench_conv_stats.py
"""
import json
import sys

import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'scripts')
from bench_1x1 import SHAPES, graph_time  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402


def main():
    dev = torch.device('cuda')
    tot = {'stats': 0.0, 'plain': 0.0}
    for name, H, Ci, Co, count in SHAPES:
        x = torch.randn(256, H, H, Ci, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, Ci, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(256, H, H, Co, device=dev, dtype=torch.bfloat16)
        s1, s2 = Fn.stat_buffers(Co, dev)
        fns = {'stats': ({}, lambda: Fn.conv2d_fwd(x, w, stats=(s1, s2), out=y)),
               'plain': ({}, lambda: Fn.conv2d_fwd(x, w, out=y))}
        t = graph_time(fns)
        for k in tot:
            tot[k] += t[k] * count
        print(json.dumps({'shape': name, 'count': count, 'us': t}), flush=True)
    print(json.dumps({'per_step_us': {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == '__main__':
    main()
