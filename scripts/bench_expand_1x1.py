"""ResNet-50's channel-expanding 1x1 convs (64->256 ... 512->2048, batch 512) on the forward
path with the BN-statistics epilogue, per main-loop variant (knob 13: the single-LDS-stage
loop, 4 blocks per CU, for splits of up to 1 / 2 / 4 K-tiles), timed in graphs, reported as achieved HBM GB/s of the
minimal operand bytes (these GEMMs are output-write bound).

    python scripts/bench_expand_1x1.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import _lib  # noqa: E402
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
    lib = _lib.load()
    N = int(os.environ.get('BATCH', 512))
    for H, C, Co in [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048), (56, 256, 64), (28, 512, 128)]:
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, C, device='cuda') * C ** -0.5).to(torch.bfloat16)
        y = torch.empty(N, H, H, Co, device='cuda', dtype=torch.bfloat16)
        st = torch.zeros(2, Fn.NSTAT * Co, device='cuda')
        fns = {}
        for kt in (1, 2, 4):     # single-LDS-stage variant up to kt K-tiles (knob 13)
            def mk(stats, kt=kt):
                def f():
                    lib.mlc_gemm_get_set(13, kt)
                    Fn.conv2d_fwd(x, w, 1, 0, 1, stats=(st[0], st[1]) if stats else None, out=y)
                return f
            fns[f'stats_kt{kt}'] = mk(True)
        t = timeit(fns)
        lib.mlc_gemm_get_set(13, 1)
        byts = x.numel() * 2 + y.numel() * 2
        print(json.dumps({'shape': [N, H, C, Co], 'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                          'GBps': {k: round(byts / v / 1e6) for k, v in t.items()}}), flush=True)


if __name__ == '__main__':
    main()
