"""ResNet-50 1x1 convolutions (batch 256, NHWC bf16) on the implicit-GEMM engine under
main-loop variants, against hipBLASLt (torch.matmul on the same [M,K]x[K,N] GEMM) and
the HBM floor (minimal operand + output bytes at 6.3 TB/s).

Forward runs with the BN-statistics epilogue (as in the training step); the input
gradient runs through the transposed-filter path (``wt``: both operands K-contiguous).
Each config's launches are captured into one HIP graph and timed in interleaved rounds
in one process.

    python scripts/bench_1x1.py
"""
import json
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import functional as Fn  # noqa: E402

# (name, H, Cin, Cout, count per step)
SHAPES = [
    ('l1 64>64', 56, 64, 64, 1), ('l1 64>256', 56, 64, 256, 4), ('l1 256>64', 56, 256, 64, 2),
    ('l2 256>128', 56, 256, 128, 1), ('l2 128>512', 28, 128, 512, 4), ('l2 512>128', 28, 512, 128, 3),
    ('l3 512>256', 28, 512, 256, 1), ('l3 256>1024', 14, 256, 1024, 6), ('l3 1024>256', 14, 1024, 256, 5),
    ('l4 1024>512', 14, 1024, 512, 1), ('l4 512>2048', 7, 512, 2048, 3), ('l4 2048>512', 7, 2048, 512, 2),
]
# (tag, {knob: value}) - knob 8: LDS-DMA main loop on/off, knob 0: register prefetch depth.
# (The ss4 / ss16 columns of profiles/round3/streamk/bench_1x1.jsonl came from a
# single-stage knob that was removed with the variant; knob 12 is now a dense-GEMM knob.)
CONFIGS = [('base', {}), ('nodma', {8: 0}), ('nodma_pf1', {8: 0, 0: 1})]


def set_knobs(kn):
    lib = _lib.load()
    return {k: lib.mlc_gemm_get_set(k, v) for k, v in kn.items()}


def graph_time(fns, rounds=7, iters=20):
    graphs = {}
    for k, (kn, f) in fns.items():
        old = set_knobs(kn)
        f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                f()
        set_knobs(old)
        graphs[k] = g
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, g in graphs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) * 1e3 / iters)
    return {k: round(sorted(v)[len(v) // 2], 2) for k, v in times.items()}


def main():
    N = 256
    tot = {}
    for name, H, C, Co, cnt in SHAPES:
        M = N * H * H
        x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, C, device='cuda') * C ** -0.5).to(torch.bfloat16)
        wt = Fn.wt_flip_transpose(w)
        dy = torch.randn(N, H, H, Co, device='cuda').to(torch.bfloat16)
        y = torch.empty(N, H, H, Co, device='cuda', dtype=torch.bfloat16)
        dx = torch.empty_like(x)
        s1, s2 = Fn.stat_buffers(Co, x.device)
        # numerics once (default config) against fp32
        Fn.conv2d_fwd(x, w, stats=(s1, s2), out=y)
        ref = (x.float().reshape(M, C) @ w.float().reshape(Co, C).t())
        err = ((y.float().reshape(M, Co) - ref).abs().max() / ref.abs().max()).item()
        fns = {}
        for tag, kn in CONFIGS:
            fns['fwd_' + tag] = (kn, lambda: Fn.conv2d_fwd(x, w, stats=(s1, s2), out=y))
            fns['dgrad_' + tag] = (kn, lambda: Fn.conv2d_dgrad(dy, w, x.shape, out=dx, wt=wt))
        a2, b2 = x.reshape(M, C), w.reshape(Co, C).t().contiguous()
        d2, wt2 = dy.reshape(M, Co), w.reshape(Co, C).contiguous()
        fns['fwd_blas'] = ({}, lambda: torch.matmul(a2, b2))
        fns['dgrad_blas'] = ({}, lambda: torch.matmul(d2, wt2))
        t = graph_time(fns)
        floor_f = (M * C + M * Co) * 2 / 6.3e12 * 1e6
        rec = {'shape': name, 'M': M, 'K': C, 'N': Co, 'count': cnt, 'err': round(err, 4),
               'floor_us': round(floor_f, 1), 'tflop': round(2 * M * C * Co / 1e12, 4), 'us': t}
        for k, v in t.items():
            tot[k] = tot.get(k, 0.0) + cnt * v
        print(json.dumps(rec), flush=True)
        del x, w, wt, dy, y, dx
    print(json.dumps({'per_step_us': {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == '__main__':
    main()
