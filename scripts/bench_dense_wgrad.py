"""BERT-base dense weight + bias gradients (dW [O, I] += dY^T X, db += colsum(dY); M = 4096
tokens) on the native kernel at several split-K factors, against hipBLASLt's plain
dY^T X (torch.mm, bf16 out, no bias).  Every config is checked against fp32, then timed in
interleaved rounds, each config's launches captured in one HIP graph.

    python scripts/bench_dense_wgrad.py [M]     # one JSON line per shape
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import _lib  # noqa: E402


def timeit(fns, rounds=7, iters=20):
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
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    _lib.load()
    shapes = [('qkv', 2304, 768), ('out', 768, 768), ('ffn1', 3072, 768), ('ffn2', 768, 3072)]
    bad = 0
    for tag, O, I in shapes:
        dy = torch.rand(M, O, device='cuda').sub(0.5).to(torch.bfloat16)
        x = torch.rand(M, I, device='cuda').sub(0.5).to(torch.bfloat16)
        dw = torch.zeros(O, I, device='cuda')
        db = torch.zeros(O, device='cuda')
        ws = torch.empty(16 * O * I, device='cuda')

        def native(split, slab):
            def f():
                _lib.call('mlc_linear_wgrad_bias_native', _lib.ptr(dy), _lib.ptr(x), _lib.ptr(dw), _lib.ptr(db),
                          O, I, M, O, I, I, split, _lib.ptr(ws) if slab else None, ws.numel() if slab else 0,
                          _lib.stream())
            return f
        cfgs = {'auto': native(0, True)}
        for s in (1, 2, 4, 8):
            cfgs[f's{s}'] = native(s, False)
            if s > 1:
                cfgs[f's{s}slab'] = native(s, True)
        ref = dy.float().t() @ x.float()
        errs = {}
        for name, f in cfgs.items():
            dw.zero_()
            db.zero_()
            f()
            torch.cuda.synchronize()
            errs[name] = ((dw - ref).abs().max() / ref.abs().max()).item()
            if not errs[name] < 1e-2:
                bad += 1
        fns = dict(cfgs)
        fns['hipblaslt'] = lambda: torch.mm(dy.t(), x)
        t = timeit(fns)
        fl = 2.0 * M * O * I
        print(json.dumps({'shape': tag, 'OIM': [O, I, M],
                          'TF': {k: round(fl / v / 1e9, 1) for k, v in t.items()},
                          'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                          'max_rel_err': {k: round(v, 5) for k, v in errs.items()}}), flush=True)
    if bad:
        print(f'NUMERICS FAILED in {bad} config(s)')
        sys.exit(1)


if __name__ == '__main__':
    main()
