"""Three-wide dense tiles (igemm TileCfg WIDE3: 128x96 / 128x192 / 128x288) against the
128x128 (+ split-K) path and hipBLASLt on BERT-base's K-contiguous dense GEMMs (forward with
the real epilogues; input gradients through the transposed-weight copy).  Every config is
checked against an fp32 reference first, then timed in interleaved rounds in one process.

    python scripts/bench_dense_tiles.py            # one JSON line per shape
"""
import json
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402

CONFIGS = [('sq', 0, 1), ('96', 5, 1), ('192', 6, 1), ('288', 7, 1), ('96s2', 5, 2), ('192s2', 6, 2)]


def knob(tile, split):
    lib = _lib.load()
    lib.mlc_gemm_get_set(10, tile)
    lib.mlc_gemm_get_set(11, split)


def r(*s):
    return torch.rand(*s, device='cuda').sub(0.5).to(torch.bfloat16)


def timeit(fns, rounds=7, iters=20):
    """fns: name -> (setup, fn).  Each config's `iters` launches are captured into one HIP
    graph (setup runs before capture: the knob is host state read at launch time), so the
    timing is GPU time, not Python launch overhead."""
    graphs = {}
    for k, (setup, f) in fns.items():
        setup()
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


def gelu(u):
    return 0.5 * u * (1.0 + torch.erf(u * 0.7071067811865476))


def main():
    M = 4096
    shapes = [  # (tag, N, K, act, addend)
        ('qkv fwd', 2304, 768, 0, False), ('ffn1 fwd', 3072, 768, 1, False),
        ('ffn2 fwd', 768, 3072, 0, True), ('out fwd', 768, 768, 0, True),
        ('qkv dgrad', 768, 2304, 0, True), ('ffn1 dgrad', 768, 3072, 0, True),
        ('ffn2 dgrad', 3072, 768, 0, False), ('out dgrad', 768, 768, 0, False)]
    bad = 0
    for tag, N, K, act, add in shapes:
        x, w = r(M, K), r(N, K)
        b = torch.randn(N, device='cuda') * 0.1
        a = r(M, N) if add else None

        def run():
            if add:
                y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
                ws = Tx.gemm_workspace(x.device, 4 * M * N)
                _lib.call('mlc_gemm_bf16_ex', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), M, N, K, K, K, N, 0, 1,
                          _lib.ptr(b), act, None, _lib.ptr(a), None, _lib.ptr(ws), 4 * M * N, _lib.stream())
                return y
            return Tx.dense_fwd(x, w, b, act=act)[0]
        ref = x.float() @ w.float().t() + b
        if act:
            ref = gelu(ref)
        if add:
            ref = ref + a.float()
        errs = {}
        for name, tile, split in CONFIGS:
            knob(tile, split)
            y = run().float()
            torch.cuda.synchronize()
            errs[name] = ((y - ref).abs().max() / ref.abs().max()).item()
            if not errs[name] < 2e-2:
                bad += 1
        fns = {}
        for name, tile, split in CONFIGS:
            fns[name] = (lambda t=tile, s=split: knob(t, s), run)
        fns['hipblaslt'] = (lambda: None, lambda: torch.mm(x, w.t()))
        t = timeit(fns)
        knob(0, 1)
        fl = 2.0 * M * N * K
        print(json.dumps({'shape': tag, 'MNK': [M, N, K],
                          'TF': {k: round(fl / v / 1e9, 1) for k, v in t.items()},
                          'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                          'max_rel_err': {k: round(v, 5) for k, v in errs.items()}}), flush=True)
    if bad:
        print(f'NUMERICS FAILED in {bad} config(s)')
        sys.exit(1)


if __name__ == '__main__':
    main()
