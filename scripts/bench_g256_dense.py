"""The 256-row LDS-DMA engine (gemm256.hip ``mlc_g256_dense``, block tiles 256 x {128, 192,
256}) against the current dense path (igemm.hip, ``mlc_gemm_bf16_ex`` with the library
selection off) and hipBLASLt (``torch.mm``) on BERT-base's dense GEMMs with their real
epilogues: forward (bias; FFN1 GELU storing gelu'; residual addend) and input gradients
(through the transposed-weight copy, K-contiguous; residual addend; FFN2's gelu'
multiply).  Every config is checked against an fp32 reference, then timed in interleaved
rounds (each config's launches captured in one HIP graph).

    python scripts/bench_g256_dense.py [M]     # one JSON line per shape
"""
import json
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def r(*s):
    return torch.rand(*s, device='cuda').sub(0.5).to(torch.bfloat16)


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


def gelu(u):
    return 0.5 * u * (1.0 + torch.erf(u * 0.7071067811865476))


def dgelu(u):
    return 0.5 * (1.0 + torch.erf(u * 0.7071067811865476)) + u * torch.exp(-0.5 * u * u) * 0.3989422804014327


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    lib = _lib.load()
    shapes = [  # (tag, N, K, bias, act, addend, dact)
        ('qkv fwd', 2304, 768, True, 0, False, False), ('ffn1 fwd gelu', 3072, 768, True, 2, False, False),
        ('ffn2 fwd', 768, 3072, True, 0, True, False), ('out fwd', 768, 768, True, 0, True, False),
        ('qkv dgrad +res', 768, 2304, False, 0, True, False), ('ffn1 dgrad +res', 768, 3072, False, 0, True, False),
        ('ffn2 dgrad dgelu', 3072, 768, False, 4, False, True), ('out dgrad', 768, 768, False, 0, False, False)]
    bad = 0
    for tag, N, K, has_b, act, add, dact in shapes:
        x, w = r(M, K), r(N, K)
        b = (torch.randn(N, device='cuda') * 0.1) if has_b else None
        a = r(M, N) if add else None
        u = (torch.randn(M, N, device='cuda') * 0.5).to(torch.bfloat16) if dact else None
        d = dgelu(u.float()).to(torch.bfloat16) if dact else None     # the stored derivative (act 4)
        pre = torch.empty(M, N, device='cuda', dtype=torch.bfloat16) if act == 2 else None
        ws = Tx.gemm_workspace(x.device, 4 * M * N)

        def native():
            y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
            _lib.call('mlc_gemm_bf16_ex', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), M, N, K, K, K, N, 0, 1,
                      _lib.ptr(b), act, _lib.ptr(pre), _lib.ptr(a), _lib.ptr(d), _lib.ptr(ws), 4 * M * N,
                      _lib.stream())
            return y

        def g256(bn):
            def f():
                y = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
                _lib.call('mlc_g256_dense', _lib.ptr(x), _lib.ptr(w), _lib.ptr(y), M, N, K, K, K, N, 1, _lib.ptr(b),
                          act, _lib.ptr(pre), _lib.ptr(a), _lib.ptr(d), bn, _lib.stream())
                return y
            return f
        ref = x.float() @ w.float().t()
        if b is not None:
            ref = ref + b
        if act == 2:
            ref = gelu(ref)
        if dact:
            ref = ref * d.float()
        if a is not None:
            ref = ref + a.float()
        cfgs = {'native': native, 'g128': g256(128), 'g192': g256(192), 'g256': g256(256), 'gauto': g256(0)}
        errs = {}
        for name, f in cfgs.items():
            y = f().float()
            torch.cuda.synchronize()
            errs[name] = ((y - ref).abs().max() / ref.abs().max()).item()
            if not errs[name] < 2e-2:
                bad += 1
        fns = dict(cfgs)
        fns['hipblaslt'] = lambda: torch.mm(x, w.t())
        t = timeit(fns)
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
