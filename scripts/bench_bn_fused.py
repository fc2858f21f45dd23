"""BatchNorm forward / backward launches in isolation: finalize + apply as two launches
(MLC_BN_FUSED=0 form) vs folded into one (batchnorm.hip bn_{fwd,bwd}_fused_kernel), on the
ResNet-50 @512 shapes.  Prints one JSON line per shape.

    python scripts/bench_bn_fused.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from mlcomp_amd.ops import functional as Fn  # noqa: E402

SHAPES = [('l1 64', 512 * 56 * 56, 64, False), ('l1 256+res', 512 * 56 * 56, 256, True),
          ('l2 128', 512 * 28 * 28, 128, False), ('l2 512+res', 512 * 28 * 28, 512, True),
          ('l3 256', 512 * 14 * 14, 256, False), ('l3 1024+res', 512 * 14 * 14, 1024, True),
          ('l4 2048+res', 512 * 7 * 7, 2048, True)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = 'cuda'
    for name, rows, C, res in SHAPES:
        y = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        r = torch.randn(rows, C, device=dev).to(torch.bfloat16) if res else None
        g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        s1, s2 = Fn.stat_buffers(C, dev)
        s1.uniform_(0, 1)
        s2.uniform_(1, 2)
        sm, si, rm, rv = (torch.zeros(C, device=dev) for _ in range(4))
        sc, sh = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        z = torch.empty_like(y)
        dz = torch.randn(rows, C, device=dev).to(torch.bfloat16)
        sums = torch.rand(Fn.NSTAT * 2 * C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        out = {'shape': name, 'rows': rows, 'C': C,
               'MB_fwd': round((y.numel() * 2 * (3 if res else 2)) / 1e6, 1)}
        for fused in (True, False):
            Fn.BN_FUSED = fused
            tf = timeit(lambda: Fn.bn_fwd_apply(y, r, s1, s2, g, b, sm, si, rm, rv, relu=True, out=z, scale=sc,
                                                shift=sh))
            tb = timeit(lambda: Fn.bn_bwd(dz, z, y, sm, si, g, want_dres=res, dgamma=dg, dbeta=db, sums=sums,
                                          prereduced=True))
            k = 'fused' if fused else 'two'
            out[f'fwd_us_{k}'] = round(tf, 1)
            out[f'bwd_us_{k}'] = round(tb, 1)
        print(json.dumps(out), flush=True)
        del y, r, z, dz


if __name__ == '__main__':
    main()
