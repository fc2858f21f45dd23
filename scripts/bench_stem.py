"""The ResNet-50 stem conv at batch 512 (the 4x4/1 conv over the space-to-depth image, with
the fused BN statistics): the persistent register-resident-filter kernel
(csrc/kernels/stemconv.hip) vs the implicit-GEMM engine (igemm.hip), timed in HIP graphs.

    python scripts/bench_stem.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import functional as Fn  # noqa: E402
from bench_gconv import timeit  # noqa: E402


def main():
    N = int(os.environ.get('BATCH', 512))
    xs = torch.randn(N, 115, 115, 16, device='cuda').to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 16, device='cuda') * 0.1).to(torch.bfloat16)
    st = torch.zeros(2, Fn.NSTAT * 64, device='cuda')
    dy = torch.randn(N, 112, 112, 64, device='cuda').to(torch.bfloat16)
    dw = torch.zeros(64, 4, 4, 16, device='cuda')
    t = timeit({'stemconv': lambda: Fn.stem_conv_fwd(xs, w, stats=(st[0], st[1])),
                'igemm': lambda: Fn.conv2d_fwd(xs, w, 1, 0, 1, stats=(st[0], st[1])),
                'igemm_wgrad': lambda: Fn.conv2d_wgrad(dy, xs, w.shape, 1, 0, 1, out=dw, accumulate=True)})
    byts = xs.numel() * 2 + N * 112 * 112 * 64 * 2
    flops = 2 * N * 112 * 112 * 64 * 256
    print(json.dumps({'batch': N, 'impl': os.environ.get('MLC_STEM_IMPL', '1'),
                      'us': {k: round(v * 1e3, 1) for k, v in t.items()},
                      'GBps': {k: round(byts / v / 1e6) for k, v in t.items()},
                      'TFps': {k: round(flops / v / 1e9) for k, v in t.items()}}), flush=True)


if __name__ == '__main__':
    main()
