"""A/B of the conv input gradient: ConvDgradB (filter read as an MN-contiguous tile
through ds_read_b64_tr_b16) vs the transposed, flipped filter (mlc_conv_dgrad_t: the
forward-conv loaders at stride 1, ConvDgradBT in the parity-class GEMMs when strided), on
ResNet-50's conv shapes (batch 256), plus the cost of
the one batched transpose launch for the whole network.

    python scripts/bench_dgrad_wt.py [--batch 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mlcomp_amd.ops import functional as Fn  # noqa: E402
from bench_convs import SHAPES, timeit  # noqa: E402


class _Slot:
    def __init__(self, w):
        self.shape, self.numel, self._w = tuple(w.shape), w.numel(), w

    @property
    def bf16(self):
        return self._w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--iters', type=int, default=20)
    a = ap.parse_args()
    N = a.batch
    tab = Fn.WtTable()
    tot_old = tot_new = 0.0
    print(f'{"shape":24s} {"plain us":>9s} {"wt us":>9s} {"x":>6s}', flush=True)
    for name, H, C, Co, k, s, cnt in SHAPES:
        if C % 64:
            continue
        p = k // 2
        Ho = (H + 2 * p - k) // s + 1
        dy = torch.randn(N, Ho, Ho, Co, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, k, k, C, device='cuda') * (k * k * C) ** -0.5).to(torch.bfloat16)
        wt = Fn.wt_flip_transpose(w)
        for _ in range(cnt):
            tab.add(_Slot(w))
        dx = torch.empty(N, H, H, C, device='cuda', dtype=torch.bfloat16)
        ref = Fn.conv2d_dgrad(dy, w, dx.shape, s, p)
        got = Fn.conv2d_dgrad(dy, w, dx.shape, s, p, wt=wt)
        err = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
        assert err < 1e-2, (name, err)
        t0 = timeit(lambda: Fn.conv2d_dgrad(dy, w, dx.shape, s, p, out=dx), a.iters)
        t1 = timeit(lambda: Fn.conv2d_dgrad(dy, w, dx.shape, s, p, out=dx, wt=wt), a.iters)
        tot_old += cnt * t0
        tot_new += cnt * t1
        print(f'{name:24s} {t0 * 1e6:9.1f} {t1 * 1e6:9.1f} {t0 / t1:6.2f}', flush=True)
    tab.finalize('cuda')
    tt = timeit(tab.refresh, a.iters)
    print(f'weighted per step: plain {tot_old * 1e3:.3f} ms, transposed {tot_new * 1e3:.3f} ms '
          f'+ transpose launch {tt * 1e3:.3f} ms ({len(tab.slots)} filters)', flush=True)


if __name__ == '__main__':
    main()
