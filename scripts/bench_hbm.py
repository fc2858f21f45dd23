"""HBM write / copy / read bandwidth of one MI355X for the ResNet-50 stem's tensor size
(822 MB bf16 = [512, 112, 112, 64]), timed in HIP graphs: the bound of a kernel that
writes that tensor.

    python scripts/bench_hbm.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_gconv import timeit  # noqa: E402


def main():
    n = 512 * 112 * 112 * 64
    a = torch.empty(n, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(n, device='cuda').to(torch.bfloat16)
    s = torch.empty((), device='cuda')
    t = timeit({'fill': lambda: a.fill_(1.0), 'copy': lambda: a.copy_(b),
                'read': lambda: torch.sum(b.view(64, -1), dim=(0, 1), dtype=torch.float32, out=s)}, rounds=5, iters=5)
    byts = {'fill': n * 2, 'copy': n * 4, 'read': n * 2}
    print(json.dumps({k: {'us': round(v * 1e3, 1), 'GBps': round(byts[k] / v / 1e6)} for k, v in t.items()}),
          flush=True)


if __name__ == '__main__':
    main()
