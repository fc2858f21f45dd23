"""A few ResNet-50 conv shapes, each op run 3x after a warmup, for counter collection:
rocprofv3 --pmc ... --kernel-trace -- python scripts/prof_convs.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import functional as Fn  # noqa: E402

N = 256
for (H, C, Co, k, s) in [(28, 128, 128, 3, 1), (56, 128, 128, 3, 2), (56, 64, 256, 1, 1)]:
    p = k // 2
    Ho = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
    w = (torch.randn(Co, k, k, C, device='cuda') * 0.05).to(torch.bfloat16)
    dy = torch.randn(N, Ho, Ho, Co, device='cuda').to(torch.bfloat16)
    dw = torch.empty(Co, k, k, C, device='cuda')
    for _ in range(3):
        Fn.conv2d_fwd(x, w, s, p)
        Fn.conv2d_dgrad(dy, w, x.shape, s, p)
        Fn.conv2d_wgrad(dy, x, w.shape, s, p, out=dw)
    torch.cuda.synchronize()
print('ok')
