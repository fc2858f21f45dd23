"""ResNet-50 conv shapes whose GEMMs take the LDS-DMA main loop (forward convs and
transposed-filter dgrads), each run 3x after a warmup, for counter collection with
MLC_GEMM_DMA=0 / 1:  rocprofv3 --pmc ... --kernel-trace -- python scripts/prof_dma.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import functional as Fn  # noqa: E402

N = 256
for (H, C, Co, k, s) in [(28, 128, 128, 3, 1), (14, 256, 256, 3, 1), (28, 512, 256, 1, 1), (28, 256, 256, 3, 2)]:
    p = k // 2
    Ho = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
    w = (torch.randn(Co, k, k, C, device='cuda') * 0.05).to(torch.bfloat16)
    wt = Fn.wt_flip_transpose(w)
    dy = torch.randn(N, Ho, Ho, Co, device='cuda').to(torch.bfloat16)
    for _ in range(4):
        Fn.conv2d_fwd(x, w, s, p)
        Fn.conv2d_dgrad(dy, w, x.shape, s, p, wt=wt)
    torch.cuda.synchronize()
print('ok')
