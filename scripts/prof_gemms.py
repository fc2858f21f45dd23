"""BERT dense-layer GEMM shapes + one large square, each run 3x after a warmup, for
counter collection: rocprofv3 --pmc ... --kernel-trace -- python scripts/prof_gemms.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mlcomp_amd.ops import transformer as Tx  # noqa: E402

for (M, N, K, act) in [(4096, 2304, 768, 0), (4096, 3072, 768, 1), (8192, 8192, 8192, 0)]:
    x = torch.randn(M, K, device='cuda').to(torch.bfloat16)
    w = (torch.randn(N, K, device='cuda') * K ** -0.5).to(torch.bfloat16)
    b = torch.zeros(N, device='cuda')
    for _ in range(4):
        Tx.dense_fwd(x, w, b, act=act, want_preact=bool(act))
    torch.cuda.synchronize()
print('ok')
