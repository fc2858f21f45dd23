"""Dense GEMMs for a PMC pass (rocprofv3 --pmc ... -- python3 scripts/prof_dense.py):
BERT-base qkv / out forward on the 128x128, 128x192 and 128x96 tiles, and hipBLASLt."""
import sys

import torch

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402
from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def main():
    lib = _lib.load()
    M = 4096
    for N, K, tiles in [(2304, 768, (0, 6, 5)), (768, 768, (0, 5))]:
        x = torch.rand(M, K, device='cuda').sub(0.5).to(torch.bfloat16)
        w = torch.rand(N, K, device='cuda').sub(0.5).to(torch.bfloat16)
        b = torch.zeros(N, device='cuda')
        for t in tiles:
            lib.mlc_gemm_get_set(10, t)
            for _ in range(3):
                Tx.dense_fwd(x, w, b)
        for _ in range(3):
            torch.mm(x, w.t())
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
