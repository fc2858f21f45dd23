"""Attention kernel timings on one GPU: whole-tile kernels (transformer.hip, S <= 128),
streaming flash kernels (flash_attn.hip) and torch's scaled_dot_product_attention on the
same shapes.  TFLOP/s counts 4*B*H*S^2*D for the forward and 2.5x that for the backward
(the backward's recompute of Q K^T not counted)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mlcomp_amd.ops import transformer as Tx  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = 'cuda'
    rows = []
    shapes = [(32, 12, 128, 64), (16, 12, 256, 64), (8, 12, 512, 64), (8, 16, 512, 128), (4, 16, 1024, 128),
              (2, 12, 2048, 64)]
    for B, H, S, D in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        qkv = (torch.randn(B * S, 3 * H * D, device=dev, generator=g) * 0.5).to(torch.bfloat16)
        dctx = torch.randn(B * S, H * D, device=dev, generator=g).to(torch.bfloat16)
        kb = torch.zeros(B, S, device=dev)
        kb[0, S // 2:] = float('-inf')
        scale = 1 / math.sqrt(D)
        fl = 4.0 * B * H * S * S * D
        r = dict(B=B, H=H, S=S, D=D)
        for name, flash in (('tile', False), ('flash', True)):
            if not flash and not (D == 64 and S in (64, 128)):
                continue
            Tx._FLASH_ONLY = flash
            ctx, lse = Tx.attn_fwd(qkv, kb, B, S, H, scale, head_dim=D)
            tf = timeit(lambda: Tx.attn_fwd(qkv, kb, B, S, H, scale, head_dim=D))
            tb = timeit(lambda: Tx.attn_bwd(qkv, kb, dctx, lse, B, S, H, scale, head_dim=D, ctx=ctx))
            r[name] = dict(fwd_ms=round(tf, 4), bwd_ms=round(tb, 4), fwd_tflops=round(fl / tf / 1e9, 1),
                           bwd_tflops=round(2.5 * fl / tb / 1e9, 1))
        Tx._FLASH_ONLY = False
        q, k, v = qkv.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4).contiguous().unbind(0)
        q, k, v = (t.detach().requires_grad_(True) for t in (q, k, v))
        mask = kb[:, None, None, :].to(torch.bfloat16)
        do = dctx.view(B, S, H, D).transpose(1, 2).contiguous()
        F = torch.nn.functional.scaled_dot_product_attention
        tf = timeit(lambda: F(q, k, v, attn_mask=mask))
        o = F(q, k, v, attn_mask=mask)
        tb = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
        r['torch_sdpa'] = dict(fwd_ms=round(tf, 4), bwd_ms=round(tb, 4), fwd_tflops=round(fl / tf / 1e9, 1),
                               bwd_tflops=round(2.5 * fl / tb / 1e9, 1))
        rows.append(r)
        print(json.dumps(r), flush=True)
    return rows


if __name__ == '__main__':
    sys.exit(0 if main() else 1)
