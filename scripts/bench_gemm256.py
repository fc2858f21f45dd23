"""A/B of the 256-row LDS-DMA GEMM engine (csrc/kernels/gemm256.hip) against the 128x128
engine (csrc/kernels/igemm.hip) and torch (hipBLASLt / MIOpen) on random bf16 operands:
numerics vs fp32 references, then interleaved timing rounds in one process."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from mlcomp_amd.ops import _lib  # noqa: E402

P = _lib.ptr
S = _lib.stream


def nt(a, b, out, bias=None, act=0, bn=0):
    M, K = a.shape
    N = b.shape[0]
    bf = out.dtype == torch.bfloat16
    _lib.call('mlc_gemm256_nt', P(a), P(b), P(out) if bf else None, None if bf else P(out), M, N, K, K, K, N,
              P(bias), act, None, None, 0, bn, S())


def tn(a, b, out, bn=0):   # out[M][N] = a[K][M]^T b[K][N]
    K, M = a.shape
    N = b.shape[1]
    _lib.call('mlc_gemm256_tn', P(a), P(b), P(out), M, N, K, M, N, N, 0, bn, S())


def old_nt(a, b, out):
    M, K = a.shape
    N = b.shape[0]
    _lib.call('mlc_gemm_bf16out', P(a), P(b), P(out), M, N, K, K, K, N, 0, 1, S())


def old_tn(a, b, out):
    K, M = a.shape
    N = b.shape[1]
    _lib.call('mlc_gemm_f32out', P(a), P(b), P(out), None, M, N, K, M, N, N, 1, 0, 0, 0, 1, S())


def conv256(x, w, y, stride, pad, stats=None, bn=0):
    N, H, W, C = x.shape
    Co, KH, KW, _ = w.shape
    Ho, Wo = y.shape[1], y.shape[2]
    s1, s2 = stats if stats is not None else (None, None)
    _lib.call('mlc_conv256_fwd', P(x), P(w), P(y), P(s1), P(s2), N, H, W, C, Co, KH, KW, stride, pad, 1, Ho, Wo,
              bn, S())


def conv_old(x, w, y, stride, pad, stats=None):
    N, H, W, C = x.shape
    Co, KH, KW, _ = w.shape
    Ho, Wo = y.shape[1], y.shape[2]
    s1, s2 = stats if stats is not None else (None, None)
    _lib.call('mlc_conv_fwd', P(x), P(w), P(y), P(s1), P(s2), N, H, W, C, Co, KH, KW, stride, pad, 1, Ho, Wo, None, None, S())


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


def check():
    torch.manual_seed(0)
    worst = 0.0
    for (M, N, K) in [(256, 256, 64), (1000, 300, 72), (4096, 768, 768), (300, 1028, 200), (2048, 2304, 768)]:
        a = torch.randn(M, K, device='cuda').to(torch.bfloat16)
        b = torch.randn(N, K, device='cuda').to(torch.bfloat16)
        ref = a.float() @ b.float().t()
        for bn in (128, 256):
            out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
            nt(a, b, out, bn=bn)
            outf = torch.empty(M, N, device='cuda', dtype=torch.float32)
            nt(a, b, outf, bn=bn)
            bias = torch.randn(N, device='cuda')
            outg = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
            nt(a, b, outg, bias=bias, act=1, bn=bn)
            refg = F.gelu(ref + bias)
            es = (rel(out, ref), rel(outf, ref), rel(outg, refg))
            if M % 8 == 0 and N % 8 == 0:
                at, bt = a.t().contiguous(), b.t().contiguous()   # [K][M], [K][N]
                o2 = torch.empty(M, N, device='cuda')
                tn(at, bt, o2, bn=bn)
                es += (rel(o2, ref),)
            torch.cuda.synchronize()
            print(f'check nt/tn {M}x{N}x{K} bn{bn}: ' + ' '.join(f'{e:.2e}' for e in es), flush=True)
            worst = max([worst, es[0], es[1] * 50, es[2]] + ([es[3] * 50] if len(es) > 3 else []))
    for (N_, H, C, Co, k, s, p) in [(4, 14, 64, 128, 3, 1, 1), (2, 15, 64, 64, 3, 2, 1), (2, 8, 16, 64, 4, 1, 0),
                                     (3, 9, 24, 40, 3, 1, 1), (2, 7, 256, 512, 1, 1, 0)]:
        x = torch.randn(N_, H, H, C, device='cuda').to(torch.bfloat16)
        w = (torch.randn(Co, k, k, C, device='cuda') * 0.1).to(torch.bfloat16)
        ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), stride=s, padding=p)
        ref = ref.permute(0, 2, 3, 1).contiguous()
        for bn in (128, 256):
            y = torch.empty_like(ref, dtype=torch.bfloat16)
            s1 = torch.zeros(32, Co, device='cuda')
            s2 = torch.zeros(32, Co, device='cuda')
            conv256(x, w, y, s, p, stats=(s1, s2), bn=bn)
            torch.cuda.synchronize()
            yf = y.float().reshape(-1, Co)
            e1 = rel(y, ref)
            e2 = rel(s1.sum(0), yf.sum(0))
            e3 = rel(s2.sum(0), (yf * yf).sum(0))
            print(f'check conv {N_}x{H}x{H}x{C}->{Co} k{k}s{s}p{p} bn{bn}: y {e1:.2e} sum {e2:.2e} sumsq {e3:.2e}',
                  flush=True)
            worst = max(worst, e1, e2 * 10, e3 * 10)
    assert worst < 2e-2, worst


def timeit(fns, rounds=5, iters=20):
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            torch.cuda.synchronize()
            times[k].append(s.elapsed_time(e) / iters)
    return {k: sorted(v)[len(v) // 2] for k, v in times.items()}


def bench():
    import os
    conv_only = os.environ.get('CONV_ONLY') == '1'     # only the ResNet conv shapes
    nb = int(os.environ.get('CONV_BATCH', 256))        # their batch
    for (M, N, K) in [] if conv_only else [(4096, 4096, 4096), (4096, 2304, 768), (4096, 3072, 768), (4096, 768, 3072),
                      (50176, 1024, 256), (12544, 2048, 512)]:
        a = torch.rand(M, K, device='cuda').sub(0.5).to(torch.bfloat16)
        b = torch.rand(N, K, device='cuda').sub(0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        t = timeit({'g256': lambda: nt(a, b, out, bn=256), 'g128': lambda: nt(a, b, out, bn=128),
                    'igemm': lambda: old_nt(a, b, out), 'torch': lambda: torch.matmul(a, b.t(), out=out)})
        fl = 2.0 * M * N * K
        print(json.dumps({'nt': [M, N, K], **{k: round(fl / v / 1e9, 1) for k, v in t.items()}}), flush=True)
    for (M, N, K) in [] if conv_only else [(512, 4608, 12544), (256, 2304, 50176), (768, 3072, 4096), (3072, 768, 4096)]:
        a = torch.rand(K, M, device='cuda').sub(0.5).to(torch.bfloat16)
        b = torch.rand(K, N, device='cuda').sub(0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device='cuda')
        t = timeit({'g256': lambda: tn(a, b, out, bn=256), 'g128': lambda: tn(a, b, out, bn=128),
                    'igemm_atomic': lambda: (out.zero_(), old_tn(a, b, out))})
        fl = 2.0 * M * N * K
        print(json.dumps({'tn': [M, N, K], **{k: round(fl / v / 1e9, 1) for k, v in t.items()}}), flush=True)
    # ResNet-50 (batch CONV_BATCH) 3x3 convs + stem (s2d 4x4 over 16 channels)
    for (Nb, H, C, Co, k, s, p) in [(nb, 56, 64, 64, 3, 1, 1), (nb, 56, 128, 128, 3, 2, 1),
                                    (nb, 28, 128, 128, 3, 1, 1), (nb, 28, 256, 256, 3, 2, 1),
                                    (nb, 14, 256, 256, 3, 1, 1), (nb, 14, 512, 512, 3, 2, 1),
                                    (nb, 7, 512, 512, 3, 1, 1), (nb, 112, 16, 64, 4, 1, 0)]:
        x = torch.rand(Nb, H + (1 if k == 4 else 0), H + (1 if k == 4 else 0), C, device='cuda').sub(0.5).to(torch.bfloat16)
        w = torch.rand(Co, k, k, C, device='cuda').sub(0.5).to(torch.bfloat16)
        Ho = (x.shape[1] + 2 * p - k) // s + 1
        y = torch.empty(Nb, Ho, Ho, Co, device='cuda', dtype=torch.bfloat16)
        s1 = torch.zeros(32, Co, device='cuda')
        s2 = torch.zeros(32, Co, device='cuda')
        t = timeit({'c256': lambda: conv256(x, w, y, s, p, (s1, s2), bn=256),
                    'c128': lambda: conv256(x, w, y, s, p, (s1, s2), bn=128),
                    'igemm': lambda: conv_old(x, w, y, s, p, (s1, s2))})
        fl = 2.0 * Nb * Ho * Ho * Co * k * k * C
        print(json.dumps({'conv': [Nb, H, C, Co, k, s], **{kk: round(fl / v / 1e9, 1) for kk, v in t.items()},
                          'ms_igemm': round(t['igemm'], 4), 'ms_best_new': round(min(t['c256'], t['c128']), 4)}),
              flush=True)


if __name__ == '__main__':
    import os
    if os.environ.get('CONV_ONLY') != '1':
        check()
    bench()
