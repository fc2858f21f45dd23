"""Numerics of the 256-row LDS-DMA GEMM engine (csrc/kernels/gemm256.hip) against fp32
PyTorch references: NT (bf16 / fp32 / bias+GELU epilogues), TN (MN-contiguous operands,
transposed LDS reads) and the implicit-GEMM conv forward with BatchNorm statistics."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


@pytest.mark.parametrize('bn', [128, 256])
@pytest.mark.parametrize('M,N,K', [(256, 256, 64), (1000, 296, 72), (4096, 768, 768), (300, 1032, 200)])
def test_gemm256_nt_tn(M, N, K, bn):
    from mlcomp_amd.ops import _lib
    P = _lib.ptr
    torch.manual_seed(0)
    a = torch.randn(M, K, device='cuda').to(torch.bfloat16)
    b = torch.randn(N, K, device='cuda').to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    _lib.call('mlc_gemm256_nt', P(a), P(b), P(out), None, M, N, K, K, K, N, None, 0, None, None, 0, bn,
              _lib.stream())
    bias = torch.randn(N, device='cuda')
    g = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
    _lib.call('mlc_gemm256_nt', P(a), P(b), P(g), None, M, N, K, K, K, N, P(bias), 1, None, None, 0, bn,
              _lib.stream())
    f = torch.empty(M, N, device='cuda')
    _lib.call('mlc_gemm256_nt', P(a), P(b), None, P(f), M, N, K, K, K, N, None, 0, None, None, 0, bn,
              _lib.stream())
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-2
    assert _rel(g, F.gelu(ref + bias)) < 1e-2
    assert _rel(f, ref) < 1e-5
    if M % 8 == 0 and N % 8 == 0:
        t = torch.empty(M, N, device='cuda')
        at, bt = a.t().contiguous(), b.t().contiguous()
        _lib.call('mlc_gemm256_tn', P(at), P(bt), P(t), M, N, K, M, N, N, 0, bn, _lib.stream())
        torch.cuda.synchronize()
        assert _rel(t, ref) < 1e-5


@pytest.mark.parametrize('bn', [128, 256])
@pytest.mark.parametrize('shape', [(4, 14, 64, 128, 3, 1, 1), (2, 15, 64, 64, 3, 2, 1), (2, 8, 16, 64, 4, 1, 0),
                                   (3, 9, 24, 40, 3, 1, 1), (2, 7, 256, 512, 1, 1, 0)])
def test_conv256_fwd_stats(shape, bn):
    from mlcomp_amd.ops import _lib
    P = _lib.ptr
    N, H, C, Co, k, s, p = shape
    torch.manual_seed(1)
    x = torch.randn(N, H, H, C, device='cuda').to(torch.bfloat16)
    w = (torch.randn(Co, k, k, C, device='cuda') * 0.1).to(torch.bfloat16)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1).contiguous()
    y = torch.empty_like(ref, dtype=torch.bfloat16)
    s1 = torch.zeros(32, Co, device='cuda')
    s2 = torch.zeros(32, Co, device='cuda')
    _lib.call('mlc_conv256_fwd', P(x), P(w), P(y), P(s1), P(s2), N, H, H, C, Co, k, k, s, p, 1, ref.shape[1],
              ref.shape[2], bn, _lib.stream())
    torch.cuda.synchronize()
    yf = y.float().reshape(-1, Co)
    assert _rel(y, ref) < 1e-2
    assert _rel(s1.sum(0), yf.sum(0)) < 1e-4
    assert _rel(s2.sum(0), (yf * yf).sum(0)) < 1e-4
