"""Channel-gate (squeeze-excitation) kernels (``normact.hip`` chscale) against fp32 PyTorch:
act(y * g [+ res]) forward, and the one-pass backward (ReLU mask, residual gradient,
dy = d * g, dg = sum over pixels of d * y)."""
import pytest
import torch

from mlcomp_amd.ops import functional as Fn


@pytest.mark.gpu
@pytest.mark.parametrize('N,H,C,res,relu', [(4, 56, 96, False, False), (3, 7, 1152, False, False),
                                            (2, 14, 40, True, True), (5, 28, 2056, True, False),
                                            (2, 9, 512, False, True)])
def test_chscale_matches_fp32(N, H, C, res, relu):
    torch.manual_seed(0)
    dev = 'cuda'
    y = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    g = torch.rand(N, C, device=dev).to(torch.bfloat16)
    r = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16) if res else None
    dout = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    z = Fn.chscale_fwd(y, g, r, relu)
    a = y.float() * g.float().view(N, 1, 1, C) + (r.float() if res else 0)
    want = a.clamp_min(0) if relu else a
    assert (z.float() - want).abs().max() <= 2e-2 * want.abs().max()
    dy, dg, dres = Fn.chscale_bwd(dout, y, g, z if relu else None, want_dres=res)
    d = dout.float() * (want > 0) if relu else dout.float()
    ref_dy = d * g.float().view(N, 1, 1, C)
    ref_dg = (d * y.float()).sum((1, 2))
    torch.cuda.synchronize()
    assert (dy.float() - ref_dy).abs().max() <= 2e-2 * ref_dy.abs().max()
    assert (dg - ref_dg).abs().max() <= 1e-3 * ref_dg.abs().max() + 1e-3
    if res:
        assert (dres.float() - d).abs().max() <= 1e-2 * d.abs().max()
