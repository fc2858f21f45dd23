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


@pytest.mark.gpu
@pytest.mark.parametrize('C', [16, 40, 320])
def test_bn_row_scale_matches_cpu_reference(C):
    """BatchNorm apply / backward with a per-sample factor (the folded drop-path mask / keep)
    and a residual: GPU kernels vs the fp32 CPU reference of the same functions."""
    torch.manual_seed(1)
    N, H = 6, 9
    y = torch.randn(N, H, H, C).to(torch.bfloat16)
    res = torch.randn(N, H, H, C).to(torch.bfloat16)
    dz = torch.randn(N, H, H, C).to(torch.bfloat16)
    scale, shift = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    mean, inv, gamma = torch.randn(C) * 0.1, torch.rand(C) + 0.5, torch.rand(C) + 0.5
    rsc = (torch.rand(N) < 0.7).float() / 0.7
    outs = {}
    for dev in ('cpu', 'cuda'):
        t = [v.to(dev) for v in (y, res, dz, scale, shift, mean, inv, gamma, rsc)]
        yy, rr, dd, sc, sh, mu, iv, ga, rs = t
        z = Fn.bnact_apply(yy, rr, sc, sh, 0, 0.0, row_scale=rs)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dy, dres = Fn.bnact_bwd(dd, z, yy, rr, mu, sc, sh, iv, ga, 0, 0.0, dgamma=dg, dbeta=db,
                                sums=torch.zeros(Fn.NSTAT * 2 * C, device=dev), want_dres=True, row_scale=rs)
        outs[dev] = [v.float().cpu() for v in (z, dy, dres, dg, db)]
    for a, b in zip(outs['cpu'], outs['cuda']):
        assert (a - b).abs().max() <= 2e-2 * a.abs().max() + 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize('N,H,W,C,k,s,p,cip', [(2, 17, 17, 192, 3, 1, 1, True), (3, 14, 15, 40, 2, 2, 0, True),
                                               (2, 13, 11, 64, 3, 2, 1, False), (1, 9, 9, 2048, 3, 1, 1, True)])
def test_avgpool2d_kernels_match_cpu_reference(N, H, W, C, k, s, p, cip):
    """Windowed average pool (pool_loss.hip) forward / backward vs the fp32 CPU path."""
    torch.manual_seed(2)
    x = torch.randn(N, H, W, C).to(torch.bfloat16)
    y_ref = Fn.avgpool2d_fwd(x, k, s, p, cip)
    dy = torch.randn_like(y_ref.float()).to(torch.bfloat16)
    dx_ref = Fn.avgpool2d_bwd(dy, x.shape, k, s, p, cip)
    y = Fn.avgpool2d_fwd(x.cuda(), k, s, p, cip)
    dx = Fn.avgpool2d_bwd(dy.cuda(), x.shape, k, s, p, cip)
    torch.cuda.synchronize()
    assert (y.float().cpu() - y_ref.float()).abs().max() <= 1e-2 * y_ref.float().abs().max()
    assert (dx.float().cpu() - dx_ref.float()).abs().max() <= 1e-2 * dx_ref.float().abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize('k,pad', [((1, 7), (0, 3)), ((7, 1), (3, 0)), ((1, 3), (0, 1)), ((3, 1), (1, 0))])
def test_dgrad_with_transposed_filter_per_axis_pad(k, pad):
    """Input gradient of Inception's 1xn / nx1 convs through the transposed-filter GEMM
    (mlc_conv_dgrad_t, per-axis padding) vs the fp32 CPU reference."""
    torch.manual_seed(3)
    N, H, W, C, Co = 2, 17, 17, 64, 96
    w = (torch.randn(Co, k[0], k[1], C) * 0.1).to(torch.bfloat16)
    dy = torch.randn(N, H, W, Co).to(torch.bfloat16)
    want = Fn.conv2d_dgrad(dy, w, (N, H, W, C), 1, pad, 1)
    wt = Fn.wt_flip_transpose(w.cuda())
    got = Fn.conv2d_dgrad(dy.cuda(), w.cuda(), (N, H, W, C), 1, pad, 1, wt=wt)
    torch.cuda.synchronize()
    assert (got.float().cpu() - want.float()).abs().max() <= 1e-2 * want.float().abs().max()
