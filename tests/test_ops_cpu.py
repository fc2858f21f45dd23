"""CPU checks of the native op reference paths against autograd of plain PyTorch
modules (the GPU kernels are in turn checked against these references)."""
import pytest
import torch
import torch.nn.functional as F

from mlcomp_amd.ops import functional as Fn


def test_bn_reference_matches_autograd():
    torch.manual_seed(0)
    C = 16
    y = (torch.randn(4, 5, 5, C) * 2).to(torch.bfloat16)
    res = torch.randn(4, 5, 5, C).to(torch.bfloat16)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    yf = y.float().reshape(-1, C)
    s1, s2 = Fn.stat_buffers(C, 'cpu')
    s1[:C], s2[:C] = yf.sum(0), (yf * yf).sum(0)
    sm, si = torch.empty(C), torch.empty(C)
    z = Fn.bn_fwd_apply(y, res, s1, s2, gamma, beta, sm, si, None, None, relu=True)
    # autograd reference in NCHW
    yt = y.float().permute(0, 3, 1, 2).requires_grad_()
    g_t, b_t = gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    rt = res.float().permute(0, 3, 1, 2).requires_grad_()
    zt = F.relu(F.batch_norm(yt, None, None, g_t, b_t, training=True) + rt)
    assert (z.float() - zt.permute(0, 2, 3, 1)).abs().max() < 0.05
    dz = torch.randn_like(z)
    zt.backward(dz.float().permute(0, 3, 1, 2))
    dg, db = torch.empty(C), torch.empty(C)
    dy, dres = Fn.bn_bwd(dz, z, y, sm, si, gamma, want_dres=True, dgamma=dg, dbeta=db)
    assert (dy.float() - yt.grad.permute(0, 2, 3, 1)).abs().max() < 0.05
    assert (dres.float() - rt.grad.permute(0, 2, 3, 1)).abs().max() < 0.05
    assert torch.allclose(dg, g_t.grad, atol=0.1, rtol=0.02)
    assert torch.allclose(db, b_t.grad, atol=0.1, rtol=0.02)


def test_conv_reference_shapes():
    x = torch.randn(2, 9, 9, 8).to(torch.bfloat16)
    w = torch.randn(16, 3, 3, 8).to(torch.bfloat16)
    y = Fn.conv2d_fwd(x, w, 2, 1)
    assert y.shape == (2, 5, 5, 16)
    dx = Fn.conv2d_dgrad(torch.randn_like(y.float()).to(torch.bfloat16), w, x.shape, 2, 1)
    assert dx.shape == x.shape
    dw = Fn.conv2d_wgrad(y, x, w.shape, 2, 1)
    assert dw.shape == w.shape and dw.dtype == torch.float32


def test_maxpool_reference_matches_autograd():
    x = torch.randn(2, 12, 12, 8).to(torch.bfloat16)
    y, i = Fn.maxpool_fwd(x)
    dy = torch.randn_like(y.float()).to(torch.bfloat16)
    dx = Fn.maxpool_bwd(dy, i, x.shape)
    xr = x.permute(0, 3, 1, 2).float().requires_grad_()
    F.max_pool2d(xr, 3, 2, 1).backward(dy.permute(0, 3, 1, 2).float())
    assert (dx.permute(0, 3, 1, 2).float() - xr.grad).abs().max() < 0.05


def test_stem_pool_reference_matches_autograd():
    """The fused stem tail's reference path (BN-apply + ReLU + maxpool, and its backward
    through a training BatchNorm) against torch autograd of the unfused graph."""
    import torch.nn.functional as F
    from mlcomp_amd.ops import functional as Fn
    torch.manual_seed(3)
    N, H, W, C = 2, 12, 10, 16
    y = torch.randn(N, H, W, C).to(torch.bfloat16)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C) * 0.2
    yf = y.float().requires_grad_(True)
    g_ = gamma.clone().requires_grad_(True)
    b_ = beta.clone().requires_grad_(True)
    bn = F.batch_norm(yf.permute(0, 3, 1, 2), None, None, g_, b_, training=True, eps=1e-5)
    ref = F.max_pool2d(F.relu(bn), 3, 2, 1)
    dp = torch.randn_like(ref)
    ref.backward(dp)
    mean = y.float().mean((0, 1, 2))
    var = y.float().var((0, 1, 2), unbiased=False)
    invstd = torch.rsqrt(var + 1e-5)
    scale, shift = gamma * invstd, beta - mean * gamma * invstd
    out, idx = Fn.stem_pool_fwd(y, scale, shift)
    assert torch.allclose(out.float(), ref.detach().permute(0, 2, 3, 1), atol=2e-2, rtol=2e-2)
    dg, db = torch.empty(C), torch.empty(C)
    dy = Fn.stem_pool_bwd(dp.permute(0, 2, 3, 1).to(torch.bfloat16), idx, y, mean, invstd, gamma, dg, db,
                          None, None)
    assert torch.allclose(dy.float(), yf.grad, atol=3e-2, rtol=3e-2)
    assert torch.allclose(dg, g_.grad, atol=3e-2, rtol=3e-2)
    assert torch.allclose(db, b_.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize('K,s,p,d', [(1, 1, 0, 1), (3, 1, 1, 1), (3, 1, 2, 2), (3, 1, 0, 1), (5, 1, 2, 1),
                                     (3, 2, 1, 1), (1, 2, 0, 1), (3, 3, 1, 1)])
def test_dgrad_transposed_filter_reference(K, s, p, d):
    """The transposed-filter dgrad (stride 1: a forward conv of dy over the flipped,
    channel-swapped filter with pad d*(K-1)-p) equals the plain input gradient."""
    torch.manual_seed(0)
    N, H, W, C, Co = 2, 9, 8, 16, 24
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, d)
    dy = torch.randn(N, Ho, Wo, Co).to(torch.bfloat16)
    w = torch.randn(Co, K, K, C).to(torch.bfloat16)
    assert Fn.dgrad_as_fwd_conv(K, K, s, p, d) == (s == 1)
    a = Fn.conv2d_dgrad(dy, w, (N, H, W, C), s, p, d)
    b = Fn.conv2d_dgrad(dy, w, (N, H, W, C), s, p, d, wt=Fn.wt_flip_transpose(w))
    assert (a.float() - b.float()).abs().max().item() <= 1e-2 * a.float().abs().max().item()
    assert torch.equal(Fn.wt_flip_transpose(Fn.wt_flip_transpose(w)), w)


class _Slot:
    def __init__(self, w):
        self.shape, self.numel, self.bf16 = tuple(w.shape), w.numel(), w


def test_wt_table_cpu_conv_and_dense():
    """WtTable on CPU: conv filters get the flipped channel-swapped copy, [out, in] dense
    weights the plain transpose; both refresh in place from the current weights."""
    torch.manual_seed(1)
    wc = torch.randn(24, 3, 3, 16).to(torch.bfloat16)
    wd = torch.randn(40, 32).to(torch.bfloat16)
    tab = Fn.WtTable()
    ic, idd = tab.add(_Slot(wc)), tab.add(_Slot(wd))
    tab.finalize('cpu')
    assert tuple(tab[ic].shape) == (16, 3, 3, 24) and tuple(tab[idd].shape) == (32, 40)
    tab.refresh()
    assert torch.equal(tab[ic], Fn.wt_flip_transpose(wc)) and torch.equal(tab[idd], wd.t())
    wd.mul_(2)                        # a weight update: the next refresh follows it
    tab.refresh()
    assert torch.equal(tab[idd], wd.t())
