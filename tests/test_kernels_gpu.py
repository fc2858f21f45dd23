"""Numerics of the HIP kernels vs the fp32 PyTorch reference of the same op.

Each test builds bf16 inputs once, runs the op on the GPU (HIP kernel from
libmlcomp_kernels.so) and on the CPU (the reference path of mlcomp_amd.ops.functional,
which is plain fp32 PyTorch math), and compares.
"""
import pytest
import torch
import torch.nn.functional as F

from mlcomp_amd.ops import functional as Fn

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.fixture(params=[0, 1], ids=['tiles-std', 'tiles-wide'], autouse=True)
def gemm_tiles(request):
    """Run every GEMM-backed test with the standard 64x64-per-wave tiles and again with the
    wide-wave 256x128 / 128x256 tiles forced on (min blocks 1)."""
    from mlcomp_amd.ops import _lib
    if not torch.cuda.is_available():
        yield
        return
    lib = _lib.load()
    old_big = lib.mlc_gemm_get_set(3, request.param)
    old_min = lib.mlc_gemm_get_set(4, 1 if request.param else 240)
    yield
    lib.mlc_gemm_get_set(3, old_big)
    lib.mlc_gemm_get_set(4, old_min)


def rel_err(a, b):
    a = a.float().cpu()
    b = b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _bf(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(torch.bfloat16)


CONV_CASES = [
    # N, H, W, C, Co, K, stride, pad
    (2, 14, 14, 64, 64, 1, 1, 0),
    (2, 14, 14, 64, 128, 3, 1, 1),
    (2, 15, 13, 32, 64, 3, 2, 1),
    (2, 16, 16, 64, 256, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),
    (3, 9, 7, 136, 40, 3, 1, 1),
    (1, 7, 7, 512, 2048, 1, 1, 0),
    (2, 16, 16, 64, 128, 3, 2, 1),
    (2, 15, 13, 128, 64, 3, 2, 1),
    (3, 15, 15, 64, 128, 1, 2, 0),
    (2, 13, 11, 64, 72, 3, 3, 1),     # stride 3: nine parity classes, Co % 64 != 0
]


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv_fwd_stats(case):
    N, H, W, C, Co, K, s, p = case
    x = _bf(N, H, W, C, seed=1)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=2)
    s1c, s2c = Fn.stat_buffers(Co, 'cpu')
    ref = Fn.conv2d_fwd(x, w, s, p, stats=(s1c, s2c))
    s1g, s2g = Fn.stat_buffers(Co, DEV)
    out = Fn.conv2d_fwd(x.to(DEV), w.to(DEV), s, p, stats=(s1g, s2g))
    torch.cuda.synchronize()
    assert out.shape == ref.shape
    assert rel_err(out, ref) < 1e-2
    red = lambda t: t.reshape(Fn.NSTAT, Co).sum(0)
    assert rel_err(red(s1g), red(s1c)) < 1e-2
    assert rel_err(red(s2g), red(s2c)) < 1e-2


def test_stat_copies_constant():
    from mlcomp_amd.ops import _lib
    assert _lib.load().mlc_bn_stat_copies() == Fn.NSTAT


@pytest.mark.parametrize('case', [c for c in CONV_CASES if c[3] != 8])
def test_conv_dgrad(case):
    N, H, W, C, Co, K, s, p = case
    x_shape = (N, H, W, C)
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    dy = _bf(N, Ho, Wo, Co, seed=3)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=4)
    ref = Fn.conv2d_dgrad(dy, w, x_shape, s, p)
    out = Fn.conv2d_dgrad(dy.to(DEV), w.to(DEV), x_shape, s, p)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv_wgrad(case):
    N, H, W, C, Co, K, s, p = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    x = _bf(N, H, W, C, seed=5)
    dy = _bf(N, Ho, Wo, Co, seed=6)
    ref = Fn.conv2d_wgrad(dy, x, (Co, K, K, C), s, p)
    out = Fn.conv2d_wgrad(dy.to(DEV), x.to(DEV), (Co, K, K, C), s, p)
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 5e-3


@pytest.mark.parametrize('case', [CONV_CASES[0], CONV_CASES[-1]])
def test_conv_wgrad_accumulate_slab_and_atomic(case):
    """split-K slab reduction (default) and the atomic fallback (no workspace) both
    accumulate into an existing gradient"""
    from mlcomp_amd.ops import _lib
    N, H, W, C, Co, K, s, p = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    x = _bf(N, H, W, C, seed=15)
    dy = _bf(N, Ho, Wo, Co, seed=16)
    ref = Fn.conv2d_wgrad(dy, x, (Co, K, K, C), s, p) + 1.0
    out = torch.ones(Co, K, K, C, device=DEV)
    Fn.conv2d_wgrad(dy.to(DEV), x.to(DEV), (Co, K, K, C), s, p, out=out, accumulate=True)
    out2 = torch.ones(Co, K, K, C, device=DEV)
    xd, dyd = x.to(DEV), dy.to(DEV)
    _lib.call('mlc_conv_wgrad', _lib.ptr(dyd), _lib.ptr(xd), _lib.ptr(out2), N, H, W, C, Co, K, K, s, p, 1,
              Ho, Wo, 0, 1, None, 0, None, None, _lib.stream())
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 5e-3
    assert rel_err(out2, ref) < 5e-3


AFF_CASES = [c for c in CONV_CASES if c[3] >= 32]


def _affine(C, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(C, generator=g) * 0.8, torch.randn(C, generator=g) * 0.5


@pytest.mark.parametrize('case', AFF_CASES)
def test_conv_fwd_bn_input_transform(case):
    """conv(relu(y*sc + sh)) with the transform inside the A loader == conv of the
    materialised input (padding taps stay zero)."""
    N, H, W, C, Co, K, s, p = case
    y = _bf(N, H, W, C, seed=31)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=32)
    sc, sh = _affine(C, 33)
    ref = Fn.conv2d_fwd(Fn.bn_relu_input(y, (sc, sh)), w, s, p)
    s1, s2 = Fn.stat_buffers(Co, DEV)
    out = Fn.conv2d_fwd(y.to(DEV), w.to(DEV), s, p, stats=(s1, s2), in_affine=(sc.to(DEV), sh.to(DEV)))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2
    assert rel_err(s1.reshape(Fn.NSTAT, Co).sum(0), ref.float().reshape(-1, Co).sum(0)) < 2e-2


@pytest.mark.parametrize('case', AFF_CASES)
def test_conv_wgrad_bn_input_transform(case):
    N, H, W, C, Co, K, s, p = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    y = _bf(N, H, W, C, seed=34)
    dy = _bf(N, Ho, Wo, Co, seed=35)
    sc, sh = _affine(C, 36)
    ref = Fn.conv2d_wgrad(dy, Fn.bn_relu_input(y, (sc, sh)), (Co, K, K, C), s, p)
    out = Fn.conv2d_wgrad(dy.to(DEV), y.to(DEV), (Co, K, K, C), s, p, in_affine=(sc.to(DEV), sh.to(DEV)))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 5e-3


def test_bn_apply_residual_affine():
    C = 64
    y = _bf(2, 3, 4, C, seed=17)
    r = _bf(2, 3, 4, C, seed=18)
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    rs, rh = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    ref = Fn.bn_apply(y, r, sc, sh, True, res_affine=(rs, rh))
    out = Fn.bn_apply(y.to(DEV), r.to(DEV), sc.to(DEV), sh.to(DEV), True,
                      res_affine=(rs.to(DEV), rh.to(DEV)))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2


@pytest.fixture(params=[1, 4], ids=['bn-u1', 'bn-u4'])
def bn_unroll(request):
    """The BN elementwise passes with 1 and with 4 chunks per thread per iteration."""
    from mlcomp_amd.ops import _lib
    lib = _lib.load()
    old = lib.mlc_bn_get_set(0, request.param)
    yield request.param
    lib.mlc_bn_get_set(0, old)


@pytest.fixture(params=[True, False], ids=['bn-fused', 'bn-2pass'])
def bn_fused(request, monkeypatch):
    """The BN passes with the per-channel finalize folded into the apply launch
    (bn_{fwd,bwd}_fused_kernel) and as separate finalize + apply launches."""
    monkeypatch.setattr(Fn, 'BN_FUSED', request.param)
    yield request.param


@pytest.mark.parametrize('relu,res', [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize('C,shape', [(64, (4, 5, 3)), (256, (4, 5, 3)), (2048, (4, 5, 3)), (256, (4, 50, 31)),
                                     (48, (4, 9, 7)), (768, (4, 50, 31)), (320, (2, 9, 7))])
def test_bn_fwd_bwd(relu, res, C, shape, bn_unroll, bn_fused):
    rows_shape = (*shape, C)
    y = _bf(*rows_shape, scale=2.0, seed=7) + 0.5
    r = _bf(*rows_shape, seed=8) if res else None
    gamma = torch.rand(C) + 0.5
    beta = torch.randn(C) * 0.1
    yf = y.float().reshape(-1, C)
    s1, s2 = Fn.stat_buffers(C, 'cpu')
    s1[:C], s2[:C] = yf.sum(0), (yf * yf).sum(0)

    def run(dev):
        t = lambda v: None if v is None else v.to(dev)
        sm, si = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        z = Fn.bn_fwd_apply(t(y), t(r), t(s1), t(s2), t(gamma), t(beta), sm, si, rm, rv, relu=relu)
        dz = _bf(*rows_shape, seed=9).to(dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        dy, dres = Fn.bn_bwd(dz, z if relu else None, t(y), sm, si, t(gamma), want_dres=res,
                             dgamma=dg, dbeta=db)
        return z, sm, si, rm, rv, dy, dres, dg, db

    ref = run('cpu')
    out = run(DEV)
    torch.cuda.synchronize()
    for a, b in zip(out, ref):
        if b is None:
            assert a is None
            continue
        assert rel_err(a, b) < 1e-2


@pytest.mark.parametrize('C', [64, 512, 1024])
def test_bn_fused_matches_two_pass_with_residual_affine(C, monkeypatch):
    """Folded finalize + apply (one launch each way) gives the two-launch form's outputs, with
    the downsample branch's BN folded in as the residual's affine and the prereduced
    backward (sums from a dgrad epilogue)."""
    rows_shape = (3, 11, 13, C)
    y = (_bf(*rows_shape, scale=2.0, seed=21) + 0.5).to(DEV)
    r = _bf(*rows_shape, seed=22).to(DEV)
    g = torch.Generator().manual_seed(23)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    rs, rh = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    yf = y.float().reshape(-1, C)
    s1, s2 = Fn.stat_buffers(C, DEV)
    s1[:C], s2[:C] = yf.sum(0), (yf * yf).sum(0)
    dz = _bf(*rows_shape, seed=24).to(DEV)

    def run(fused):
        monkeypatch.setattr(Fn, 'BN_FUSED', fused)
        sm, si, rm, rv = (torch.zeros(C, device=DEV) for _ in range(4))
        sc, sh = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        z = Fn.bn_fwd_apply(y, r, s1, s2, gamma, beta, sm, si, rm, rv, relu=True, scale=sc, shift=sh,
                            res_affine=(rs, rh))
        d = dz * (z > 0)
        sums = torch.zeros(Fn.NSTAT * 2 * C, device=DEV)
        df = d.float().reshape(-1, C)
        sums[:C] = df.sum(0)
        sums[C:2 * C] = (df * (yf - sm)).sum(0)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        dy, dres = Fn.bn_bwd(d, None, y, sm, si, gamma, want_dres=True, dgamma=dg, dbeta=db, sums=sums,
                             prereduced=True)
        torch.cuda.synchronize()
        return [z, sm, si, rm, rv, sc, sh, dy, dres, dg, db]

    for a, b in zip(run(True), run(False)):
        # fp32 statistics: summation order only; bf16 tensors: an fp32-ulp change of a
        # coefficient may flip an element's bf16 rounding
        tol = 1e-5 if a.dtype == torch.float32 else 5e-3
        assert rel_err(a, b) < tol, (a.shape, a.dtype, rel_err(a, b))


def test_maxpool():
    x = _bf(2, 12, 12, 64, seed=10)
    y_ref, idx_ref = Fn.maxpool_fwd(x)
    y, idx = Fn.maxpool_fwd(x.to(DEV))
    assert rel_err(y, y_ref) == 0.0
    dy = _bf(*y.shape, seed=11)
    dx_ref = Fn.maxpool_bwd(dy, idx_ref, x.shape)
    dx = Fn.maxpool_bwd(dy.to(DEV), idx, x.shape)
    torch.cuda.synchronize()
    assert rel_err(dx, dx_ref) < 1e-2


def test_avgpool():
    x = _bf(3, 7, 7, 2048, seed=12)
    assert rel_err(Fn.avgpool_fwd(x.to(DEV)), Fn.avgpool_fwd(x)) < 1e-2
    dy = _bf(3, 2048, seed=13)
    assert rel_err(Fn.avgpool_bwd(dy.to(DEV), x.shape), Fn.avgpool_bwd(dy, x.shape)) < 1e-2


@pytest.mark.parametrize('B,I,O', [(16, 2048, 1000), (40, 64, 24)])
def test_linear(B, I, O):
    x = _bf(B, I, seed=14)
    w = _bf(O, I, scale=I ** -0.5, seed=15)
    b = torch.randn(O)
    assert rel_err(Fn.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV)), Fn.linear_fwd(x, w, b)) < 1e-2
    do = _bf(B, O, seed=16)
    assert rel_err(Fn.linear_dgrad(do.to(DEV), w.to(DEV)), Fn.linear_dgrad(do, w)) < 1e-2
    assert rel_err(Fn.linear_wgrad(do.to(DEV), x.to(DEV)), Fn.linear_wgrad(do, x)) < 1e-2


def test_softmax_ce():
    B, V = 32, 1000
    logits = torch.randn(B, V) * 3
    labels = torch.randint(0, V, (B,))
    lc, cc = torch.zeros(1), torch.zeros(1)
    dref = Fn.softmax_ce(logits, labels, lc, cc, smoothing=0.1)
    lg, cg = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    d = Fn.softmax_ce(logits.to(DEV), labels.to(DEV), lg, cg, smoothing=0.1)
    torch.cuda.synchronize()
    assert abs(lg.item() - lc.item()) / lc.item() < 1e-4
    assert cg.item() == cc.item()
    assert rel_err(d, dref) < 1e-2


def test_sgd_adam():
    n, nd, nb = 4096, 3000, 3000
    p = torch.randn(n)
    g = torch.randn(n)
    hyper = torch.tensor([0.1, 0.5, 0.9, 0.99])
    for first in (True, False):
        pc, mc = p.clone(), torch.randn(n)
        pg, mg = pc.to(DEV), mc.to(DEV)
        bfc, bfg = torch.zeros(n, dtype=torch.bfloat16), torch.zeros(n, dtype=torch.bfloat16, device=DEV)
        Fn.sgd_step(pc, g, mc, bfc, hyper, nd, nb, 0.9, 0.0, 1e-4, True, first)
        Fn.sgd_step(pg, g.to(DEV), mg, bfg, hyper.to(DEV), nd, nb, 0.9, 0.0, 1e-4, True, first)
        torch.cuda.synchronize()
        assert rel_err(pg, pc) < 1e-6 and rel_err(mg, mc) < 1e-6 and rel_err(bfg, bfc) < 1e-2
    pc, mc, vc = p.clone(), torch.zeros(n), torch.zeros(n)
    pg, mg, vg = pc.to(DEV), mc.to(DEV), vc.to(DEV)
    Fn.adam_step(pc, g, mc, vc, None, hyper, nd, 0, wd=0.01)
    Fn.adam_step(pg, g.to(DEV), mg, vg, None, hyper.to(DEV), nd, 0, wd=0.01)
    torch.cuda.synchronize()
    assert rel_err(pg, pc) < 1e-5


@pytest.mark.parametrize('variant', [0, 1, 2])
def test_adam_kernel_variants(variant):
    """Every Adam kernel variant (float4 pairs / 8-float chunks / nontemporal) against the
    CPU reference, with n % 8 == 4 and the decay / bf16-mirror boundaries inside a chunk."""
    from mlcomp_amd.ops import _lib
    lib = _lib.load()
    old = lib.mlc_opt_config(0, variant)
    try:
        n, nd, nb = 8196, 4100, 4100
        p, g = torch.randn(n), torch.randn(n)
        hyper = torch.tensor([0.01, 0.5, 0.9, 0.99])
        pc, mc, vc = p.clone(), torch.randn(n) * 0.1, torch.rand(n) * 0.1
        pg, mg, vg = pc.to(DEV), mc.to(DEV), vc.to(DEV)
        bfc, bfg = torch.zeros(n, dtype=torch.bfloat16), torch.zeros(n, dtype=torch.bfloat16, device=DEV)
        Fn.adam_step(pc, g, mc, vc, bfc, hyper, nd, nb, wd=0.01)
        Fn.adam_step(pg, g.to(DEV), mg, vg, bfg, hyper.to(DEV), nd, nb, wd=0.01)
        torch.cuda.synchronize()
        assert rel_err(pg, pc) < 1e-5 and rel_err(mg, mc) < 1e-6 and rel_err(vg, vc) < 1e-6
        assert rel_err(bfg[:nb], bfc[:nb]) < 1e-2 and bfg[nb:].abs().max().item() == 0
    finally:
        lib.mlc_opt_config(0, old)


@pytest.mark.parametrize('case', [(2, 16, 16, 64, 128, 1, 2, 0), (2, 14, 14, 64, 64, 3, 1, 1),
                                  (2, 16, 16, 64, 128, 3, 2, 1)])
def test_conv_dgrad_addend(case):
    N, H, W, C, Co, K, s, p = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    dy = _bf(N, Ho, Wo, Co, seed=21)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=22)
    add = _bf(N, H, W, C, seed=23)
    ref = Fn.conv2d_dgrad(dy, w, (N, H, W, C), s, p, addend=add)
    a = add.to(DEV)
    out = Fn.conv2d_dgrad(dy.to(DEV), w.to(DEV), (N, H, W, C), s, p, addend=a, out=a)  # in place
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize('aff', [False, True])
@pytest.mark.parametrize('case,two', [((2, 14, 14, 64, 64, 1, 1, 0), False),
                                      ((2, 14, 14, 64, 64, 1, 1, 0), True),
                                      ((2, 14, 14, 64, 128, 3, 1, 1), True),
                                      ((2, 16, 16, 64, 128, 3, 2, 1), False),
                                      ((2, 15, 13, 128, 64, 3, 2, 1), True),
                                      ((1, 7, 7, 2048, 512, 1, 1, 0), True)])
def test_conv_dgrad_bn_epilogue(case, two, aff):
    """Fused BN-backward reduction in the dgrad epilogue: masked dx and per-channel
    sums match the CPU reference (which reduces the same bf16-rounded values)."""
    N, H, W, C, Co, K, s, p = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    dy = _bf(N, Ho, Wo, Co, seed=31)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=32)
    add = _bf(N, H, W, C, seed=33)
    z = _bf(N, H, W, C, seed=34)
    y0, y1 = _bf(N, H, W, C, seed=35), _bf(N, H, W, C, seed=36)
    m0, m1 = torch.randn(C) * 0.1, torch.randn(C) * 0.1

    def run(dev):
        t = lambda v: v.to(dev)  # noqa: E731
        sums = [torch.zeros(Fn.NSTAT * 2 * C, device=dev) for _ in range(2)]
        ys = [(t(y0), t(m0), sums[0])] + ([(t(y1), t(m1), sums[1])] if two else [])
        if aff:   # ReLU mask recomputed from y0 (and y1) with per-channel affines
            spec = Fn.BnBwdSpec(None, ys, affine=[(t(a0), t(h0))] + ([(t(a1), t(h1))] if two else []))
        else:
            spec = Fn.BnBwdSpec(t(z), ys)
        dx = Fn.conv2d_dgrad(t(dy), t(w), (N, H, W, C), s, p, addend=t(add), bn=spec)
        return dx, [x.view(Fn.NSTAT, 2, C).sum(0).cpu() for x in sums]

    a0, h0, a1, h1 = torch.rand(C) + 0.5, torch.randn(C) * 0.2, torch.rand(C) + 0.5, torch.randn(C) * 0.2
    ref_dx, ref_s = run('cpu')
    dx, sg = run(DEV)
    torch.cuda.synchronize()
    assert rel_err(dx, ref_dx) < 1e-2
    if aff:
        q = y0.float() * a0 + h0 + ((y1.float() * a1 + h1) if two else 0)
        assert ((dx.cpu().float() != 0) <= (q > 0)).all()
    else:
        assert ((dx.cpu().float() != 0) <= (z.float() > 0)).all()    # masked
    for k in range(2 if two else 1):
        assert rel_err(sg[k][0], ref_s[k][0]) < 2e-2, k
        assert rel_err(sg[k][1], ref_s[k][1]) < 2e-2, k


def test_native_fused_bn_bwd_matches_unfused():
    """Engine-level: gradients with the BN-backward reduction fused into dgrad epilogues and
    the inner BN+ReLU applied inside the next conv's loaders equal (up to float-atomic
    order) the ones from the separate reduction / apply kernels."""
    torch.manual_seed(5)
    from mlcomp_amd.models import build_model
    from mlcomp_amd.train.native_step import NativeClassifierStep
    tm1 = build_model('resnet50', num_classes=16)
    tm2 = build_model('resnet50', num_classes=16)
    tm2.load_state_dict(tm1.state_dict())
    a = NativeClassifierStep(torch_model=tm1, batch=8, image_size=64, device=DEV, num_classes=16,
                             use_graph=False, lr=0.0, momentum=0.0)
    b = NativeClassifierStep(torch_model=tm2, batch=8, image_size=64, device=DEV, num_classes=16,
                             use_graph=False, lr=0.0, momentum=0.0)
    for blk in a.net.blocks:
        blk.fuse_bn_fwd = True     # every inner BN+ReLU applied in the next conv's loaders
    for blk in b.net.blocks:
        blk.fuse_bn_bwd = False
        blk.fuse_bn_fwd = False
    b.load_batch(a.x, a.y)
    a()
    b()
    torch.cuda.synchronize()
    ga, gb = a.net.arena.decay.grad, b.net.arena.decay.grad
    assert ((ga - gb).norm() / gb.norm()).item() < 2e-2
    na, nb = a.net.arena.nodecay.grad, b.net.arena.nodecay.grad
    assert ((na - nb).norm() / nb.norm()).item() < 2e-2


@pytest.mark.parametrize('shape', [(2, 12, 12, 64), (3, 11, 13, 64), (2, 10, 9, 32)])
def test_stem_pool_fused(shape):
    """Fused BN-apply + ReLU + maxpool 3x3/2 and its backward through the BN (stem.hip)
    vs the fp32 reference path."""
    C = shape[-1]
    y = _bf(*shape, scale=2.0, seed=21)
    g = torch.Generator().manual_seed(22)
    scale = torch.rand(C, generator=g) * 2 - 0.5      # some negative gammas
    shift = torch.randn(C, generator=g) * 0.5
    mean = torch.randn(C, generator=g) * 0.1
    invstd = torch.rand(C, generator=g) + 0.5
    gamma = torch.rand(C, generator=g) + 0.5
    Ho, Wo = (shape[1] - 1) // 2 + 1, (shape[2] - 1) // 2 + 1
    dp = _bf(shape[0], Ho, Wo, C, seed=23)

    def run(dev):
        t = lambda v: v.to(dev)
        out, idx = Fn.stem_pool_fwd(t(y), t(scale), t(shift))
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        sums = torch.zeros(Fn.NSTAT * 2 * C, device=dev)
        coef = torch.empty(3 * C, device=dev)
        dy = Fn.stem_pool_bwd(t(dp), idx, t(y), t(mean), t(invstd), t(gamma), dg, db, sums, coef)
        return out, dy, dg, db

    ref = run('cpu')
    res = run(DEV)
    torch.cuda.synchronize()
    assert rel_err(res[0], ref[0]) < 5e-3
    for a, b in zip(res[1:], ref[1:]):
        assert rel_err(a, b) < 1e-2


def test_stem_s2d_conv():
    """Space-to-depth stem: the HIP s2d transform matches the reference, and the 4x4/1 conv
    over it with the regrouped filter equals the 7x7/2 pad-3 conv."""
    x = _bf(2, 30, 26, 8, seed=31)
    x[..., 3:] = 0
    xs_ref = Fn.stem_s2d(x)
    xs = Fn.stem_s2d(x.to(DEV))
    torch.cuda.synchronize()
    assert rel_err(xs, xs_ref) == 0.0
    w = torch.randn(64, 3, 7, 7, generator=torch.Generator().manual_seed(32)) * 0.1
    w2 = Fn.stem_w_to_s2d(w).to(torch.bfloat16)
    y = Fn.conv2d_fwd(xs, w2.to(DEV), 1, 0, 1)
    ref = torch.nn.functional.conv2d(x[..., :3].permute(0, 3, 1, 2).float(), w.to(torch.bfloat16).float(),
                                     stride=2, padding=3).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert rel_err(y, ref) < 1e-2


def test_splitk_fused_reduction_matches_separate_pass():
    """Split-K GEMMs reduce their slabs inside the launch (last-arriving split; knob 6 =
    the per-tile slab KB it may read, here large enough for every split count) or in a
    separate reduce / finalize kernel (knob 6 = 0): same results, and repeated launches
    (tile counters reset by the reducer) stay identical."""
    import math
    from mlcomp_amd.ops import _lib
    from mlcomp_amd.ops import transformer as Tx
    lib = _lib.load()
    N, H, W, C, Co = 16, 14, 14, 256, 256
    x, dy = _bf(N, H, W, C, seed=31).to(DEV), _bf(N, H, W, Co, seed=32).to(DEV)
    T, I, O = 4096, 768, 768
    a, wt = _bf(T, I, seed=33).to(DEV), _bf(O, I, scale=I ** -0.5, seed=34).to(DEV)
    bias = torch.randn(O, device=DEV)
    u = _bf(T, I, seed=35).to(DEV)
    add = _bf(T, I, seed=36).to(DEV)
    g = _bf(T, O, seed=37).to(DEV)

    def run():
        outs = []
        for _ in range(3):
            wg = torch.full((Co, 3, 3, C), 0.5, device=DEV)
            Fn.conv2d_wgrad(dy, x, (Co, 3, 3, C), 1, 1, out=wg, accumulate=True)
            y, pre = Tx.dense_fwd(a, wt, bias, act=1, want_preact=True)
            dx = Tx.dense_dgrad(g, wt, dact_u=u, addend=add)
            dw, db = torch.zeros(O, I, device=DEV), torch.zeros(O, device=DEV)
            Fn.linear_wgrad_bias(g, a, dw, db)
            outs.append([wg, y, pre, dx, dw, db])
        torch.cuda.synchronize()
        names = ['conv wgrad', 'dense fwd', 'preact', 'dense dgrad', 'linear wgrad']
        for o in outs[1:]:
            for k, nm in enumerate(names):   # deterministic: the reducer sums slabs in split order
                assert torch.equal(o[k], outs[0][k]), (nm, rel_err(o[k], outs[0][k]))
            assert rel_err(o[5], outs[0][5]) < 1e-6   # bias gradient: column-sum atomics
        return outs[0]

    old = lib.mlc_gemm_get_set(6, 1 << 20)
    try:
        fused = run()
        assert lib.mlc_gemm_get_set(6, 0) == 1 << 20 and lib.mlc_gemm_get_set(6, -1) == 0
        sep = run()
    finally:
        lib.mlc_gemm_get_set(6, old)
    for f, s_ in zip(fused, sep):
        assert rel_err(f, s_) < 1e-5
    ref = Fn.conv2d_wgrad(dy.cpu(), x.cpu(), (Co, 3, 3, C), 1, 1) + 0.5
    assert rel_err(fused[0], ref) < 5e-3
    z = a.float() @ wt.float().t() + bias
    assert rel_err(fused[2], z) < 1e-2
    assert rel_err(fused[1], 0.5 * z * (1 + torch.erf(z / math.sqrt(2)))) < 1e-2


class _FakeSlot:
    """Stand-in for an arena slot: a [Co, KH, KW, Ci] bf16 filter."""

    def __init__(self, w):
        self.shape, self.numel, self._w = tuple(w.shape), w.numel(), w

    @property
    def bf16(self):
        return self._w


def test_wt_table_transpose_batched():
    """One launch transposes + flips every registered filter (odd channel counts, 1x1,
    3x3, 5x3 taps, > 64 channels on both axes) exactly."""
    ws = [_bf(64, 3, 3, 64, seed=40), _bf(200, 1, 1, 72, seed=41), _bf(40, 5, 3, 136, seed=42),
          _bf(512, 3, 3, 256, seed=43)]
    tab = Fn.WtTable()
    for w in ws:
        tab.add(_FakeSlot(w.to(DEV)))
    tab.finalize(DEV)
    tab.refresh()
    torch.cuda.synchronize()
    for i, w in enumerate(ws):
        assert torch.equal(tab[i].cpu(), Fn.wt_flip_transpose(w)), i


WT_CASES = [
    # N, H, W, C, Co, K, stride, pad, dil
    (2, 14, 14, 64, 64, 1, 1, 0, 1),
    (2, 14, 14, 64, 128, 3, 1, 1, 1),
    (3, 9, 7, 136, 40, 3, 1, 1, 1),
    (1, 7, 7, 512, 2048, 1, 1, 0, 1),
    (2, 12, 12, 64, 64, 3, 1, 2, 2),      # dilated
    (2, 10, 10, 64, 96, 3, 1, 0, 1),      # 'valid' conv: dx padded by 2
    (2, 56, 56, 64, 64, 3, 1, 1, 1),
    (2, 16, 16, 64, 128, 3, 2, 1, 1),     # strided: parity classes + ConvDgradBT
    (2, 15, 13, 128, 64, 3, 2, 1, 1),
    (3, 15, 15, 64, 128, 1, 2, 0, 1),     # 1x1/2: three classes no tap reaches
    (2, 13, 11, 64, 72, 3, 3, 1, 1),      # stride 3, Co % 64 != 0
]


@pytest.mark.parametrize('case', WT_CASES)
def test_conv_dgrad_transposed_filter(case):
    """dgrad over the flipped transposed filter (stride 1: as a forward conv; strided: the
    parity-class GEMMs with the K-contiguous filter loader) matches the fp32 reference of
    the plain dgrad, with the addend + fused BN-backward epilogue too."""
    N, H, W, C, Co, K, st, p, d = case
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, st, p, d)
    dy = _bf(N, Ho, Wo, Co, seed=44)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=45)
    wt = Fn.wt_flip_transpose(w)
    ref = Fn.conv2d_dgrad(dy, w, (N, H, W, C), st, p, d)
    out = Fn.conv2d_dgrad(dy.to(DEV), w.to(DEV), (N, H, W, C), st, p, d, wt=wt.to(DEV))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2
    add, z, y0 = _bf(N, H, W, C, seed=46), _bf(N, H, W, C, seed=47), _bf(N, H, W, C, seed=48)
    m0 = torch.randn(C) * 0.1

    def run(dev, use_wt):
        t = lambda v: v.to(dev)  # noqa: E731
        sums = torch.zeros(Fn.NSTAT * 2 * C, device=dev)
        spec = Fn.BnBwdSpec(t(z), [(t(y0), t(m0), sums)])
        dx = Fn.conv2d_dgrad(t(dy), t(w), (N, H, W, C), st, p, d, addend=t(add), bn=spec,
                             wt=t(wt) if use_wt else None)
        return dx, sums.view(Fn.NSTAT, 2, C).sum(0).cpu()

    rdx, rs = run('cpu', False)
    gdx, gs = run(DEV, True)
    torch.cuda.synchronize()
    assert rel_err(gdx, rdx) < 1e-2
    assert rel_err(gs[0], rs[0]) < 2e-2 and rel_err(gs[1], rs[1]) < 2e-2


@pytest.fixture(params=[0, 1], ids=['regs', 'dma'])
def gemm_dma(request):
    """The register-staged and the LDS-DMA main loop (knob 8), restored after."""
    from mlcomp_amd.ops import _lib
    lib = _lib.load()
    old = lib.mlc_gemm_get_set(8, request.param)
    yield
    lib.mlc_gemm_get_set(8, 1 if old < 0 else old)


@pytest.mark.parametrize('case', [c for c in CONV_CASES if c[3] != 8] + [(2, 28, 28, 128, 128, 3, 1, 1)])
def test_conv_fwd_dgrad_lds_dma(case, gemm_dma):
    """Forward conv (+BN statistics), transposed-filter dgrad and weight gradient on both
    main loops: register-staged, and LDS-DMA (operands copied global -> LDS by
    buffer_load ... lds, the swizzle applied on the source side)."""
    N, H, W, C, Co, K, s, p = case
    x = _bf(N, H, W, C, seed=51)
    w = _bf(Co, K, K, C, scale=(1.0 / (K * K * C)) ** 0.5, seed=52)
    s1c, s2c = Fn.stat_buffers(Co, 'cpu')
    ref = Fn.conv2d_fwd(x, w, s, p, stats=(s1c, s2c))
    s1g, s2g = Fn.stat_buffers(Co, DEV)
    out = Fn.conv2d_fwd(x.to(DEV), w.to(DEV), s, p, stats=(s1g, s2g))
    torch.cuda.synchronize()
    assert rel_err(out, ref) < 1e-2
    red = lambda t: t.reshape(Fn.NSTAT, Co).sum(0)  # noqa: E731
    assert rel_err(red(s1g), red(s1c)) < 1e-2 and rel_err(red(s2g), red(s2c)) < 1e-2
    Ho, Wo = Fn.conv_out_hw(H, W, K, K, s, p, 1)
    dy = _bf(N, Ho, Wo, Co, seed=53)
    rd = Fn.conv2d_dgrad(dy, w, (N, H, W, C), s, p)
    gd = Fn.conv2d_dgrad(dy.to(DEV), w.to(DEV), (N, H, W, C), s, p, wt=Fn.wt_flip_transpose(w).to(DEV))
    torch.cuda.synchronize()
    assert rel_err(gd, rd) < 1e-2
    # weight gradient (MN-contiguous operands: register-staged copy in both modes)
    rw = Fn.conv2d_wgrad(dy, x, w.shape, s, p)
    gw = Fn.conv2d_wgrad(dy.to(DEV), x.to(DEV), w.shape, s, p)
    torch.cuda.synchronize()
    assert rel_err(gw, rw) < 1e-2


@pytest.mark.parametrize('B,I,O', [(4096, 768, 2304), (300, 3072, 768), (512, 136, 72)])
def test_linear_lds_dma(B, I, O, gemm_dma):
    """Plain-matrix GEMM (both operands K-contiguous) on the LDS-DMA main loop, including
    row / column / K tails."""
    from mlcomp_amd.ops import transformer as Tx
    x, w = _bf(B, I, seed=54), _bf(O, I, seed=55, scale=I ** -0.5)
    bias = torch.randn(O) * 0.1
    yr, _ = Tx.dense_fwd(x, w, bias)
    yg, _ = Tx.dense_fwd(x.to(DEV), w.to(DEV), bias.to(DEV))
    torch.cuda.synchronize()
    assert rel_err(yg, yr) < 1e-2
    dy = _bf(B, O, seed=56)     # input gradient: the filter operand is MN-contiguous
    dr = Tx.dense_dgrad(dy, w)
    dg = Tx.dense_dgrad(dy.to(DEV), w.to(DEV))
    torch.cuda.synchronize()
    assert rel_err(dg, dr) < 1e-2



@pytest.mark.parametrize('kt,st,pt,dt', [(3, 1, 1, 1), (3, 2, 1, 1), (5, 1, 2, 1), (3, 1, 2, 2), (2, 2, 0, 1)])
def test_temporal_unfold_fold_match_torch(kt, st, pt, dt):
    """Native temporal unfold (Conv3d taps -> channels of the frame tensor) and its gradient
    fold (a gather over taps, csrc/kernels/video.hip) against the torch pad / index_select
    reference and its autograd gradient (fp32)."""
    from mlcomp_amd.ops.glayers import Conv3dAs2d
    conv = torch.nn.Conv3d(16, 8, (kt, 3, 3), (st, 1, 1), (pt, 1, 1), (dt, 1, 1))
    c = Conv3dAs2d(conv)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 16, 7, 5, 6, generator=g).to(torch.bfloat16)
    xg = x.cuda().contiguous(memory_format=torch.channels_last_3d).requires_grad_()
    got = c.unfold(xg)
    xr = x.float().requires_grad_()
    want = c.unfold(xr)                             # CPU: the torch gather path
    assert got.shape == want.shape
    assert torch.equal(got.float().cpu(), want.to(torch.bfloat16).float())
    dg = torch.randn(want.shape, generator=g).to(torch.bfloat16)
    got.backward(dg.cuda())
    want.backward(dg.float())
    err = (xg.grad.float().cpu() - xr.grad).abs().max() / xr.grad.abs().max()
    assert err < 1e-2, err


@pytest.mark.parametrize('frames_layout', [True, False])
def test_temporal_fold_sums_the_handed_off_gradient(frames_layout):
    """The fold kernel's addend (the other branch's gradient of a residual block's input,
    glayers.Frames hand-off): fold(dcol) + addend in one pass, for an addend given as a
    site's NHWC frame gradient or as a logical channels_last_3d tensor, against fp32."""
    from mlcomp_amd.ops.glayers import temporal_fold, temporal_unfold
    g = torch.Generator().manual_seed(3)
    N, C, T, H, W, kt, st, pt, dt = 2, 16, 6, 5, 4, 3, 2, 1, 1
    To = (T + 2 * pt - dt * (kt - 1) - 1) // st + 1
    x = torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16).requires_grad_()
    dcol = torch.randn(N * To, C * kt, H, W, generator=g).to(torch.bfloat16)
    add5 = torch.randn(N, C, T, H, W, generator=g).to(torch.bfloat16)
    xr = x.float().detach().requires_grad_()
    from mlcomp_amd.ops.glayers import Conv3dAs2d
    conv = Conv3dAs2d(torch.nn.Conv3d(C, 8, (kt, 1, 1), (st, 1, 1), (pt, 0, 0), (dt, 1, 1)))
    conv.unfold(xr).backward(dcol.float())
    want = xr.grad + add5.float()
    addend = (add5.permute(0, 2, 3, 4, 1).reshape(N * T, H, W, C) if frames_layout
              else add5.contiguous(memory_format=torch.channels_last_3d)).cuda()
    dm = dcol.cuda().contiguous(memory_format=torch.channels_last)
    got = temporal_fold(dm, N, C, T, H, W, kt, st, pt, dt, To, addend=addend)
    torch.cuda.synchronize()
    err = (got.float().cpu() - want).abs().max() / want.abs().max()
    assert err < 1e-2, err
    plain = temporal_fold(dm, N, C, T, H, W, kt, st, pt, dt, To)
    assert torch.allclose(plain.float().cpu(), xr.grad, atol=3e-2, rtol=1e-2)
    assert temporal_unfold is not None


@pytest.mark.parametrize('N,H,C,Co,S', [(64, 28, 128, 512, 1), (24, 56, 64, 256, 1), (96, 28, 256, 1024, 2),
                                        (42, 28, 256, 256, 1)])
def test_persistent_short_k_gemm_matches_tile_kernel(N, H, C, Co, S):
    """The persistent short-K GEMM (knob 14, igemm.hip gemm_persist_kernel: a DMA ring across
    output tiles, raw-barrier epilogue) gives the per-tile kernel's output and BN statistics
    on 1x1 convs (partial last tile, stride 2), and both match the fp32 reference."""
    from mlcomp_amd.ops import _lib
    lib = _lib.load()
    Ho = H // S
    assert (N * Ho * Ho + 127) // 128 * ((Co + 127) // 128) >= 512      # enough tiles for the persistent path
    g = torch.Generator(device='cuda').manual_seed(0)
    x = torch.randn(N, H, H, C, device='cuda', generator=g).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, C, device='cuda', generator=g) * C ** -0.5).to(torch.bfloat16)
    outs = []
    old = lib.mlc_gemm_get_set(14, -1)
    try:
        for p in (0, 1):
            lib.mlc_gemm_get_set(14, p)
            st = torch.zeros(2, Fn.NSTAT * Co, device='cuda')
            y = Fn.conv2d_fwd(x, w, S, 0, 1, stats=(st[0], st[1]))
            torch.cuda.synchronize()
            outs.append((y.float(), st.view(2, Fn.NSTAT, Co).sum(1)))
    finally:
        lib.mlc_gemm_get_set(14, max(old, 0))
    want = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=S)
    want = want.permute(0, 2, 3, 1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert (outs[1][0] - want).abs().max() <= 2e-2 * want.abs().max()
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize('H,W,Ho,Wo', [(16, 16, 6, 6), (16, 16, 3, 3), (17, 13, 6, 4), (8, 8, 2, 2), (5, 7, 6, 6)])
def test_adaptive_avg_pool_matches_fp32(H, W, Ho, Wo):
    """Native adaptive average pool (pool_loss.hip: PyTorch's overlapping bins, fp32 sums) and
    its gather backward against fp32 F.adaptive_avg_pool2d / autograd."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3, H, W, 24, generator=g).to(torch.bfloat16)
    dy = torch.randn(3, Ho, Wo, 24, generator=g).to(torch.bfloat16)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    want = F.adaptive_avg_pool2d(xr, (Ho, Wo))
    want.backward(dy.float().permute(0, 3, 1, 2))
    got = Fn.adaptive_avg_fwd(x.cuda(), Ho, Wo)
    dx = Fn.adaptive_avg_bwd(dy.cuda(), tuple(x.shape))
    torch.cuda.synchronize()
    assert (got.float().cpu() - want.detach().permute(0, 2, 3, 1)).abs().max() <= 8e-3 * want.abs().max()
    assert (dx.float().cpu() - xr.grad.permute(0, 2, 3, 1)).abs().max() <= 8e-3 * xr.grad.abs().max()


@pytest.mark.parametrize('act,res,rowscale', [(1, True, False), (3, False, False), (0, True, True), (8, False, False)])
@pytest.mark.parametrize('C', [48, 256, 1024])
def test_bnact_fused_matches_finalize_then_apply(act, res, rowscale, C):
    """normact.hip apply_fused_kernel (the generic engine's BN finalize folded into its apply
    pass) gives the outputs of mlc_bn_finalize + mlc_bnact_apply: z, the per-channel
    mean / invstd / scale / shift and the running statistics."""
    N, HW = 3, 37
    y = (_bf(N, HW, 1, C, scale=2.0, seed=41) + 0.5).to(DEV)
    r = _bf(N, HW, 1, C, seed=42).to(DEV) if res else None
    g = torch.Generator().manual_seed(43)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    rsc = (torch.rand(N, generator=g) + 0.5).to(DEV) if rowscale else None
    yf = y.float().reshape(-1, C)
    s1, s2 = Fn.stat_buffers(C, DEV)
    s1[:C], s2[:C] = yf.sum(0), (yf * yf).sum(0)
    outs = []
    for fused in (True, False):
        st = torch.zeros(4, C, device=DEV)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        if fused:
            z = Fn.bnact_fused(y, r, s1, s2, gamma, beta, st[2], st[3], st[0], st[1], rm, rv, 1e-5, 0.1, act,
                               0.0, row_scale=rsc)
            assert z is not None
        else:
            Fn.bn_finalize(s1, s2, N * HW, gamma, beta, st[2], st[3], st[0], st[1], rm, rv, 1e-5, 0.1)
            z = Fn.bnact_apply(y, r, st[0], st[1], act, 0.0, row_scale=rsc)
        torch.cuda.synchronize()
        outs.append([z, st, rm, rv])
    for a, b in zip(*outs):
        tol = 1e-5 if a.dtype == torch.float32 else 5e-3
        assert rel_err(a, b) < tol, (a.dtype, rel_err(a, b))


def test_bn_stats_into_a_channel_slice():
    """mlc_bn_stats_ld: the per-channel sums of a 16-channel tensor land in channels 24..39 of
    40-wide statistics copies (a DenseNet concat's new segment), equal to the plain reduction."""
    x = _bf(2, 9, 7, 16, seed=61).to(DEV)
    s1, s2 = Fn.stat_buffers(40, DEV)
    Fn.bn_stats(x, s1.view(-1, 40)[:, 24:], s2.view(-1, 40)[:, 24:], ld=40)
    r1, r2 = Fn.stat_buffers(16, DEV)
    Fn.bn_stats(x, r1, r2)
    torch.cuda.synchronize()
    got1, got2 = s1.view(-1, 40).sum(0), s2.view(-1, 40).sum(0)
    assert float(got1[:24].abs().max()) == 0.0 and float(got2[:24].abs().max()) == 0.0
    assert rel_err(got1[24:], r1.view(-1, 16).sum(0)) < 1e-5
    assert rel_err(got2[24:], r2.view(-1, 16).sum(0)) < 1e-5


@pytest.mark.parametrize('act', [1, 3])
def test_bnact_bwd_adds_a_strided_channel_slice(act):
    """normact backward apply with an addend that is a channel slice of a wider NHWC gradient
    (a DenseNet concat's gradient, row stride 40 for 24 channels): GPU against the fp32 CPU
    path of the same call."""
    C, W = 24, 40
    y = (_bf(2, 5, 6, C, scale=2.0, seed=71) + 0.3)
    dz = _bf(2, 5, 6, C, seed=72)
    wide = _bf(2, 5, 6, W, seed=73)
    g = torch.Generator().manual_seed(74)
    gamma, beta = torch.rand(C, generator=g) + 0.5, torch.randn(C, generator=g) * 0.1
    yf = y.float().reshape(-1, C)
    mean, var = yf.mean(0), yf.var(0, unbiased=False)
    inv = torch.rsqrt(var + 1e-5)
    scale, shift = gamma * inv, beta - mean * gamma * inv
    z = Fn.bnact_apply(y, None, scale, shift, act)

    def run(dev):
        t = lambda v: v.to(dev)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dy, _ = Fn.bnact_bwd(t(dz), t(z), t(y), None, t(mean), t(scale), t(shift), t(inv), t(gamma), act,
                             dgamma=dg, dbeta=db, addend=t(wide)[..., :C])
        return dy, dg, db

    ref, out = run('cpu'), run(DEV)
    torch.cuda.synchronize()
    for a, b in zip(out, ref):
        assert rel_err(a, b) < 1e-2


@pytest.mark.parametrize('C,W', [(24, 40), (64, 256), (2064, 2080)])
@pytest.mark.parametrize('act', [1, 3])
def test_bnact_reads_the_leading_channels_of_wider_rows(C, W, act):
    """The normact forward (folded finalize + apply) and backward (reduce, finalize, apply;
    C > 2048 takes the atomic-copies reduce) reading y as the leading C channels of W-wide rows
    (a DenseNet concat buffer, glayers.DenseChain) give what they give on a dense copy of y,
    and the backward matches the fp32 CPU path."""
    N, H, Wd = 2, 3, 4
    wide = (_bf(N, H, Wd, W, scale=2.0, seed=81) + 0.3).to(DEV)
    y = wide[..., :C]
    assert Fn.rows_ld(y) == W
    dz = _bf(N, H, Wd, C, seed=82).to(DEV)
    g = torch.Generator().manual_seed(83)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(DEV), (torch.randn(C, generator=g) * 0.1).to(DEV)
    yf = y.float().reshape(-1, C)
    s1, s2 = Fn.stat_buffers(C, DEV)
    s1[:C], s2[:C] = yf.sum(0), (yf * yf).sum(0)

    def run(yy):
        st = torch.zeros(4, C, device=DEV)
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        z = Fn.bnact_fused(yy, None, s1, s2, gamma, beta, st[2], st[3], st[0], st[1], rm, rv, 1e-5, 0.1, act, 0.0)
        assert z is not None and z.is_contiguous()
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        dy, _ = Fn.bnact_bwd(dz, z, yy, None, st[2], st[0], st[1], st[3], gamma, act, dgamma=dg, dbeta=db)
        torch.cuda.synchronize()
        return [z, st, rm, rv, dy, dg, db]

    strided, dense = run(y), run(y.contiguous())
    for a, b in zip(strided, dense):
        assert rel_err(a, b) < 1e-6, rel_err(a, b)
    # the input gradient stored split in two dense tensors (a DenseNet concat's operands)
    z, st = strided[0], strided[1]
    sp = C - 8
    (da, db), _ = Fn.bnact_bwd(dz, z, y, None, st[2], st[0], st[1], st[3], gamma, act,
                               dgamma=torch.zeros(C, device=DEV), dbeta=torch.zeros(C, device=DEV), split=sp)
    torch.cuda.synchronize()
    assert da.is_contiguous() and db.is_contiguous() and da.shape[-1] == sp and db.shape[-1] == C - sp
    assert torch.equal(da, strided[4][..., :sp]) and torch.equal(db, strided[4][..., sp:])
    z, st = strided[0], strided[1]
    dg, db = torch.zeros(C), torch.zeros(C)
    cpu = Fn.bnact_bwd(dz.cpu(), z.cpu(), y.cpu(), None, st[2].cpu(), st[0].cpu(), st[1].cpu(), st[3].cpu(),
                       gamma.cpu(), act, dgamma=dg, dbeta=db)[0]
    assert rel_err(strided[4], cpu) < 1e-2
    assert rel_err(strided[5], dg) < 1e-2 and rel_err(strided[6], db) < 1e-2


@pytest.mark.parametrize('k,Ci,Co,off,W', [(3, 64, 32, 96, 160), (1, 128, 32, 64, 96), (3, 32, 48, 0, 48 + 80)])
def test_conv_fwd_into_a_channel_slice(k, Ci, Co, off, W):
    """mlc_conv_fwd_ld: a conv writes its output as channels [off, off + Co) of W-wide rows (a
    DenseNet layer's growth channels straight into its block's concat buffer), leaving the other
    channels untouched; equal to the dense conv, which matches fp32 F.conv2d; and the BN
    statistics of that slice read in place equal those of a dense copy."""
    N, H, Wd = 2, 9, 7
    x = _bf(N, H, Wd, Ci, seed=91).to(DEV)
    w = (_bf(Co, k, k, Ci, seed=92) * 0.2).to(DEV)
    buf = torch.full((N, H, Wd, W), 7.0, device=DEV, dtype=torch.bfloat16)
    out = buf[..., off:off + Co]
    y = Fn.conv2d_fwd(x, w, 1, k // 2, 1, out=out)
    dense = Fn.conv2d_fwd(x, w, 1, k // 2, 1)
    torch.cuda.synchronize()
    assert y.data_ptr() == out.data_ptr()
    assert torch.equal(buf[..., off:off + Co], dense)
    assert bool((buf[..., :off] == 7.0).all()) and bool((buf[..., off + Co:] == 7.0).all())
    ref = F.conv2d(x.float().permute(0, 3, 1, 2).cpu(), w.float().permute(0, 3, 1, 2).cpu(), None, 1, k // 2)
    assert rel_err(dense, ref.permute(0, 2, 3, 1)) < 1e-2
    s1, s2 = Fn.stat_buffers(Co, DEV)
    Fn.bn_stats(out, s1, s2)
    r1, r2 = Fn.stat_buffers(Co, DEV)
    Fn.bn_stats(dense, r1, r2)
    torch.cuda.synchronize()
    assert rel_err(s1.view(-1, Co).sum(0), r1.view(-1, Co).sum(0)) < 1e-5
    assert rel_err(s2.view(-1, Co).sum(0), r2.view(-1, Co).sum(0)) < 1e-5
