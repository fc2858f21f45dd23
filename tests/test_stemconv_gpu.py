"""The space-to-depth stem conv kernel (csrc/kernels/stemconv.hip) against fp32 PyTorch:
output and the fused BN statistics (per-channel sum / sum of squares over the NSTAT copies),
with a pixel count that is and one that is not a multiple of the 32-pixel tile."""
import pytest
import torch
import torch.nn.functional as F

from mlcomp_amd.ops import functional as Fn


@pytest.mark.gpu
@pytest.mark.parametrize('N,Hb,Wb', [(3, 35, 35), (2, 16, 19), (5, 115, 115)])
def test_stem_conv_matches_fp32(N, Hb, Wb):
    torch.manual_seed(0)
    xs = torch.randn(N, Hb, Wb, 16).to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 16) * 0.1).to(torch.bfloat16)
    want = F.conv2d(xs.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float()).permute(0, 2, 3, 1)
    st = torch.zeros(2, Fn.NSTAT * 64, device='cuda')
    y = Fn.stem_conv_fwd(xs.cuda(), w.cuda(), stats=(st[0], st[1]))
    torch.cuda.synchronize()
    assert y.shape == want.shape
    assert (y.float().cpu() - want).abs().max() <= 1e-2 * want.abs().max()
    sums = st.view(2, Fn.NSTAT, 64).sum(1).cpu()
    ref1, ref2 = want.sum((0, 1, 2)), (want * want).sum((0, 1, 2))
    assert (sums[0] - ref1).abs().max() <= 1e-3 * ref2.sqrt().max() * want[..., 0].numel() ** 0.5
    assert ((sums[1] - ref2).abs() / ref2).max() <= 1e-3
    # no statistics requested
    y2 = Fn.stem_conv_fwd(xs.cuda(), w.cuda())
    assert torch.equal(y2, y)
