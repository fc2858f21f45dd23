"""Native U-Net (encoder blocks, fused upsample+concat, fused head + BCE/Dice) against
plain PyTorch autograd of the same model, on CPU (reference op paths)."""
import pytest
import torch

from mlcomp_amd.contrib.criterion import BCEDiceLoss
from mlcomp_amd.contrib.segmentation.models import Unet
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops import seg
from mlcomp_amd.train.native_seg_step import NativeSegmentationStep


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def test_upcat_reference():
    torch.manual_seed(0)
    lo = torch.randn(2, 3, 4, 8).to(torch.bfloat16)
    sk = torch.randn(2, 6, 8, 16).to(torch.bfloat16)
    out = seg.upcat_fwd(lo, sk)
    assert out.shape == (2, 6, 8, 24)
    assert torch.equal(out[:, 5, 7, :8], lo[:, 2, 3])
    assert torch.equal(out[..., 8:], sk)
    d = torch.randn(2, 6, 8, 24).to(torch.bfloat16)
    dlo, dsk = seg.upcat_bwd(d, 8)
    assert torch.allclose(dlo.float()[:, 1, 2], d.float()[:, 2:4, 4:6, :8].sum((1, 2)), atol=2e-2, rtol=1e-2)
    assert torch.equal(dsk, d[..., 8:])


def test_seg_head_matches_bce_dice_autograd():
    P, C = 500, 16
    x = torch.randn(P, C).to(torch.bfloat16)
    w, b = torch.randn(C) * 0.3, torch.randn(1) * 0.1
    t = (torch.rand(P) > 0.6).float()
    sums = torch.zeros(4)
    seg.seg_head_fwd(x, w, b, t, sums)
    xf, wf, bf = x.float().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    ref = BCEDiceLoss()(xf @ wf + bf, t)
    ref.backward()
    assert abs(seg.seg_loss(sums, P).item() - ref.item()) < 1e-5
    dw, db = torch.zeros(C), torch.zeros(1)
    dx = seg.seg_head_bwd(x, w, b, t, sums, dw, db)
    assert torch.allclose(dw, wf.grad, atol=1e-5) and torch.allclose(db, bf.grad, atol=1e-6)
    assert _cos(dx, xf.grad) > 0.9999


def test_native_unet_matches_torch_autograd():
    torch.manual_seed(0)
    tm = Unet(encoder_name='resnet18', classes=1)
    ref = Unet(encoder_name='resnet18', classes=1)
    with torch.no_grad():
        for m in tm.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
    ref.load_state_dict(tm.state_dict())
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', lr=1e-3, use_graph=False)
    x = Fn.stem_s2d_to_nhwc(step.x).permute(0, 3, 1, 2).contiguous()   # the step holds the s2d image
    t = step.t.view(2, 1, 64, 64)
    ref.train()
    loss = BCEDiceLoss()(ref(x), t)
    loss.backward()
    # gradients of one step (before the optimizer mutates the arena: run fwd/bwd by hand)
    net = step.net
    net.ctx.ws.zero()
    net.arena.zero_grad()
    l_nat = net.loss(step.x, step.t)
    l_nat.backward()
    assert abs(l_nat.item() - loss.item()) / loss.item() < 0.03
    a = net.arena.by_name
    # bf16 activations through ~40 BN layers on a 2x64x64 batch: stock torch bf16 autocast
    # of this model reaches only cosine ~0.76-0.78 vs fp32 on the encoder convs (checked
    # when writing this test); the native path measures ~0.83-0.87, so the bar is 0.8
    assert _cos(a['decoder.final_conv.weight'].grad, ref.decoder.final_conv.weight.grad) > 0.95
    g = a['decoder.blocks.4.convs.1.conv.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, ref.decoder.blocks[4].convs[1][0].weight.grad) > 0.9
    g = a['decoder.blocks.0.convs.0.conv.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, ref.decoder.blocks[0].convs[0][0].weight.grad) > 0.8
    g = a['encoder.body.layer2.0.cb1.conv.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, ref.encoder.body.layer2[0].cb1.conv.weight.grad) > 0.8
    g = Fn.stem_w_from_s2d(a['encoder.body.stem.conv.weight'].grad)
    assert _cos(g, ref.encoder.body.stem.conv.weight.grad) > 0.8
    # a full step trains
    losses = []
    for _ in range(4):
        step()
        losses.append(step.last_loss())
    assert losses[-1] < losses[0]
    net.export_to_torch()


@pytest.mark.parametrize('K', [2, 4])
def test_multiclass_seg_head_matches_bce_dice_autograd(K):
    """K sigmoid classes (Severstal-style multi-label masks): BCE mean over pixels x classes
    plus one soft Dice over everything, as contrib.criterion.BCEDiceLoss computes it."""
    P, C = 300, 16
    torch.manual_seed(K)
    x = torch.randn(P, C).to(torch.bfloat16)
    w, b = torch.randn(K, C) * 0.3, torch.randn(K) * 0.1
    t = (torch.rand(P, K) > 0.6).float()
    sums = torch.zeros(4)
    seg.seg_head_fwd(x, w, b, t, sums)
    xf, wf, bf = x.float().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    ref = BCEDiceLoss()(xf @ wf.t() + bf, t)
    ref.backward()
    assert abs(seg.seg_loss(sums, P * K).item() - ref.item()) < 1e-5
    dw, db = torch.zeros(K, C), torch.zeros(K)
    dx = seg.seg_head_bwd(x, w, b, t, sums, dw, db)
    assert torch.allclose(dw, wf.grad, atol=1e-5) and torch.allclose(db, bf.grad, atol=1e-6)
    assert _cos(dx, xf.grad) > 0.9999


def test_native_unet_four_classes_matches_torch():
    torch.manual_seed(1)
    tm = Unet(encoder_name='resnet18', classes=4)
    ref = Unet(encoder_name='resnet18', classes=4)
    ref.load_state_dict(tm.state_dict())
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', lr=1e-3, use_graph=False)
    assert step.classes == 4 and step.t.numel() == 2 * 64 * 64 * 4
    x = Fn.stem_s2d_to_nhwc(step.x).permute(0, 3, 1, 2).contiguous()
    t = step.t.view(2, 64, 64, 4).permute(0, 3, 1, 2)
    ref.train()
    loss = BCEDiceLoss()(ref(x), t)
    loss.backward()
    net = step.net
    net.ctx.ws.zero()
    net.arena.zero_grad()
    l_nat = net.loss(step.x, step.t)
    l_nat.backward()
    assert abs(l_nat.item() - loss.item()) / loss.item() < 0.03
    g = net.arena.by_name['decoder.final_conv.weight'].grad
    assert _cos(g, ref.decoder.final_conv.weight.grad.reshape(4, -1)) > 0.95
    step.load_batch(torch.randn(2, 3, 64, 64), (torch.rand(2, 4, 64, 64) > 0.5).float())
    losses = []
    for _ in range(3):
        step()
        losses.append(step.last_loss())
    assert all(v == v for v in losses)


def test_native_unet_predict_matches_torch_eval():
    """Native validation forward (inference BN, fused head logits + loss) == torch eval."""
    torch.manual_seed(0)
    tm = Unet(encoder_name='resnet18', classes=2)
    with torch.no_grad():
        for m in tm.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    ref = Unet(encoder_name='resnet18', classes=2)
    ref.load_state_dict(tm.state_dict())
    ref.eval()
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', use_graph=False,
                                  bce_w=0.5, dice_w=2.0)
    x = torch.randn(3, 3, 64, 64)          # an eval batch of another size than the train batch
    t = (torch.rand(3, 2, 64, 64) > 0.5).float()
    logits, loss = step.net.predict(Fn.nchw_to_nhwc(x, pad_to=8), t)
    with torch.no_grad():
        want = ref(x.to(torch.bfloat16).float())
    assert logits.shape == want.shape == (3, 2, 64, 64)
    assert _cos(logits, want) > 0.999
    ref_loss = BCEDiceLoss(bce_weight=0.5, dice_weight=2.0)(logits, t)
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    assert step.net.ctx.training           # predict restores the training mode
