"""Native FPN (ResNet encoder; lateral / output 1x1 convs as bias-epilogue GEMMs, 3x3 head
convs on the implicit-GEMM kernels, GroupNorm+ReLU with a hand-written backward) against
plain PyTorch autograd of the same model, on CPU (reference op paths).  Reference model:
`mlcomp/contrib/segmentation/fpn/`."""
import torch

from mlcomp_amd.contrib.criterion import BCEDiceLoss
from mlcomp_amd.contrib.segmentation.models import FPN
from mlcomp_amd.models.native_fpn import GNRelu
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import NativeContext
from mlcomp_amd.train.native_seg_step import NativeSegmentationStep


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def test_gn_relu_matches_autograd():
    torch.manual_seed(0)
    gn = torch.nn.GroupNorm(8, 32)
    with torch.no_grad():
        gn.weight.uniform_(0.5, 1.5)
        gn.bias.uniform_(-0.3, 0.3)
    ctx = NativeContext()
    u = GNRelu(ctx, 'gn', gn)
    ctx.finalize('cpu')
    u.load_from_torch()
    x = torch.randn(2, 5, 6, 32).to(torch.bfloat16)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    ref = torch.relu(gn(xr))
    d = torch.randn_like(ref)
    (ref * d).sum().backward()
    xn = x.clone().requires_grad_()
    z = u(xn)
    assert torch.allclose(z.float().permute(0, 3, 1, 2), ref, atol=3e-2, rtol=2e-2)
    (z.float() * d.permute(0, 2, 3, 1)).sum().backward()
    assert _cos(xn.grad.permute(0, 3, 1, 2), xr.grad) > 0.999
    # (the ReLU mask of a few near-zero outputs differs: the reference runs on fp32 x)
    assert (u.g.grad - gn.weight.grad).norm() < 1e-2 * gn.weight.grad.norm()
    assert (u.b.grad - gn.bias.grad).norm() < 1e-2 * gn.bias.grad.norm()


def _pair(classes, seed):
    torch.manual_seed(seed)
    tm = FPN(encoder_name='resnet18', classes=classes, dropout=0.0)
    with torch.no_grad():
        for m in tm.modules():
            if isinstance(m, (torch.nn.BatchNorm2d, torch.nn.GroupNorm)):
                m.weight.uniform_(0.5, 1.5)
    ref = FPN(encoder_name='resnet18', classes=classes, dropout=0.0)
    ref.load_state_dict(tm.state_dict())
    return tm, ref


def test_native_fpn_matches_torch_autograd():
    tm, ref = _pair(1, 0)
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', lr=1e-3, use_graph=False)
    x = Fn.stem_s2d_to_nhwc(step.x).permute(0, 3, 1, 2).contiguous()
    t = step.t.view(2, 1, 64, 64)
    ref.train()
    loss = BCEDiceLoss()(ref(x), t)
    loss.backward()
    net = step.net
    net.ctx.ws.zero()
    net.arena.zero_grad()
    l_nat = net.loss(step.x, step.t)
    l_nat.backward()
    assert abs(l_nat.item() - loss.item()) / loss.item() < 0.03
    a = net.arena.by_name
    d = ref.decoder
    # the output conv's rows are padded to 8 (zero, with zero gradient)
    assert a['decoder.final_conv.weight'].grad[1:].abs().max() == 0
    assert _cos(a['decoder.final_conv.weight'].grad[:1], d.final_conv.weight.grad) > 0.95
    assert _cos(a['decoder.final_conv.bias'].grad[:1], d.final_conv.bias.grad) > 0.95
    g = a['decoder.heads.3.0.0.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, d.heads[3][0][0].weight.grad) > 0.9
    assert _cos(a['decoder.heads.0.2.1.weight'].grad, d.heads[0][2][1].weight.grad) > 0.9
    g = a['decoder.laterals.2.weight'].grad
    assert _cos(g, d.laterals[2].weight.grad.reshape(g.shape)) > 0.85
    assert _cos(a['decoder.lateral_top.bias'].grad, d.lateral_top.bias.grad) > 0.85
    # bf16 activations through the encoder's BatchNorms on a 2x64x64 batch (see
    # test_linknet_cpu for the torch-autocast comparison)
    g = a['encoder.body.layer3.0.cb1.conv.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, ref.encoder.body.layer3[0].cb1.conv.weight.grad) > 0.55
    losses = []
    for _ in range(4):
        step()
        losses.append(step.last_loss())
    assert losses[-1] < losses[0]


def test_native_fpn_predict_matches_torch_eval():
    tm, ref = _pair(2, 1)
    with torch.no_grad():
        for m in tm.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 1.5)
    ref.load_state_dict(tm.state_dict())
    ref.eval()
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', use_graph=False)
    x = torch.randn(3, 3, 64, 64)
    t = (torch.rand(3, 2, 64, 64) > 0.5).float()
    logits, loss = step.net.predict(Fn.nchw_to_nhwc(x, pad_to=8), t)
    with torch.no_grad():
        want = ref(x.to(torch.bfloat16).float())
    assert logits.shape == want.shape == (3, 2, 64, 64)
    assert _cos(logits, want) > 0.995
    ref_loss = BCEDiceLoss()(logits, t)
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    step.net.export_to_torch()


def test_runner_picks_native_engine_for_fpn():
    from mlcomp_amd.train.runner import _native_kind
    assert _native_kind(FPN(encoder_name='resnet18'), torch.device('cuda')) == 'unet'
