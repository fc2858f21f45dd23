"""Native PSPNet (ResNet encoder; pyramid-level 1x1 convs as native ConvBN / bias GEMMs,
native bilinear upsampling, fusion ConvBN, 3x3 output conv with bias) against plain PyTorch
autograd of the same model, on CPU (reference op paths).  Reference model:
`mlcomp/contrib/segmentation/pspnet/`."""
import torch

from mlcomp_amd.contrib.criterion import BCEDiceLoss
from mlcomp_amd.contrib.segmentation.models import PSPNet
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.train.native_seg_step import NativeSegmentationStep


def _cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return (a @ b / (a.norm() * b.norm() + 1e-12)).item()


def _pair(classes, seed):
    torch.manual_seed(seed)
    tm = PSPNet(encoder_name='resnet18', classes=classes, dropout=0.0)
    with torch.no_grad():
        for m in tm.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
    ref = PSPNet(encoder_name='resnet18', classes=classes, dropout=0.0)
    ref.load_state_dict(tm.state_dict())
    return tm, ref


def test_native_pspnet_matches_torch_autograd():
    tm, ref = _pair(1, 0)
    step = NativeSegmentationStep(torch_model=tm, batch=4, image_size=64, device='cpu', lr=1e-3, use_graph=False)
    x = Fn.stem_s2d_to_nhwc(step.x).permute(0, 3, 1, 2).contiguous()
    t = step.t.view(4, 1, 64, 64)
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
    g = a['decoder.final_conv.weight'].grad
    assert g[1:].abs().max() == 0                       # output channels padded to 8
    assert _cos(g[:1].permute(0, 3, 1, 2), d.final_conv.weight.grad) > 0.95
    assert _cos(a['decoder.final_conv.bias'].grad[:1], d.final_conv.bias.grad) > 0.99
    g = a['decoder.conv.conv.weight'].grad
    assert _cos(g.permute(0, 3, 1, 2), d.conv[0].weight.grad) > 0.9
    assert _cos(a['decoder.conv.bn.weight'].grad, d.conv[1].weight.grad) > 0.9
    g = a['decoder.psp.stages.0.1.0.weight'].grad                     # the no-BN 1x1 level
    assert _cos(g, d.psp.stages[0][1][0].weight.grad.reshape(g.shape)) > 0.8
    g = a['decoder.psp.stages.3.1.conv.weight'].grad
    assert _cos(g.permute(0, 3, 1, 2), d.psp.stages[3][1][0].weight.grad) > 0.8
    g = a['encoder.body.layer2.0.cb1.conv.weight'].grad.permute(0, 3, 1, 2)
    assert _cos(g, ref.encoder.body.layer2[0].cb1.conv.weight.grad) > 0.7
    # stages below the decoder's level get no gradient (as in the reference)
    assert a['encoder.body.layer4.0.cb1.conv.weight'].grad.abs().max() == 0
    losses = []
    for _ in range(4):
        step()
        losses.append(step.last_loss())
    assert all(v == v for v in losses)


def test_native_pspnet_predict_matches_torch_eval():
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
    assert abs(loss.item() - BCEDiceLoss()(logits, t).item()) < 1e-4
    step.net.export_to_torch()


def test_runner_picks_native_engine_for_pspnet():
    from mlcomp_amd.train.runner import _native_kind
    assert _native_kind(PSPNet(encoder_name='resnet18', classes=1), torch.device('cuda')) == 'unet'
    assert _native_kind(PSPNet(encoder_name='resnet18'), torch.device('cuda')) == 'generic'   # 21-class softmax


def test_native_pspnet_unused_stages_frozen_under_weight_decay():
    """The encoder stages past the decoder level never run: with weight_decay > 0 the fused
    optimizer must leave them bitwise unchanged (torch.optim skips grad-None parameters),
    while the used layers do move (ADVICE r3 / VERDICT r3 item 5)."""
    tm, _ = _pair(1, 1)
    step = NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device='cpu', lr=1e-2,
                                  optimizer='AdamW', weight_decay=0.1, use_graph=False)
    a = step.net.arena.by_name
    frozen = [k for k, s in a.items() if s.frozen]
    assert frozen and all(k.startswith(('encoder.body.layer4', 'encoder.body.layer3')) for k in frozen), frozen
    before = {k: a[k].master.clone() for k in a}
    step()
    for k in frozen:
        assert torch.equal(a[k].master, before[k]), k
    moved = [k for k in a if not a[k].frozen and not torch.equal(a[k].master, before[k])]
    assert 'encoder.body.layer1.0.cb1.conv.weight' in moved and 'decoder.conv.conv.weight' in moved
