"""Every hand-lowered native engine (ResNet, U-Net, LinkNet, FPN, PSPNet, DeepLab, BERT):
one step of the GPU kernels against the CPU path of the same native ops - same weights, same
batch, same bf16 rounding points, fp32 accumulation in both.

Bitwise agreement is impossible (fp32 summation order differs) and a deep ReLU / max-pool
network turns one-ulp differences into flipped masks that move whole gradients, so the
anchor is measured per engine: the CPU step run again with every weight perturbed by about
one bf16 ulp (x (1 + 2^-9 n)).  The GPU must be no further from the CPU step than that
perturbation moves it - loss, mean gradient direction over the parameter slots, and no
slot whose gradient error exceeds 3 x its perturbation error + 5e-2 (a wrong kernel for one
layer shows up there even when the means agree)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _make(kind, device):
    torch.manual_seed(0)
    if kind == 'resnet50':
        from mlcomp_amd.train.native_step import NativeClassifierStep
        return NativeClassifierStep('resnet50', batch=8, image_size=64, device=device, num_classes=10,
                                    use_graph=False, lr=0.0, momentum=0.0, weight_decay=0.0)
    from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
    if kind == 'unet':
        return NativeSegmentationStep('resnet34', batch=2, image_size=64, device=device, use_graph=False, lr=0.0)
    if kind in ('linknet', 'fpn', 'pspnet', 'deeplab'):
        from mlcomp_amd.contrib.segmentation.deeplab import DeepLab
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet
        tm = (Linknet(encoder_name='resnet34') if kind == 'linknet' else
              FPN(encoder_name='resnet34', dropout=0.0) if kind == 'fpn' else
              PSPNet(encoder_name='resnet34', classes=1, dropout=0.0) if kind == 'pspnet' else
              DeepLab(backbone='resnet', num_classes=1))
        for m in tm.modules():
            if isinstance(m, (torch.nn.Dropout, torch.nn.Dropout2d)):
                m.p = 0.0
        return NativeSegmentationStep(torch_model=tm, batch=2, image_size=64, device=device, use_graph=False,
                                      lr=0.0)
    from mlcomp_amd.train.native_bert_step import NativeBertStep
    return NativeBertStep('bert-base', batch=4, seq_len=32, device=device, use_graph=False, lr=0.0, dropout=0.0)


_INPUTS = ('x', 'y', 't', 'ids', 'tt', 'key_bias')


def _copy_inputs(dst, src):
    for name in _INPUTS:
        a, b = getattr(dst, name, None), getattr(src, name, None)
        if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            a.copy_(b.to(a.device))


def _grads(step):
    step()
    if step.device.type == 'cuda':
        torch.cuda.synchronize()
    out = {}
    for name, slot in step.net.arena.by_name.items():
        g = slot.grad.detach().float().cpu().flatten()
        if float(g.norm()) > 0:
            out[name] = g.clone()
    return step.last_loss(), out


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-20))


def _cos(a, b):
    return float(a @ b / (a.norm() * b.norm() + 1e-20))


@pytest.mark.parametrize('kind', ['resnet50', 'unet', 'linknet', 'fpn', 'pspnet', 'deeplab', 'bert'])
def test_native_engine_gpu_step_matches_cpu_within_bf16_noise(kind):
    cpu = _make(kind, 'cpu')
    per = _make(kind, 'cpu')
    gpu = _make(kind, DEV)
    _copy_inputs(per, cpu)
    _copy_inputs(gpu, cpu)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for a in per.net.arena.arenas():
            a.master.mul_(1 + 2 ** -9 * torch.randn(a.master.shape, generator=g))
        per.net.arena.decay.refresh_mirror()
    l_c, g_c = _grads(cpu)
    l_p, g_p = _grads(per)
    l_g, g_g = _grads(gpu)
    assert set(g_g) == set(g_c) and len(g_c) > 5, (kind, sorted(set(g_c) ^ set(g_g))[:5])
    noise_l, err_l = abs(l_p - l_c) / abs(l_c), abs(l_g - l_c) / abs(l_c)
    assert err_l <= max(1e-2, 2 * noise_l), (kind, l_g, l_c, l_p)
    cos_n = sum(_cos(g_p[n], g_c[n]) for n in g_c) / len(g_c)
    cos_g = sum(_cos(g_g[n], g_c[n]) for n in g_c) / len(g_c)
    assert cos_g >= cos_n - 0.02, (kind, cos_g, cos_n)
    rn = {n: _rel(g_p[n], g_c[n]) for n in g_c}
    rg = {n: _rel(g_g[n], g_c[n]) for n in g_c}
    bad = {n: (round(rg[n], 4), round(rn[n], 4)) for n in g_c if rg[n] > 3 * rn[n] + 5e-2}
    assert not bad, (kind, bad)
    med = sorted(rg.values())[len(rg) // 2]
    med_n = sorted(rn.values())[len(rn) // 2]
    print(f'{kind}: {len(g_c)} slots, loss err {err_l:.2e} (noise {noise_l:.2e}), grad cos {cos_g:.4f} '
          f'(noise {cos_n:.4f}), median grad rel {med:.4f} (noise {med_n:.4f})')
