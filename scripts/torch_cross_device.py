"""Stock PyTorch against itself: one bf16-autocast training step of a torch.nn model on the CPU
and on the GPU from the same weights and batch, per-parameter relative gradient error
||g_gpu - g_cpu|| / ||g_cpu||, next to the CPU step's own sensitivity to moving every weight
by one fp32 ulp (x (1 + 2^-24 n)).  NO mlcomp_amd kernels: this is the floor the reference's
own framework sits on for the same comparison that scripts/engines_det_compare.py makes for
the native engines (docs/numerics.md).

    python scripts/torch_cross_device.py [model ...]

Models: resnext50, efficientnet-b0, unet-resnext50 (tests/test_generic_gpu.py definitions),
linknet / fpn (contrib.segmentation, ResNet-34 encoder), resnext50-g1 (ResNeXt-50 with
every BatchNorm weight 1, i.e. without the zero-init of the last BN of each residual branch).
Prints one JSON line per model."""
import copy
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path[:0] = [root, os.path.join(root, 'tests')]
torch.backends.cudnn.deterministic = True
B, R = int(os.environ.get('DET_BATCH', 8)), int(os.environ.get('DET_RES', 128))


def make(name):
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(7)
    if name in ('linknet', 'fpn'):
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet
        m = Linknet(encoder_name='resnet34') if name == 'linknet' else FPN(encoder_name='resnet34', dropout=0.0)
        x = torch.randn(B, 3, R, R, generator=g)
        y = (torch.rand(B, 1, R, R, generator=g) > 0.5).float()
        return m, x, y, nn.BCEWithLogitsLoss()
    from test_generic_gpu import _models, _no_stochastic
    mk, shape, ncls = _models()[name.replace('-g1', '')]
    m = _no_stochastic(mk())
    if name.endswith('-g1'):
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, nn.BatchNorm2d) and mod.weight is not None:
                    mod.weight.fill_(1.0)
    x = torch.randn(*shape, generator=g)
    if ncls is None:
        return m, x, (torch.rand(shape[0], 1, shape[2], shape[3], generator=g) > 0.5).float(), nn.BCEWithLogitsLoss()
    return m, x, torch.randint(0, ncls, (shape[0],), generator=g), nn.CrossEntropyLoss()


def step(m, x, y, crit, dev):
    m = m.to(dev).train()
    m.zero_grad(set_to_none=True)
    with torch.autocast(dev, dtype=torch.bfloat16):
        out = m(x.to(dev))
    if isinstance(out, dict):
        out = out['out']
    loss = crit(out.float(), y.to(dev))
    loss.backward()
    if dev == 'cuda':
        torch.cuda.synchronize()
    return float(loss.detach()), {n: p.grad.detach().float().cpu().flatten() for n, p in m.named_parameters()
                         if p.grad is not None and float(p.grad.norm()) > 0}


def rel(a, b):
    r = {n: float((a[n] - b[n]).norm() / (b[n].norm() + 1e-20)) for n in b if n in a}
    v = sorted(r.values())
    return r, v[len(v) // 2], v[-1]


def main():
    names = sys.argv[1:] or ['resnext50', 'resnext50-g1', 'efficientnet-b0', 'unet-resnext50', 'linknet', 'fpn']
    for name in names:
        m, x, y, crit = make(name)
        base = copy.deepcopy(m)
        l_c, g_c = step(copy.deepcopy(base), x, y, crit, 'cpu')
        l_g, g_g = step(copy.deepcopy(base), x, y, crit, 'cuda')
        per = copy.deepcopy(base)
        gen = torch.Generator().manual_seed(1)
        with torch.no_grad():
            for p in per.parameters():
                p.mul_(1 + 2.0 ** -24 * torch.randn(p.shape, generator=gen))
        l_p, g_p = step(per, x, y, crit, 'cpu')
        _, med, mx = rel(g_g, g_c)
        _, nmed, nmx = rel(g_p, g_c)
        print(json.dumps({'model': name, 'framework': 'stock torch bf16 autocast', 'batch': B, 'slots': len(g_c),
                          'loss_rel_err': abs(l_g - l_c) / abs(l_c), 'gpu_vs_cpu_median': med, 'gpu_vs_cpu_max': mx,
                          'cpu_fp32ulp_noise_median': nmed, 'cpu_fp32ulp_noise_max': nmx}), flush=True)


if __name__ == '__main__':
    main()
