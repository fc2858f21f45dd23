"""Throughput of one model on the generic native engine vs stock PyTorch-ROCm.

    python scripts/bench_generic.py --model resnext50_32x4d --batch 64 --size 224 --impl native
    python scripts/bench_generic.py --model unet:resnext50_32x4d --batch 16 --size 256 --impl torch

``--impl native``: :class:`~mlcomp_amd.train.native_generic_step.NativeGenericStep` (HIP graph).
``--impl torch``: the same model with channels_last + bf16 autocast, torch.optim (foreach)
- the stock PyTorch-ROCm path (MIOpen convs, hipBLASLt GEMMs).
Random-init weights, synthetic data; prints one JSON line (img/s, ms/step)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn as nn


VIDEO = {   # the reference's video models (mlcomp/contrib/model/video/resnext3d): ClassyVision-style configs
    'r2plus1d_18': dict(residual_transformation_type='basic_r2plus1d_transformation', stem_name='r2plus1d_stem',
                        num_blocks=(2, 2, 2, 2), stage_planes=64, in_plane=512),
    'resnext3d_18': dict(residual_transformation_type='basic_transformation', num_blocks=(2, 2, 2, 2),
                         stage_planes=64, in_plane=512),
}


def build(name, classes):
    if name.startswith('video:'):
        from mlcomp_amd.contrib.video import ResNeXt3D
        return ResNeXt3D(num_classes=classes, **VIDEO[name.split(':', 1)[1]]), False
    if ':' in name:
        arch, enc = name.split(':')
        from mlcomp_amd.contrib.segmentation import models as S
        from mlcomp_amd.contrib.segmentation.deeplab import DeepLab
        if arch == 'deeplab':
            return DeepLab(backbone=enc, num_classes=classes), True
        return getattr(S, {'unet': 'Unet', 'fpn': 'FPN', 'psp': 'PSPNet', 'linknet': 'Linknet'}[arch])(
            encoder_name=enc, classes=classes), True
    if name == 'ref_cifar_net':
        sys.path.insert(0, 'tests')
        from test_generic_cpu import RefCifarNet
        return RefCifarNet(), False
    from mlcomp_amd.models import build_model
    return build_model(name, num_classes=classes), False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--model', default='resnext50_32x4d')
    ap.add_argument('--batch', type=int, default=64)
    ap.add_argument('--size', type=int, default=224)
    ap.add_argument('--channels', type=int, default=3)
    ap.add_argument('--frames', type=int, default=0, help='video models: clip length (5-D input)')
    ap.add_argument('--classes', type=int, default=1000)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--impl', default='native', choices=['native', 'torch'])
    ap.add_argument('--optimizer', default='SGD')
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device('cuda')
    model, seg = build(a.model, a.classes)
    x = torch.randn(a.batch, a.channels, *((a.frames,) if a.frames else ()), a.size, a.size, device=dev)
    if seg:
        y = torch.randint(0, a.classes, (a.batch, a.size, a.size), device=dev)
    else:
        y = torch.randint(0, a.classes, (a.batch,), device=dev)
    crit = nn.CrossEntropyLoss()
    okw = dict(lr=0.01, momentum=0.9, weight_decay=1e-4) if a.optimizer == 'SGD' else dict(lr=1e-3)
    if a.impl == 'native':
        from mlcomp_amd.train.native_generic_step import NativeGenericStep
        step = NativeGenericStep(model, x, y, device=dev, criterion=crit, optimizer=a.optimizer, **okw)
        run = step
    else:
        model = model.to(dev)
        xc = x
        try:                      # channels_last (MIOpen's NHWC kernels) unless the model's
            with torch.no_grad(), torch.autocast('cuda', dtype=torch.bfloat16):   # views need NCHW
                model.to(memory_format=torch.channels_last)(x.contiguous(memory_format=torch.channels_last))
            xc = x.contiguous(memory_format=torch.channels_last)
        except RuntimeError:
            model = model.to(memory_format=torch.contiguous_format)
        opt = getattr(torch.optim, a.optimizer)(model.parameters(), **okw)

        def run():
            with torch.autocast('cuda', dtype=torch.bfloat16):
                out = model(xc)
            loss = crit(out.float(), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
    for _ in range(a.warmup):
        run()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(a.steps):
        run()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / a.steps
    print(json.dumps({'model': a.model, 'impl': a.impl, 'batch': a.batch, 'size': a.size,
                      'ms_per_step': round(dt * 1e3, 3), 'img_per_s': round(a.batch / dt, 1)}), flush=True)


if __name__ == '__main__':
    main()
