"""Synthetic U-Net segmentation train step (BASELINE config 3: U-Net, ResNet-34 encoder,
1 class, 256x256, batch 32 per GPU, Adam lr 3e-4, BCE + Dice loss).

* ``impl='native'`` - :class:`~mlcomp_amd.train.native_seg_step.NativeSegmentationStep`
  (NHWC bf16, fused conv+BN+ReLU, fused upsample+concat, fused head+BCE+Dice, fused Adam,
  bucketed RCCL all-reduce, HIP graph).
* ``impl='torch'`` - stock PyTorch-ROCm on the same model/data/loss/optimizer:
  channels_last + autocast(bf16), MIOpen convs, torch DDP (the measured baseline).
"""
from __future__ import annotations

from typing import Optional

import torch


class _TorchSegStep:
    def __init__(self, encoder, batch, image_size, device, world_size, arch='unet'):
        from mlcomp_amd.contrib.criterion import BCEDiceLoss
        from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet, Unet
        from mlcomp_amd.train.native_seg_step import synthetic_masks
        if arch == 'deeplab':
            from mlcomp_amd.contrib.segmentation.deeplab import DeepLab
            model = DeepLab(backbone='resnet', num_classes=1)
        else:
            model = {'unet': Unet, 'linknet': Linknet, 'fpn': FPN, 'pspnet': PSPNet}[arch](encoder_name=encoder,
                                                                                          classes=1)
        model = model.to(device=device, memory_format=torch.channels_last)
        self.model = model
        if world_size > 1:
            from torch.nn.parallel import DistributedDataParallel as DDP
            self.model = DDP(model, device_ids=[device.index], gradient_as_bucket_view=True)
        self.opt = torch.optim.Adam(model.parameters(), lr=3e-4, foreach=True)
        self.crit = BCEDiceLoss()
        g = torch.Generator(device=device)
        g.manual_seed(4321)
        self.x = torch.randn(batch, 3, image_size, image_size, device=device,
                             generator=g).contiguous(memory_format=torch.channels_last)
        self.t = synthetic_masks(batch, image_size, device, g)
        self._loss = None

    def __call__(self):
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = self.model(self.x)
        loss = self.crit(out.float(), self.t)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()

    def last_loss(self):
        return None if self._loss is None else float(self._loss.item())


def build_seg_step(encoder: str = 'resnet34', batch: int = 32, impl: str = 'native', image_size: int = 256,
                   device=None, world_size: int = 1, use_graph: Optional[bool] = None, arch: str = 'unet'):
    """``arch``: 'unet' (BASELINE config 3), 'linknet', 'fpn', 'pspnet' (same encoder, data, loss, optimizer) or 'deeplab' (ResNet-101 backbone)."""
    device = device or torch.device('cuda')
    if impl == 'torch':
        return _TorchSegStep(encoder, batch, image_size, device, world_size, arch)
    from mlcomp_amd.train.native_seg_step import NativeSegmentationStep
    return NativeSegmentationStep(encoder, batch=batch, image_size=image_size, device=device,
                                  world_size=world_size, use_graph=(True if use_graph is None else use_graph),
                                  arch=arch)
