"""Synthetic ImageNet-shape classification train step (the headline DAG train task).

Two implementations of the SAME step (model, data shape, loss, optimizer):

* ``impl='native'`` - the mlcomp_amd engine: NHWC bf16 activations, fp32 master
  weights, HIP kernels (`mlcomp_amd.ops`) for conv / BN(+ReLU+residual) / pooling /
  softmax-CE / fused SGD, gradient all-reduce by `mlcomp_amd.parallel.ddp.GradBucketer`
  on a side stream overlapped with backward, optional HIP-graph capture of the step.
* ``impl='torch'`` - stock PyTorch-ROCm: channels_last + autocast(bf16), MIOpen convs,
  torch DDP.  This is the measured comparison baseline.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from mlcomp_amd.models import build_model


class _TorchStep:
    def __init__(self, model_name, batch, image_size, device, world_size, num_classes=1000, precision='bf16'):
        # precision 'fp32': no autocast - what a reference config with the Catalyst default
        # precision (fp32) runs when it lands on the torch engine
        self.amp = precision != 'fp32'
        model = build_model(model_name, num_classes=num_classes)
        model = model.to(device=device, memory_format=torch.channels_last)
        self.model = model
        if world_size > 1:
            from torch.nn.parallel import DistributedDataParallel as DDP
            self.model = DDP(model, device_ids=[device.index], gradient_as_bucket_view=True)
        self.opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9,
                                   weight_decay=5e-5, foreach=True)
        g = torch.Generator(device=device)
        g.manual_seed(1234)
        self.x = torch.randn(batch, 3, image_size, image_size, device=device,
                             generator=g).contiguous(memory_format=torch.channels_last)
        self.y = torch.randint(0, num_classes, (batch,), device=device, generator=g)
        self._loss = None

    def __call__(self):
        with torch.autocast('cuda', dtype=torch.bfloat16, enabled=self.amp):
            out = self.model(self.x)
            loss = F.cross_entropy(out.float(), self.y)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()

    def last_loss(self):
        return None if self._loss is None else float(self._loss.item())


def build_train_step(model_name: str = 'resnet50', batch: int = 256, impl: str = 'native',
                     image_size: int = 224, device=None, world_size: int = 1,
                     use_graph: Optional[bool] = None, num_classes: int = 1000, comm=None,
                     precision: str = 'bf16'):
    device = device or torch.device('cuda')
    if impl == 'torch':
        return _TorchStep(model_name, batch, image_size, device, world_size, num_classes, precision)
    from mlcomp_amd.train.native_step import NativeClassifierStep
    return NativeClassifierStep(model_name, batch=batch, image_size=image_size,
                                device=device, world_size=world_size,
                                use_graph=(True if use_graph is None else use_graph),
                                num_classes=num_classes, comm=comm)
