"""Benchmark / DAG train steps for models that have no hand-lowered engine (the
``transformer-*`` text classifiers and ``vit-*`` models of :mod:`mlcomp_amd.models.transformers`,
or any registered model): the generic native engine
(:class:`~mlcomp_amd.train.native_generic_step.NativeGenericStep`, torch.fx lowering onto the
framework's kernels) and the stock PyTorch-ROCm comparison (autocast bf16, fused AdamW,
torch DDP).  Same model, synthetic data, loss and optimizer on both."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from mlcomp_amd.models import build_model


def is_text(model_name: str) -> bool:
    return model_name.startswith('transformer-')


def synthetic_batch(model, model_name, batch, seq_len, image_size, num_classes, device, seed=1234):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    if is_text(model_name):
        vocab = model.word.num_embeddings
        x = torch.randint(1, vocab, (batch, seq_len), device=device, generator=g)
    else:
        x = torch.randn(batch, 3, image_size, image_size, device=device, generator=g)
    y = torch.randint(0, num_classes, (batch,), device=device, generator=g)
    return x, y


class _TorchStep:
    def __init__(self, model, x, y, device, world_size, lr, weight_decay):
        self.model = model.to(device)
        self.net = self.model
        if world_size > 1:
            from torch.nn.parallel import DistributedDataParallel as DDP
            self.net = DDP(self.model, device_ids=[device.index], gradient_as_bucket_view=True)
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr, weight_decay=weight_decay, fused=True)
        self.x, self.y = x, y
        self._loss = None

    def __call__(self):
        with torch.autocast('cuda', dtype=torch.bfloat16):
            out = self.net(self.x)
        loss = F.cross_entropy(out.float(), self.y)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        self._loss = loss.detach()

    def last_loss(self):
        return None if self._loss is None else float(self._loss.item())


def build_generic_step(model_name: str, batch: int, seq_len: int = 128, image_size: int = 224, impl='native',
                       device=None, world_size: int = 1, use_graph: Optional[bool] = None, num_classes=None,
                       comm=None, lr=None, weight_decay=0.01):
    """AdamW (lr 2e-5 for text, 1e-3 for images; weight decay 0.01) on synthetic data."""
    device = device or torch.device('cuda')
    torch.manual_seed(0)
    text = is_text(model_name)
    if num_classes is None:
        num_classes = 2 if text else 1000
    kw = dict(num_classes=num_classes)
    if not text and model_name.startswith('vit'):
        kw['image_size'] = image_size
    model = build_model(model_name, **kw)
    lr = lr if lr is not None else (2e-5 if text else 1e-3)
    x, y = synthetic_batch(model, model_name, batch, seq_len, image_size, num_classes, device)
    if impl == 'torch':
        return _TorchStep(model, x, y, device, world_size, lr, weight_decay)
    from .native_generic_step import NativeGenericStep
    return NativeGenericStep(model, x, y, device=device, world_size=world_size,
                             use_graph=True if use_graph is None else use_graph, optimizer='AdamW', lr=lr,
                             weight_decay=weight_decay, comm=comm)


__all__ = ['build_generic_step', 'is_text']
