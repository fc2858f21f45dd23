"""Training step of the generic native engine (:mod:`mlcomp_amd.models.native_generic`).

Any model the fx lowering accepts: forward through the lowered graph (native sites +
PyTorch tensor ops), the stage's criterion (any torch loss, on fp32 logits), autograd
backward (native sites write weight gradients straight into the grad arena; the bucketer
all-reduces completed buckets on its side stream), one fused optimizer launch per arena
with torch.optim's semantics (weight decay on every parameter), the BN buffer broadcast.
The whole step - including the criterion and autograd's backward - is captured into one
HIP graph after the eager warm-up (:class:`~mlcomp_amd.train.graphed.GraphedStep`).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from mlcomp_amd.models.native_generic import GenericNet
from mlcomp_amd.ops.layers import flatten_bn_buffers
from mlcomp_amd.parallel.comm import make_comm
from mlcomp_amd.parallel.ddp import GradBucketer
from mlcomp_amd.train.graphed import GraphedStep, work_stream
from mlcomp_amd.train.optim import FusedAdam, FusedSGD


class NativeGenericStep(GraphedStep):
    def __init__(self, torch_model, x, y, device=None, world_size=1, use_graph=True,
                 criterion: Optional[Callable] = None, optimizer='SGD', lr=0.1, momentum=0.0, weight_decay=0.0,
                 nesterov=False, dampening=0.0, betas=(0.9, 0.999), eps=1e-8, comm=None, warmup_eager=2, **_):
        self.device = torch.device(device or 'cuda')
        self.net = GenericNet(torch_model, self.device)
        self.world = world_size
        self.comm = comm if comm is not None else (make_comm(self.device) if world_size > 1 else None)
        self.bucketer = GradBucketer(self.net.arena, self.comm)
        self.bn_buffers = flatten_bn_buffers(self.net._units())
        self.bucketer.broadcast_params()
        if optimizer in ('Adam', 'AdamW'):
            self.opt = FusedAdam(self.net.arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                 decoupled=optimizer == 'AdamW', grad_scale=1.0 / world_size, decay_all=True)
        elif optimizer == 'SGD':
            self.opt = FusedSGD(self.net.arena, lr=lr, momentum=momentum, weight_decay=weight_decay,
                                nesterov=nesterov, dampening=dampening, grad_scale=1.0 / world_size, decay_all=True)
        else:
            raise ValueError(f'native optimizers: SGD / Adam / AdamW, not {optimizer!r}')
        self.criterion = criterion if criterion is not None else torch.nn.CrossEntropyLoss()
        # static input buffers (the captured graph reads them; load_batch copies into them)
        self.x = x.detach().to(self.device).clone()
        self.y = y.detach().to(self.device).clone()
        self.batch = int(self.x.shape[0])
        self.use_graph = use_graph and self.device.type == 'cuda'
        self.warmup_eager = warmup_eager
        self.graph = None
        self.calls = 0
        self.out = None
        self._loss = None

    def load_batch(self, x, y):
        self.x.copy_(x.to(self.device, non_blocking=True))
        self.y.copy_(y.to(self.device, non_blocking=True))

    def _body(self):
        self.net.ctx.ws.zero()
        self.net.arena.zero_grad()
        self.bucketer.begin()
        self.net.train()
        out = self.net(self.x)
        loss = self.criterion(out.float() if out.is_floating_point() else out, self.y)
        loss.backward()
        self.bucketer.finish()
        self.opt.step()
        self._end_of_step_buffers()
        self.out = out.detach()
        self._loss = loss.detach()

    def predict(self, x):
        self.net.eval()
        try:
            with torch.no_grad(), work_stream(self.device):
                return self.net(x.to(self.device))
        finally:
            self.net.train()

    def set_lr(self, lr):
        self.opt.set_lr(lr)

    def last_loss(self) -> Optional[float]:
        return None if self._loss is None else float(self._loss.item())


__all__ = ['NativeGenericStep']
