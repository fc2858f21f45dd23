"""The native training step for image classifiers (the headline ResNet-50 task).

forward (fused conv+BN+ReLU nodes) -> fused avgpool/FC/softmax-CE -> backward (wgrad
straight into the flat grad arena, bucketed RCCL all-reduce on a side stream as buckets
fill) -> one fused SGD launch per arena (also refreshing the bf16 weight mirror).

After ``warmup_eager`` eager iterations the whole step is captured into ONE HIP graph
(``torch.cuda.CUDAGraph``; HIP graph on ROCm) and replayed: ~400 kernel launches per
step cost one graph launch.  Inputs are static device buffers; ``load_batch`` copies a
new batch into them (outside the graph) for real-data training.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from mlcomp_amd.models import build_model
from mlcomp_amd.models.native_resnet import STEM_CIN, NativeResNet
from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.layers import flatten_bn_buffers
from mlcomp_amd.parallel.comm import make_comm
from mlcomp_amd.parallel.ddp import GradBucketer
from mlcomp_amd.train.graphed import GraphedStep
from mlcomp_amd.train.optim import FusedAdam, FusedSGD


class NativeClassifierStep(GraphedStep):
    def __init__(self, model_name='resnet50', batch=256, image_size=224, device=None,
                 world_size=1, use_graph=True, num_classes=1000, lr=0.1, momentum=0.9,
                 weight_decay=5e-5, nesterov=False, smoothing=0.0, seed=0, warmup_eager=2,
                 torch_model=None, optimizer='SGD', betas=(0.9, 0.999), eps=1e-8,
                 comm=None, dampening=0.0):
        self.device = torch.device(device or 'cuda')
        torch.manual_seed(seed)
        tm = torch_model if torch_model is not None else build_model(model_name, num_classes=num_classes)
        self.net = NativeResNet(tm, self.device, smoothing=smoothing)
        self.net.ctx.grad_prezeroed = True
        self.world = world_size
        # comm: an explicit communicator (tests inject a 1-rank RCCL one to exercise
        # bucketed all-reduce inside graph capture on a single GPU)
        self.comm = comm if comm is not None else (make_comm(self.device) if world_size > 1 else None)
        self.bucketer = GradBucketer(self.net.arena, self.comm)
        self.bn_buffers = flatten_bn_buffers(self.net._units())
        self.bucketer.broadcast_params()
        if optimizer in ('Adam', 'AdamW'):
            self.opt = FusedAdam(self.net.arena, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                 decoupled=optimizer == 'AdamW', grad_scale=1.0 / world_size)
        else:
            if optimizer != 'SGD':
                raise ValueError(f'native optimizers: SGD / Adam / AdamW, not {optimizer!r}')
            self.opt = FusedSGD(self.net.arena, lr=lr, momentum=momentum, weight_decay=weight_decay,
                                nesterov=nesterov, dampening=dampening, grad_scale=1.0 / world_size)
        # optimizer-in-backward (MLC_OPT_IN_BWD=1): each gradient bucket is updated on the side
        # stream as soon as it is complete (and all-reduced).  Measured slower on MI355X
        # (profiles/round2_ab): the memory-bound update competes with the memory-bound
        # backward passes, so the default is one update launch per arena after backward.
        self.opt_in_bwd = os.environ.get('MLC_OPT_IN_BWD', '0') == '1'
        if self.opt_in_bwd:
            self.bucketer.attach_optimizer(self.opt)
        self.batch = batch
        rank = int(os.environ.get('RANK', '0'))
        g = torch.Generator(device=self.device)
        g.manual_seed(1234 + rank)
        img = torch.randn(batch, image_size, image_size, 3, device=self.device, generator=g)
        self.x = self._prep(torch.nn.functional.pad(img, (0, STEM_CIN - 3)).to(torch.bfloat16).contiguous())
        self.y = torch.randint(0, num_classes, (batch,), device=self.device, generator=g)
        self.use_graph = use_graph and self.device.type == 'cuda'
        self.warmup_eager = warmup_eager
        self.graph = None
        self.calls = 0
        self._loss = None

    # ------------------------------------------------------------------ data
    def load_batch(self, images_nchw_or_nhwc: torch.Tensor, labels: torch.Tensor):
        """Copy a batch into the static input buffers (NCHW float or NHWC bf16)."""
        x = images_nchw_or_nhwc
        if x.dim() == 4 and x.shape[1] in (1, 3) and x.dtype != torch.bfloat16:
            x = Fn.nchw_to_nhwc(x.to(self.device, non_blocking=True).float(), pad_to=STEM_CIN)
        self.x.copy_(self._prep(x.to(self.device, non_blocking=True)))
        self.y.copy_(labels.to(self.device, non_blocking=True))

    def _prep(self, x_nhwc):
        """Input-pipeline layout of the stem: the space-to-depth image when the stem runs as
        a 4x4 conv over it (done here, once per batch, not inside the captured step)."""
        if getattr(self.net.stem, 's2d', False) and x_nhwc.shape[-1] != 16:
            return Fn.stem_s2d(x_nhwc, 3)
        return x_nhwc

    # ------------------------------------------------------------------ step
    def _body(self):
        # the workspace and both gradient arenas in one launch; wgrad kernels then accumulate
        Fn.zero_many([self.net.ctx.ws.buf] + [a.grad for a in self.net.arena.arenas()])
        self.bucketer.begin()
        loss = self.net.loss(self.x, self.y)
        if getattr(self, '_one', None) is None or self._one.device != loss.device:
            self._one = torch.ones_like(loss)        # the backward seed, made once (not per step)
        loss.backward(self._one)
        self.bucketer.finish()
        if not self.opt_in_bwd:
            self.opt.step()
        self._end_of_step_buffers()
        self._loss = self.net.head.loss_sum()

    def set_lr(self, lr):
        self.opt.set_lr(lr)

    def last_loss(self) -> Optional[float]:
        if self._loss is None:
            return None
        return float(self._loss.item()) / self.batch

    def accuracy(self) -> float:
        return float(self.net.head.correct().item()) / self.batch
