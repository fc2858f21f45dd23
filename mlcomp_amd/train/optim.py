"""Fused optimizers over :class:`~mlcomp_amd.ops.arena.ParamArena`.

One kernel launch per arena per step (`csrc/kernels/optim.hip`).  The learning rate and
gradient scale live in a small device tensor (``hyper``) so a HIP-graph-captured step
picks up LR-schedule changes without re-capture: ``set_lr`` is a tiny H2D copy outside
the graph.
"""
from __future__ import annotations

import torch

from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.arena import ParamArena


class FusedSGD:
    def __init__(self, arena: ParamArena, lr=0.1, momentum=0.9, weight_decay=0.0,
                 nesterov=False, dampening=0.0, grad_scale=1.0):
        self.arena = arena
        self.momentum = momentum
        self.wd = weight_decay
        self.nesterov = nesterov
        self.dampening = dampening
        self.lr = lr
        self.hyper = torch.tensor([lr, grad_scale, 1.0, 1.0], dtype=torch.float32,
                                  device=arena.device)
        self.steps = 0
        for a in arena.arenas():
            a.state_buffer('momentum')

    def set_lr(self, lr):
        self.lr = lr
        self.hyper[0].fill_(lr)

    def set_grad_scale(self, s):
        self.hyper[1].fill_(s)

    def step(self):
        # the first step seeds momentum = grad (torch.optim.SGD semantics); with zeroed
        # buffers "mu*0 + (1-dampening)*g" equals that when dampening == 0, which keeps
        # the kernel arguments identical across steps (HIP-graph friendly).
        for a in self.arena.arenas():
            Fn.sgd_step(a.master, a.grad, a.state['momentum'], a.mirror, self.hyper,
                        a.numel if a.decay else 0, a.numel if a.mirror is not None else 0,
                        self.momentum, self.dampening, self.wd, self.nesterov, False)
        self.steps += 1


class FusedAdam:
    def __init__(self, arena: ParamArena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, decoupled=True, grad_scale=1.0):
        self.arena = arena
        self.b1, self.b2 = betas
        self.eps = eps
        self.wd = weight_decay
        self.decoupled = decoupled
        self.lr = lr
        self.hyper = torch.tensor([lr, grad_scale, 1.0, 1.0], dtype=torch.float32,
                                  device=arena.device)
        self.steps = 0
        for a in arena.arenas():
            a.state_buffer('exp_avg')
            a.state_buffer('exp_avg_sq')

    def set_lr(self, lr):
        self.lr = lr
        self.hyper[0].fill_(lr)

    def set_grad_scale(self, s):
        self.hyper[1].fill_(s)

    def prepare(self):
        """Update the bias corrections for the coming step (outside any graph)."""
        t = self.steps + 1
        self.hyper[2].fill_(1 - self.b1 ** t)
        self.hyper[3].fill_(1 - self.b2 ** t)

    def step(self):
        for a in self.arena.arenas():
            Fn.adam_step(a.master, a.grad, a.state['exp_avg'], a.state['exp_avg_sq'], a.mirror,
                         self.hyper, a.numel if a.decay else 0,
                         a.numel if a.mirror is not None else 0, self.b1, self.b2, self.eps,
                         self.wd, self.decoupled)
        self.steps += 1
