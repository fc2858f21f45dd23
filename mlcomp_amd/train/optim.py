"""Fused optimizers over :class:`~mlcomp_amd.ops.arena.ParamArena`.

One kernel launch per arena per step (`csrc/kernels/optim.hip`).  The learning rate and
gradient scale live in a small device tensor (``hyper``) so a HIP-graph-captured step
picks up LR-schedule changes without re-capture: ``set_lr`` is a tiny H2D copy outside
the graph.

Step counting is host work: ``prepare()`` runs once per training step on the host
(outside any captured graph) and advances ``steps``; ``step()`` only enqueues the update
kernels, so a graph that captured ``step()`` once and is replayed N times still sees N
distinct bias corrections.
"""
from __future__ import annotations

import torch

from mlcomp_amd.ops import functional as Fn
from mlcomp_amd.ops.arena import ParamArena


class _ArenaStateMixin:
    def _slice(self, a, start, end):
        """views of one contiguous slice of an arena: (master, grad, mirror, n, ndecay, nbf)"""
        n = end - start
        mirror = a.mirror[start:end] if a.mirror is not None else None
        decay = a.decay or getattr(self, 'decay_all', False)
        return a.master[start:end], a.grad[start:end], mirror, n, n if decay else 0, n if mirror is not None else 0

    """Checkpointable optimizer state: the step counter and every arena state buffer
    (momentum / Adam moments) as CPU tensors, keyed ``<arena>.<buffer>``."""

    def state_dict(self) -> dict:
        bufs = {f'{a.name}.{k}': v.detach().cpu() for a in self.arena.arenas() for k, v in a.state.items()}
        return {'steps': int(self.steps), 'buffers': bufs}

    def load_state_dict(self, d: dict):
        self.steps = int(d.get('steps', 0))
        for a in self.arena.arenas():
            for k, v in a.state.items():
                src = d.get('buffers', {}).get(f'{a.name}.{k}')
                if src is not None and src.numel() == v.numel():
                    v.copy_(src.to(v.device))


class FusedSGD(_ArenaStateMixin):
    def __init__(self, arena: ParamArena, lr=0.1, momentum=0.9, weight_decay=0.0,
                 nesterov=False, dampening=0.0, grad_scale=1.0, decay_all=False):
        self.arena = arena
        # decay_all: weight decay on every parameter (torch.optim's semantics, the generic
        # engine); otherwise only the decay arena (matmul weights; the hand-lowered engines)
        self.decay_all = decay_all
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

    def prepare(self):
        """Host side of one step (call once per step, outside any graph)."""
        self.steps += 1

    def step(self):
        # the first step seeds momentum = grad (torch.optim.SGD semantics); with zeroed
        # buffers "mu*0 + (1-dampening)*g" equals that when dampening == 0, which keeps
        # the kernel arguments identical across steps (HIP-graph friendly).
        for a in self.arena.arenas():
            segs = a.segments()
            if segs != [(0, a.numel)]:       # frozen slots: update the live ranges only
                for s, e in segs:
                    self.step_slice(a, s, e)
                continue
            Fn.sgd_step(a.master, a.grad, a.state['momentum'], a.mirror, self.hyper,
                        a.numel if (a.decay or self.decay_all) else 0, a.numel if a.mirror is not None else 0,
                        self.momentum, self.dampening, self.wd, self.nesterov, False)

    def step_slice(self, a, start, end):
        """The update of elements [start, end) of arena ``a`` (one gradient bucket)."""
        p, g, bf, n, nd, nb = self._slice(a, start, end)
        Fn.sgd_step(p, g, a.state['momentum'][start:end], bf, self.hyper, nd, nb, self.momentum, self.dampening,
                    self.wd, self.nesterov, False)


class FusedAdam(_ArenaStateMixin):
    def __init__(self, arena: ParamArena, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, decoupled=True, grad_scale=1.0, decay_all=False):
        self.arena = arena
        self.decay_all = decay_all
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
        """Advance the step counter and write the bias corrections of the coming step
        into ``hyper`` (a host->device fill, outside any graph)."""
        self.steps += 1
        t = self.steps
        self.hyper[2].fill_(1 - self.b1 ** t)
        self.hyper[3].fill_(1 - self.b2 ** t)

    def step(self):
        for a in self.arena.arenas():
            segs = a.segments()
            if segs != [(0, a.numel)]:       # frozen slots: update the live ranges only
                for s, e in segs:
                    self.step_slice(a, s, e)
                continue
            Fn.adam_step(a.master, a.grad, a.state['exp_avg'], a.state['exp_avg_sq'], a.mirror,
                         self.hyper, a.numel if (a.decay or self.decay_all) else 0,
                         a.numel if a.mirror is not None else 0, self.b1, self.b2, self.eps,
                         self.wd, self.decoupled)

    def step_slice(self, a, start, end):
        """The update of elements [start, end) of arena ``a`` (one gradient bucket)."""
        p, g, bf, n, nd, nb = self._slice(a, start, end)
        Fn.adam_step(p, g, a.state['exp_avg'][start:end], a.state['exp_avg_sq'][start:end], bf, self.hyper, nd, nb,
                     self.b1, self.b2, self.eps, self.wd, self.decoupled)
