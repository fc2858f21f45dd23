"""LR schedulers referenced by name from ``scheduler_params.scheduler``
(`mlcomp/contrib/catalyst/optim/cosineanneal.py`)."""
from __future__ import annotations

import math

from torch.optim.lr_scheduler import LRScheduler


class OneCycleCosineAnnealLR(LRScheduler):
    """Cosine annealing from the base LR to ``eta_min`` over ``T_max`` steps, then a
    warm restart at the base LR - repeated every ``T_max`` steps (closed form, so
    resuming from ``last_epoch`` reproduces the schedule exactly)."""

    def __init__(self, optimizer, T_max: int, eta_min: float = 0.0, last_epoch: int = -1):
        self.T_max, self.eta_min = max(1, int(T_max)), eta_min
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        t = self.last_epoch % self.T_max
        f = 0.5 * (1 + math.cos(math.pi * t / self.T_max))
        return [self.eta_min + (b - self.eta_min) * f for b in self.base_lrs]

    _get_closed_form_lr = get_lr


class WarmupCosineLR(LRScheduler):
    """Linear warm-up for ``warmup`` steps then cosine decay to ``eta_min`` at ``total``."""

    def __init__(self, optimizer, total: int, warmup: int = 0, eta_min: float = 0.0, last_epoch: int = -1):
        self.total, self.warmup, self.eta_min = max(1, int(total)), int(warmup), eta_min
        super().__init__(optimizer, last_epoch)

    def get_lr(self):
        t = self.last_epoch
        if t < self.warmup:
            return [b * (t + 1) / self.warmup for b in self.base_lrs]
        p = min(1.0, (t - self.warmup) / max(1, self.total - self.warmup))
        return [self.eta_min + (b - self.eta_min) * 0.5 * (1 + math.cos(math.pi * p)) for b in self.base_lrs]


__all__ = ['OneCycleCosineAnnealLR', 'WarmupCosineLR']
