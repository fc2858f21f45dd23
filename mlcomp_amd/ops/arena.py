"""Flat parameter arenas.

All parameters of a native model live in two contiguous fp32 buffers:

* the *decay* arena: matmul weights (conv / linear), kept in kernel layout
  ([Co, KH, KW, Ci] for convs) with a bf16 mirror that the MFMA kernels read;
* the *no-decay* arena: BatchNorm affine parameters and biases.

Each arena owns master, grad and optimizer-state buffers of identical layout, so

* the optimizer is ONE fused kernel per arena (``mlc_sgd`` / ``mlc_adam``), which also
  refreshes the bf16 mirror - no per-step cast or repack pass;
* gradients are produced in place by the backward kernels (wgrad writes straight into
  its slice of the grad arena) and the RCCL bucketer all-reduces contiguous slices of
  it with zero copies (`mlcomp_amd.parallel.ddp`).

Parameters are laid out in *reverse registration order* (registration follows the
forward pass) so gradients become ready front-to-back during backward: bucket 0 fills
first and its all-reduce starts while the rest of backward still runs.
Segments are padded to 64 floats (256 B) so every view is 16-byte aligned.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

_ALIGN = 64


@dataclass
class Slot:
    name: str
    shape: Tuple[int, ...]
    numel: int
    offset: int = 0
    arena: 'Arena' = None
    # frozen: the optimizer skips the slot entirely (no update, no weight decay) - the
    # parameters a model never runs, which torch.optim skips because their grad is None
    frozen: bool = False

    @property
    def master(self) -> torch.Tensor:
        return self.arena.master[self.offset:self.offset + self.numel].view(self.shape)

    @property
    def grad(self) -> torch.Tensor:
        return self.arena.grad[self.offset:self.offset + self.numel].view(self.shape)

    @property
    def bf16(self) -> torch.Tensor:
        return self.arena.mirror[self.offset:self.offset + self.numel].view(self.shape)


class Arena:
    def __init__(self, name: str, mirror: bool, decay: bool):
        self.name = name
        self.want_mirror = mirror
        self.decay = decay
        self.slots: List[Slot] = []
        self.master = self.grad = self.mirror = None
        self.state: Dict[str, torch.Tensor] = {}
        self.numel = 0

    def add(self, name, shape) -> Slot:
        n = 1
        for s in shape:
            n *= int(s)
        slot = Slot(name, tuple(int(s) for s in shape), n, arena=self)
        self.slots.append(slot)
        return slot

    def finalize(self, device):
        off = 0
        for slot in reversed(self.slots):  # reverse forward order == backward order
            slot.offset = off
            off += (slot.numel + _ALIGN - 1) // _ALIGN * _ALIGN
        self.numel = max(off, _ALIGN)
        self.master = torch.zeros(self.numel, device=device, dtype=torch.float32)
        self.grad = torch.zeros(self.numel, device=device, dtype=torch.float32)
        if self.want_mirror:
            self.mirror = torch.zeros(self.numel, device=device, dtype=torch.bfloat16)

    def state_buffer(self, key: str) -> torch.Tensor:
        if key not in self.state:
            self.state[key] = torch.zeros_like(self.master)
        return self.state[key]

    def refresh_mirror(self):
        if self.mirror is not None:
            self.mirror.copy_(self.master.to(torch.bfloat16))

    def slots_in_backward_order(self) -> List[Slot]:
        return sorted(self.slots, key=lambda s: s.offset)

    def segments(self) -> List[Tuple[int, int]]:
        """[start, end) element ranges the optimizer updates: the whole arena, minus the
        (padded) extents of frozen slots, neighbouring live slots merged."""
        if not any(s.frozen for s in self.slots):
            return [(0, self.numel)]
        out: List[Tuple[int, int]] = []
        for s in self.slots_in_backward_order():
            if s.frozen:
                continue
            end = s.offset + (s.numel + _ALIGN - 1) // _ALIGN * _ALIGN
            if out and out[-1][1] == s.offset:
                out[-1] = (out[-1][0], end)
            else:
                out.append((s.offset, end))
        return out


class ParamArena:
    """The pair of arenas of one model."""

    def __init__(self):
        self.decay = Arena('decay', mirror=True, decay=True)
        self.nodecay = Arena('nodecay', mirror=False, decay=False)
        self.by_name: Dict[str, Slot] = {}
        self.device = None
        self.ready_hook = None  # callable(slot) set by the gradient bucketer
        self.flush = None       # callable() joining gradient work still in flight (native layers)
        # streams other than the current one that write gradients without joining per
        # layer (NativeContext.wgrad_defer): a bucket's all-reduce / update waits on them too
        self.grad_streams = []

    def weight(self, name, shape) -> Slot:
        s = self.decay.add(name, shape)
        self.by_name[name] = s
        return s

    def vector(self, name, shape) -> Slot:
        s = self.nodecay.add(name, shape)
        self.by_name[name] = s
        return s

    def finalize(self, device):
        self.device = torch.device(device)
        self.decay.finalize(self.device)
        self.nodecay.finalize(self.device)

    def arenas(self):
        return (self.decay, self.nodecay)

    def mark_ready(self, slot: Slot):
        if self.ready_hook is not None:
            self.ready_hook(slot)

    def zero_grad(self):
        for a in self.arenas():
            a.grad.zero_()

    def num_params(self) -> int:
        return sum(s.numel for a in self.arenas() for s in a.slots)
