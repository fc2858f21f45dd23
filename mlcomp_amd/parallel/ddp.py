"""Bucketed gradient all-reduce overlapped with backward (the native DDP).

Replaces the DDP that the reference inherits from Catalyst/PyTorch
(`mlcomp/worker/executors/catalyst_/catalyst_.py:214-236` only calls
``init_process_group('nccl')``; bucketing happens inside torch DDP).  Design points for
MI355X:

* Gradients already live in one flat fp32 arena, laid out in backward order
  (`mlcomp_amd.ops.arena`).  A bucket is a contiguous slice of it, so an all-reduce is
  issued on the slice itself - no flatten/unflatten copies.
* Native layers call ``arena.mark_ready(slot)`` once a gradient is written and nothing
  later in backward reads the weight; when the last slot of a bucket is ready the bucket
  is all-reduced on a dedicated side stream (event fence from the compute stream),
  overlapping the rest of backward, and (``attach_optimizer``) its fused optimizer
  update follows on the same stream - so on one GPU too the optimizer pass overlaps
  backward instead of running after it.
* Bucket size: an 8-GPU ring all-reduce moves 2*(7/8)*S per GPU over point-to-point
  xGMI (7 links x ~153 GB/s); with RCCL using several channels the per-peer chunk
  (S/8) should stay >= ~1-4 MB to amortise latency, hence 32 MB buckets, a smaller
  first bucket (8 MB) so communication starts early in backward, and a final bucket
  capped at 4 MB (``MLC_LAST_BUCKET_MB``): it holds the first layers' gradients, which
  are ready only when backward ends, so its all-reduce is the exposed tail of the step.
* The collectives are stream work of the framework's own RCCL communicator, so the
  whole step (forward, backward, all-reduces, optimizer) is captured in one HIP graph.
* Bucket assignment is a pure function of the arena layout, hence identical on every
  rank (deterministic ordering is required for collectives to match up).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from mlcomp_amd.ops.arena import Arena, ParamArena, Slot


class Bucket:
    def __init__(self, arena: Arena, start: int, end: int, slots: List[Slot]):
        self.arena = arena
        self.start, self.end = start, end
        self.slots = slots
        self.pending = len(slots)
        self.launched = False

    @property
    def view(self) -> torch.Tensor:
        return self.arena.grad[self.start:self.end]

    @property
    def nbytes(self) -> int:
        return (self.end - self.start) * 4


def plan_buckets(arena: Arena, bucket_bytes: int, first_bucket_bytes: int,
                 last_bucket_bytes: Optional[int] = None) -> List[Bucket]:
    """Contiguous arena slices in backward order: a small first bucket (communication
    starts early in backward), ``bucket_bytes`` buckets, and - when ``last_bucket_bytes``
    is given - a final bucket of at most that size.  The final bucket is the only one whose
    all-reduce cannot overlap backward (its last gradient is the network's first layer), so
    keeping it small keeps the exposed tail short."""
    slots = arena.slots_in_backward_order()
    if not slots:
        return []
    ends = [slots[i + 1].offset if i + 1 < len(slots) else arena.numel for i in range(len(slots))]
    tail_from = len(slots)   # index of the first slot of the capped final bucket
    if last_bucket_bytes:
        j = len(slots) - 1
        while j > 0 and (arena.numel - slots[j - 1].offset) * 4 <= last_bucket_bytes:
            j -= 1
        tail_from = j if j > 0 else len(slots)
    buckets = []
    cur: List[Slot] = []
    start = 0
    limit = first_bucket_bytes
    for i, s in enumerate(slots[:tail_from]):
        cur.append(s)
        end = ends[i]
        if (end - start) * 4 >= limit or i + 1 == tail_from:
            buckets.append(Bucket(arena, start, end, cur))
            cur, start, limit = [], end, bucket_bytes
    if tail_from < len(slots):
        buckets.append(Bucket(arena, slots[tail_from].offset, arena.numel, slots[tail_from:]))
    return buckets


class GradBucketer:
    def __init__(self, params: ParamArena, comm, bucket_mb: Optional[float] = None,
                 first_bucket_mb: Optional[float] = None):
        self.params = params
        self.comm = comm
        bmb = bucket_mb or float(os.environ.get('MLC_BUCKET_MB', 32))
        fmb = first_bucket_mb or float(os.environ.get('MLC_FIRST_BUCKET_MB', 8))
        lmb = float(os.environ.get('MLC_LAST_BUCKET_MB', 4))
        self.buckets: List[Bucket] = plan_buckets(params.decay, int(bmb * 2 ** 20),
                                                  int(fmb * 2 ** 20), int(lmb * 2 ** 20) if lmb > 0 else None)
        # BN affine + biases: small, reduced as one trailing bucket
        self.buckets += plan_buckets(params.nodecay, 1 << 62, 1 << 62)
        self.slot_bucket: Dict[int, Bucket] = {}
        for b in self.buckets:
            for s in b.slots:
                self.slot_bucket[id(s)] = b
        self.is_cuda = params.device.type == 'cuda'
        self.side = torch.cuda.Stream(params.device) if self.is_cuda else None
        self.opt = None
        # debug / test mode: run each bucket's work on the compute stream at the moment the
        # bucket completes, so a weight read after its slot was marked ready shows up as a
        # numeric difference instead of a timing-dependent race
        self.sync = os.environ.get('MLC_BUCKET_SYNC', '0') == '1'
        params.ready_hook = self._ready

    def attach_optimizer(self, opt):
        """Optimizer-in-backward: each bucket's fused update (``opt.step_slice``) follows
        its all-reduce on the side stream, overlapping the rest of backward; the step then
        needs no optimizer launch of its own (``opt.step()`` must not be called)."""
        self.opt = opt

    def begin(self):
        for b in self.buckets:
            b.pending = len(b.slots)
            b.launched = False

    # the bucket collective's reduction: 'sum' (the optimizer applies 1/world); the
    # one-GPU overlap evidence (bench.py --comm rccl1) sets 'avg', because RCCL skips an
    # in-place one-rank SUM entirely but runs its device kernel for AVG
    op = 'sum'

    def _work(self, b: Bucket, stream=None):
        if self.comm is not None:
            self.comm.all_reduce(b.view, self.op, stream=stream)
        if self.opt is not None:
            self.opt.step_slice(b.arena, b.start, b.end)

    def _launch(self, b: Bucket):
        b.launched = True
        if self.comm is None and self.opt is None:
            return
        if self.is_cuda and not self.sync:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.params.device))
            self.side.wait_event(ev)
            # gradients written on streams that are not joined per layer (deferred weight
            # gradients): everything they issued so far covers this bucket's slots
            for s in getattr(self.params, 'grad_streams', ()):
                e2 = torch.cuda.Event()
                e2.record(s)
                self.side.wait_event(e2)
            with torch.cuda.stream(self.side):
                self._work(b, self.side)
        else:
            self._work(b)

    def _ready(self, slot: Slot):
        b = self.slot_bucket.get(id(slot))
        if b is None:
            return
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self._launch(b)

    def finish(self):
        """Launch buckets whose params got no gradient this step, then make the compute
        stream wait for every all-reduce."""
        if getattr(self.params, 'flush', None) is not None:
            self.params.flush()      # lagged weight gradients (MLC_WGRAD_LAG) are complete
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        if self.is_cuda and (self.comm is not None or self.opt is not None) and not self.sync:
            ev = torch.cuda.Event()
            ev.record(self.side)
            torch.cuda.current_stream(self.params.device).wait_event(ev)

    def broadcast_params(self):
        """Make every rank start from rank 0's weights."""
        if self.comm is None:
            return
        for a in self.params.arenas():
            self.comm.broadcast(a.master, 0)
        if self.is_cuda:
            torch.cuda.current_stream(self.params.device).synchronize()
        self.params.decay.refresh_mirror()
