"""Shared driver of the native training steps: eager warmup -> one HIP-graph capture ->
replay, with a collective fallback to eager execution.

The three native steps (:class:`~mlcomp_amd.train.native_step.NativeClassifierStep`,
:class:`~mlcomp_amd.train.native_bert_step.NativeBertStep`,
:class:`~mlcomp_amd.train.native_seg_step.NativeSegmentationStep`) implement ``_body()``
(zero grads, forward, backward with bucketed all-reduce, fused optimizer) and inherit the
step protocol from :class:`GraphedStep`:

* every call first runs the optimizer's host-side ``prepare()`` (step counter, Adam bias
  corrections written into device memory), so graph replays see a fresh step each time;
* ``warmup_eager`` calls run ``_body()`` eagerly on a side stream (allocator warmup, lazy
  kernel-library init), then the next call captures ``_body()`` into one graph;
* if capture fails on ANY rank, every rank discards its graph and runs eagerly from then
  on.  Capture records work without executing it, so no device state (and no collective)
  has moved when the failure is seen; the ranks agree with one all-reduce of a flag before
  anything runs, which keeps the collective sequence identical on every rank.  Host state
  that ``_body()`` touched (bucket counters) is reset by ``_body()`` itself on the retry.
"""
from __future__ import annotations

import contextlib
import gc
import os
import warnings

import torch


_WORK_STREAMS = {}


@contextlib.contextmanager
def work_stream(device):
    """Run the enclosed GPU work on a stream of the framework's own instead of the NULL
    (default) stream, fenced to it on both sides; a no-op off the GPU or when the caller is
    already on a non-default stream.

    Why (profiles/round5/graph_null_stream.md): on ROCm 7 / PyTorch 2.10, eager work on the
    legacy NULL stream in a process that replays a captured training-step graph corrupts
    the replays - stock PyTorch reproduces it with no framework code
    (scripts/graph_torch_twin.py), a device sync after each replay does not always help, and
    the same eager work on a created stream is fine.  The runner, every native step and
    predict therefore keep their kernels off the NULL stream."""
    device = torch.device(device)
    if device.type != 'cuda' or os.environ.get('MLC_WORK_STREAM', '1') == '0':
        yield
        return
    cur = torch.cuda.current_stream(device)
    if cur.cuda_stream != 0:
        yield
        return
    key = device.index if device.index is not None else torch.cuda.current_device()
    st = _WORK_STREAMS.get(key)
    if st is None:
        st = _WORK_STREAMS[key] = torch.cuda.Stream(device)
    st.wait_stream(cur)
    with torch.cuda.stream(st):
        yield
    cur.wait_stream(st)


class GraphedStep:
    use_graph: bool
    warmup_eager: int
    graph = None
    calls: int = 0
    comm = None
    capture_error = None
    # BatchNorm running statistics (flat buffer, ops.layers.flatten_bn_buffers) and when rank
    # 0's copy is broadcast: 'step' (default; PyTorch DDP's broadcast_buffers=True, which the
    # reference's Catalyst DDP used) = at the end of every step, inside the captured graph;
    # 'eval' = only when the runner asks (before validation and checkpoints)
    bn_buffers = None
    bn_broadcast = os.environ.get('MLC_BN_BROADCAST', 'step')

    def broadcast_buffers(self):
        """Rank 0's BatchNorm running statistics to every rank: one
        broadcast of the flat buffer on the current stream.  A no-op on one rank."""
        if self.comm is None or self.bn_buffers is None or getattr(self.comm, 'world', 1) <= 1:
            return
        self.comm.broadcast(self.bn_buffers, 0)

    def _end_of_step_buffers(self):
        if self.bn_broadcast == 'step':
            self.broadcast_buffers()

    def _body(self):  # pragma: no cover - implemented by the concrete steps
        raise NotImplementedError

    def _agree(self, ok: bool) -> bool:
        """True only when every rank reports ``ok`` (one MIN all-reduce of a flag)."""
        if self.comm is None or getattr(self.comm, 'world', 1) <= 1:
            return ok
        flag = torch.tensor([1.0 if ok else 0.0], device=self.device)
        self.comm.all_reduce(flag, 'min')
        return bool(flag.item() > 0.5)

    def _capture(self):
        from ..ops import functional as Fn
        torch.cuda.synchronize(self.device)
        graph = torch.cuda.CUDAGraph()
        err = None
        # the graph's split-K slabs and zero-on-entry scratch belong to this step (and
        # die with it): eager work elsewhere never writes what a replay reads
        self._capture_ws = {}
        # no garbage collection while the stream captures: a collected object from earlier
        # work (an event, a graph, a stream) whose destructor calls the HIP runtime during
        # capture aborts the process (seen once in the full GPU suite: "Fatal Python error:
        # Aborted" with "Garbage-collecting" at the top of the capturing thread's stack)
        gc.collect()
        was = gc.isenabled()
        gc.disable()
        from ..parallel.comm import WATCHDOG
        try:
            # the RCCL watchdog's event probes wait while this thread captures
            with WATCHDOG.paused(), torch.cuda.graph(graph), Fn.capture_scope(self._capture_ws):
                self._body()
        except Exception as e:   # capture refused (a collective or op the runtime cannot
            err = e              # capture): decided collectively below
        finally:
            if was:
                gc.enable()
        torch.cuda.synchronize(self.device)
        if self._agree(err is None):
            return graph
        self.capture_error = err if err is not None else RuntimeError('capture failed on a peer rank')
        warnings.warn(f'HIP graph capture failed, running the step eagerly: {self.capture_error}')
        del graph
        return None

    def __call__(self):
        self.calls += 1
        comm = self.comm
        watched = comm is not None and hasattr(comm, 'watch_stream')
        if watched:
            comm.check()        # a failure the RCCL watchdog saw: raise before replaying
        self.opt.prepare()
        with work_stream(self.device):
            self._call()
            if watched:         # the watchdog times this step's collectives (MLC_COMM_TIMEOUT)
                comm.watch_stream()

    def _call(self):
        if not self.use_graph:
            self._body()
            return
        if self.graph is None:
            if self.calls <= self.warmup_eager:
                s = torch.cuda.Stream(self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    self._body()
                torch.cuda.current_stream(self.device).wait_stream(s)
                return
            self.graph = self._capture()
            if self.graph is None:
                self.use_graph = False
                self._body()
                return
        self.graph.replay()
