"""Communicators for the native data-parallel engine.

``RcclComm`` - the GPU path: an RCCL communicator owned by this framework
(`csrc/kernels/rccl_comm.hip`).  Collectives are enqueued on an explicit HIP stream, so
they overlap compute through events and are captured into HIP graphs like any kernel.
The unique id travels through the ``torch.distributed`` TCP store (rank 0 publishes, the
others read), so the only requirement is an initialised default process group (the
bench and the training executor create one with backend "nccl" == RCCL on ROCm).

``TorchComm`` - the CPU path (gloo) with the same interface, used by the multi-process
CPU tests and by CPU-only workers.

Failure handling.  By bypassing the ProcessGroup the communicator also bypasses torch's
NCCL watchdog, which the reference relies on through ``init_process_group('nccl')``
(`mlcomp/worker/executors/catalyst_/catalyst_.py:228-230`), so it brings its own:

* the RCCL communicator is created non-blocking and its init is polled under
  ``MLC_COMM_INIT_TIMEOUT`` seconds: a peer that never joins aborts the communicator and
  raises :class:`CommTimeout` instead of hanging;
* a :class:`Watchdog` thread polls every live communicator's async error and the
  completion events of the steps that issued collectives (``watch``); an async error or a
  step still running ``MLC_COMM_TIMEOUT`` seconds after it was issued aborts the
  communicator (``ncclCommAbort``: RCCL kernels spinning on a dead peer exit, so the rank's
  stream drains) and the next call on it raises;
* every failure message starts with ``RCCL watchdog:``, which the scheduler's fatal-error
  list matches (`server/supervisor.py` FATAL_RESTART_MESSAGES -> the DAG restarts from its
  last checkpoint, as the reference does for NCCL errors, `supervisor.py:400-410`).
"""
from __future__ import annotations

import collections
import contextlib
import ctypes as C
import os
import threading
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

from mlcomp_amd.ops import _lib

import glob
import re

_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3, torch.int32: 4}
_OP = {'sum': 0, 'max': 1, 'min': 2, 'avg': 3}


# RCCL's own INFO log, filtered to the per-channel connection lines ("Channel 00/0 :
# 0[0] -> 1[1] via P2P/IPC"): which transport each rank's rings / trees use.  Intra-node
# on MI355X every pair should say P2P (xGMI); SHM means the peers could not map each
# other's memory (e.g. each process saw only its own GPU) and traffic bounces off the host.
_VIA = re.compile(r'via (\S+)')
LAST_TRANSPORTS: dict = {}


def enable_transport_log(folder: str) -> Optional[str]:
    """Route RCCL's INIT/P2P/SHM/NET info lines into ``folder/rccl.<host>.<pid>.log``
    (must run before the process's first RCCL call; a user-set NCCL_DEBUG wins)."""
    if os.environ.get('NCCL_DEBUG'):
        return os.environ.get('NCCL_DEBUG_FILE')
    os.makedirs(folder, exist_ok=True)
    path = os.path.join(folder, 'rccl.%h.%p.log')
    os.environ.update(NCCL_DEBUG='INFO', NCCL_DEBUG_SUBSYS='INIT,P2P,SHM,NET', NCCL_DEBUG_FILE=path)
    return path


def transport_summary(text: str) -> dict:
    """{transport: number of channel connections} from RCCL INFO log text."""
    out: dict = {}
    for line in text.splitlines():
        if 'Channel' not in line:
            continue
        m = _VIA.search(line)
        if m:
            out[m.group(1)] = out.get(m.group(1), 0) + 1
    return out


def _read_transport_log() -> dict:
    pattern = os.environ.get('NCCL_DEBUG_FILE')
    if not pattern:
        return {}
    path = pattern.replace('%h', os.uname().nodename).replace('%p', str(os.getpid()))
    text = ''
    for f in ([path] if os.path.exists(path) else glob.glob(pattern.replace('%h', '*').replace('%p', str(os.getpid())))):
        with open(f, errors='replace') as fh:
            text += fh.read()
    return transport_summary(text)


WATCHDOG_MESSAGE = 'RCCL watchdog:'
COMM_TIMEOUT = float(os.environ.get('MLC_COMM_TIMEOUT', '600'))
INIT_TIMEOUT = float(os.environ.get('MLC_COMM_INIT_TIMEOUT', str(COMM_TIMEOUT)))
_IN_PROGRESS = 7             # ncclInProgress
_TIMED_OUT = 1000            # rccl_comm.hip kCommTimeout


class CommError(RuntimeError):
    """The communicator failed (async RCCL error, abort); the message starts with
    ``RCCL watchdog:``."""


class CommTimeout(CommError):
    """A rendezvous or a collective outlived its deadline."""


class Watched:
    """What the :class:`Watchdog` needs of a communicator: ``_async_error()`` (0 ok, 7 in
    progress, else failed), ``_abort()``, ``rank`` / ``world``, ``timeout`` seconds, and the
    ``failed`` message it sets.  ``check()`` raises that failure in the caller's thread."""
    failed: Optional[str] = None
    failed_timeout = False
    timeout = COMM_TIMEOUT
    rank = 0
    world = 1

    def _async_error(self) -> int:  # pragma: no cover - implemented by the communicators
        return 0

    def _abort(self):  # pragma: no cover
        pass

    def _error_name(self, code: int) -> str:
        return f'error {code}'

    def fail(self, msg: str, timeout: bool = False):
        """Record the first failure and abort the communicator (idempotent)."""
        if self.failed is not None:
            return
        self.failed, self.failed_timeout = msg, timeout
        try:
            self._abort()
        except Exception:
            pass

    def check(self):
        if self.failed is not None:
            raise (CommTimeout if self.failed_timeout else CommError)(self.failed)

    def watch(self, done: Callable[[], bool], what: str = 'step'):
        """Hand the watchdog a completion probe of work that issued collectives on this
        communicator (a recorded event's ``query``)."""
        WATCHDOG.watch(self, done, what)


class Watchdog:
    """Polls every registered communicator (``register``) for async errors and every
    watched piece of work (``watch``) for completion; fails and aborts a communicator whose
    work is still pending ``comm.timeout`` seconds after it was issued.  ``check_once`` is
    the whole state machine (the CPU tests drive it with a fake communicator and clock);
    ``start`` runs it on a daemon thread every ``poll`` seconds."""

    MAX_PENDING = 64

    def __init__(self, poll: float = 1.0, clock: Callable[[], float] = time.monotonic):
        self.poll, self.clock = poll, clock
        self.comms: list = []
        self.pending: collections.deque = collections.deque()
        self.lock = threading.Lock()
        self._thread = None
        self._stop = threading.Event()
        # graph capture in progress (GraphedStep._capture): no probes - an event query from
        # this thread while another thread captures invalidates the capture (global mode)
        self._busy = threading.Lock()
        self._paused = 0

    @contextlib.contextmanager
    def paused(self):
        """No probe runs while the block runs (a pass in progress finishes first)."""
        with self._busy:
            self._paused += 1
        try:
            yield
        finally:
            with self._busy:
                self._paused -= 1

    def register(self, comm: Watched):
        with self.lock:
            if comm not in self.comms:
                self.comms.append(comm)
        self.start()

    def unregister(self, comm: Watched):
        with self.lock:
            if comm in self.comms:
                self.comms.remove(comm)
            self.pending = collections.deque(p for p in self.pending if p[0] is not comm)

    def watch(self, comm: Watched, done: Callable[[], bool], what: str = 'step'):
        with self.lock:
            # the oldest pending items decide a timeout; a full queue only drops new ones
            if len(self.pending) < self.MAX_PENDING:
                self.pending.append((comm, done, self.clock(), what))

    def check_once(self) -> list:
        """One pass; returns the communicators it failed in this pass."""
        failed = []
        with self.lock:
            comms = list(self.comms)
        for c in comms:
            if c.failed is not None:
                continue
            try:
                st = c._async_error()
            except Exception as e:          # the handle is gone: nothing to watch
                st = 0 if getattr(c, '_h', 1) is None else -1
                if st:
                    c.fail(f'{WATCHDOG_MESSAGE} async error query failed on rank {c.rank} of {c.world}: {e}')
                    failed.append(c)
                continue
            if st not in (0, _IN_PROGRESS):
                c.fail(f'{WATCHDOG_MESSAGE} RCCL async error on rank {c.rank} of {c.world}: {c._error_name(st)} '
                       '(communicator aborted)')
                failed.append(c)
        now = self.clock()
        keep = collections.deque()
        with self.lock:
            items = list(self.pending)
        for comm, done, t0, what in items:
            if comm.failed is not None:
                continue
            try:
                ok = bool(done())
            except Exception:
                ok = True                   # the event's stream / device is gone
            if ok:
                continue
            if now - t0 > comm.timeout:
                comm.fail(f'{WATCHDOG_MESSAGE} {what} with RCCL collectives not finished after {now - t0:.1f} s '
                          f'(MLC_COMM_TIMEOUT={comm.timeout:g}) on rank {comm.rank} of {comm.world}: a peer rank '
                          'died or hangs; communicator aborted', timeout=True)
                failed.append(comm)
                continue
            keep.append((comm, done, t0, what))
        with self.lock:
            done_ids = {id(i) for i in items}
            # items watched while this pass ran stay queued
            self.pending = keep + collections.deque(p for p in self.pending if id(p) not in done_ids)
        return failed

    def start(self):
        if self._thread is not None and self._thread.is_alive():
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name='mlc-rccl-watchdog', daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()

    def _loop(self):
        while not self._stop.wait(self.poll):
            with self._busy:
                if self._paused:
                    continue
                try:
                    self.check_once()
                except Exception:   # never let the watchdog thread die on a probe
                    pass


WATCHDOG = Watchdog(poll=float(os.environ.get('MLC_COMM_WATCHDOG_POLL', '1.0')))


class RcclComm(Watched):
    def __init__(self, rank: int, world: int, device: torch.device, store=None, tag='mlc',
                 init_timeout: Optional[float] = None, timeout: Optional[float] = None):
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        self.timeout = COMM_TIMEOUT if timeout is None else float(timeout)
        self._h = None
        # the handle is read by the watchdog thread (async-error polls) and torn down by
        # abort / close: every RCCL call that takes it runs under this lock, so no call ever
        # sees a communicator that another thread has already freed
        self._hlock = threading.RLock()
        lib = _lib.load()
        lib.mlc_comm_set_timeout(int(self.timeout * 1000))
        nbytes = lib.mlc_comm_unique_id_bytes()
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        key = f'{tag}/rccl_uid'
        if rank == 0:
            buf = C.create_string_buffer(nbytes)
            rc = lib.mlc_comm_get_unique_id(buf)
            if rc != 0:
                raise RuntimeError(f'ncclGetUniqueId failed ({rc})')
            store.set(key, buf.raw)
            uid = buf.raw
        else:
            uid = store.get(key)
        err = C.c_int(0)
        blocking = int(os.environ.get('MLC_COMM_BLOCKING', '0') == '1')
        self._h = lib.mlc_comm_init(C.c_char_p(uid), world, rank, self.device.index or 0, blocking,
                                    C.byref(err))
        if not self._h:
            raise CommError(f'{WATCHDOG_MESSAGE} ncclCommInitRankConfig failed on rank {rank} of {world}: '
                            f'{self._error_name(err.value)}')
        self._wait_init(INIT_TIMEOUT if init_timeout is None else float(init_timeout), err.value)
        # the connections are made lazily by the first collective of each kind: the bucketer's
        # initial broadcast / first all-reduce; read the log then (transports())
        self.transports = {}
        WATCHDOG.register(self)

    def _wait_init(self, limit: float, state: int):
        """Poll the non-blocking init until every rank has joined, or abort at ``limit`` s."""
        t0 = time.monotonic()
        while state == _IN_PROGRESS:
            if time.monotonic() - t0 > limit:
                self._abort()
                self._h = None
                raise CommTimeout(f'{WATCHDOG_MESSAGE} communicator init timed out after {limit:g} s on rank '
                                  f'{self.rank} of {self.world} (a peer rank never joined; MLC_COMM_INIT_TIMEOUT)')
            time.sleep(0.002)
            state = self._async_error()
        if state != 0:
            name = self._error_name(state)
            self._abort()
            self._h = None
            raise CommError(f'{WATCHDOG_MESSAGE} communicator init failed on rank {self.rank} of {self.world}: {name}')

    # ---- Watched
    def _async_error(self) -> int:
        with self._hlock:
            if self._h is None:
                return 0
            return int(_lib.load().mlc_comm_async_error(C.c_void_p(self._h)))

    def _abort(self):
        with self._hlock:
            h, self._h = self._h, None
            if h is not None:
                _lib.load().mlc_comm_abort(C.c_void_p(h))
        if h is not None:
            WATCHDOG.unregister(self)

    def _error_name(self, code: int) -> str:
        lib = _lib.load()
        s = (lib.mlc_comm_error_string(int(code)) or b'').decode(errors='replace')
        last = ''
        with self._hlock:
            if self._h is not None and code not in (0, _TIMED_OUT):
                last = (lib.mlc_comm_last_error(C.c_void_p(self._h)) or b'').decode(errors='replace')
        return f'{s} ({code})' + (f': {last}' if last else '')

    def _call(self, name, *args):
        self.check()
        with self._hlock:
            if self._h is None:
                raise CommError(f'{WATCHDOG_MESSAGE} {name} on a closed communicator (rank {self.rank} of '
                                f'{self.world})')
            rc = int(getattr(_lib.load(), name)(C.c_void_p(self._h), *args))
        if rc == 0:
            return
        if rc == _TIMED_OUT:
            self.fail(f'{WATCHDOG_MESSAGE} {name} was not issued within {self.timeout:g} s on rank {self.rank} of '
                      f'{self.world} (MLC_COMM_TIMEOUT); communicator aborted', timeout=True)
        else:
            self.fail(f'{WATCHDOG_MESSAGE} {name} failed on rank {self.rank} of {self.world}: '
                      f'{self._error_name(rc)}; communicator aborted')
        self.check()

    def transports_now(self) -> dict:
        """Transport histogram of this process's RCCL connections so far (needs
        :func:`enable_transport_log` before the first RCCL call)."""
        torch.cuda.synchronize(self.device)
        self.transports = _read_transport_log()
        LAST_TRANSPORTS.clear()
        LAST_TRANSPORTS.update(self.transports)
        return self.transports

    def _stream(self, stream):
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        return C.c_void_p(s.cuda_stream)

    def all_reduce(self, t: torch.Tensor, op='sum', stream=None):
        self._call('mlc_allreduce', _lib.ptr(t), _lib.ptr(t), t.numel(), _DT[t.dtype], _OP[op], self._stream(stream))

    def broadcast(self, t: torch.Tensor, root=0, stream=None):
        self._call('mlc_broadcast', _lib.ptr(t), _lib.ptr(t), t.numel(), _DT[t.dtype], root, self._stream(stream))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op='sum', stream=None):
        self._call('mlc_reduce_scatter', _lib.ptr(inp), _lib.ptr(out), out.numel(), _DT[out.dtype], _OP[op],
                   self._stream(stream))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        self._call('mlc_allgather', _lib.ptr(inp), _lib.ptr(out), inp.numel(), _DT[inp.dtype], self._stream(stream))

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        n = inp.numel() // self.world
        self._call('mlc_alltoall', _lib.ptr(inp), _lib.ptr(out), n, _DT[inp.dtype], inp.element_size(), self.world,
                   self._stream(stream))

    def watch_stream(self, stream=None, what: str = 'step'):
        """Record an event on ``stream`` (default: current) after work that issued this
        communicator's collectives and let the watchdog time it."""
        ev = torch.cuda.Event()
        ev.record(stream if stream is not None else torch.cuda.current_stream(self.device))
        self.watch(ev.query, what)

    def close(self):
        if getattr(self, '_h', None) is None or not hasattr(self, '_hlock'):
            return
        WATCHDOG.unregister(self)
        with self._hlock:
            h, self._h = self._h, None
            if h is not None:
                _lib.load().mlc_comm_destroy(C.c_void_p(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TorchComm:
    """torch.distributed (gloo / any backend) with the RcclComm interface; ``stream`` is
    ignored (CPU collectives are synchronous)."""

    def __init__(self, rank: int, world: int, group=None):
        self.rank, self.world, self.group = rank, world, group

    def all_reduce(self, t, op='sum', stream=None):
        if op == 'avg':
            dist.all_reduce(t, group=self.group)
            t.div_(self.world)
            return
        rop = {'sum': dist.ReduceOp.SUM, 'max': dist.ReduceOp.MAX, 'min': dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)

    def broadcast(self, t, root=0, stream=None):
        dist.broadcast(t, src=root, group=self.group)

    def reduce_scatter(self, out, inp, op='sum', stream=None):
        tmp = inp.clone()
        dist.all_reduce(tmp, group=self.group)
        out.copy_(tmp.chunk(self.world)[self.rank])

    def all_gather(self, out, inp, stream=None):
        parts = list(out.chunk(self.world))
        dist.all_gather(parts, inp, group=self.group)

    def all_to_all(self, out, inp, stream=None):
        dist.all_to_all_single(out, inp, group=self.group)

    def close(self):
        pass


_COMMS_MADE = 0


def make_comm(device: Optional[torch.device] = None):
    """Communicator for the current process group (None when world size is 1).

    Every rank creates its communicators in the same order (one per native step, e.g. one
    per training stage), so the n-th one of each rank publishes / reads the unique id under
    its own store key ``mlc<n>/rccl_uid``: a later communicator can never pick up the id
    of an earlier one that is still in the store."""
    global _COMMS_MADE
    if not dist.is_available() or not dist.is_initialized():
        return None
    world = dist.get_world_size()
    if world == 1:
        return None
    rank = dist.get_rank()
    _COMMS_MADE += 1
    # GPU tensors under an nccl (= RCCL) process group: the framework's own RCCL
    # communicator; any other backend (gloo: CPU runs, or several ranks sharing one GPU in a
    # rehearsal of the multi-rank path) goes through torch.distributed itself
    if device is not None and torch.device(device).type == 'cuda' and dist.get_backend() == 'nccl':
        return RcclComm(rank, world, device, tag=f'mlc{_COMMS_MADE}')
    return TorchComm(rank, world)
