"""Communicators for the native data-parallel engine.

``RcclComm`` - the GPU path: an RCCL communicator owned by this framework
(`csrc/kernels/rccl_comm.hip`).  Collectives are enqueued on an explicit HIP stream, so
they overlap compute through events and are captured into HIP graphs like any kernel.
The unique id travels through the ``torch.distributed`` TCP store (rank 0 publishes, the
others read), so the only requirement is an initialised default process group (the
bench and the training executor create one with backend "nccl" == RCCL on ROCm).

``TorchComm`` - the CPU path (gloo) with the same interface, used by the multi-process
CPU tests and by CPU-only workers.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

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


class RcclComm:
    def __init__(self, rank: int, world: int, device: torch.device, store=None, tag='mlc'):
        self.rank, self.world = rank, world
        self.device = torch.device(device)
        lib = _lib.load()
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
        self._h = lib.mlc_comm_init(C.c_char_p(uid), world, rank, self.device.index or 0,
                                    C.byref(err))
        if not self._h:
            raise RuntimeError(f'ncclCommInitRank failed ({err.value})')
        # the connections are made lazily by the first collective of each kind: the bucketer's
        # initial broadcast / first all-reduce; read the log then (transports())
        self.transports = {}

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
        _lib.call('mlc_allreduce', C.c_void_p(self._h), _lib.ptr(t), _lib.ptr(t), t.numel(),
                  _DT[t.dtype], _OP[op], self._stream(stream))

    def broadcast(self, t: torch.Tensor, root=0, stream=None):
        _lib.call('mlc_broadcast', C.c_void_p(self._h), _lib.ptr(t), _lib.ptr(t), t.numel(),
                  _DT[t.dtype], root, self._stream(stream))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op='sum', stream=None):
        _lib.call('mlc_reduce_scatter', C.c_void_p(self._h), _lib.ptr(inp), _lib.ptr(out),
                  out.numel(), _DT[out.dtype], _OP[op], self._stream(stream))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        _lib.call('mlc_allgather', C.c_void_p(self._h), _lib.ptr(inp), _lib.ptr(out), inp.numel(),
                  _DT[inp.dtype], self._stream(stream))

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        n = inp.numel() // self.world
        _lib.call('mlc_alltoall', C.c_void_p(self._h), _lib.ptr(inp), _lib.ptr(out), n,
                  _DT[inp.dtype], inp.element_size(), self.world, self._stream(stream))

    def close(self):
        if getattr(self, '_h', None):
            _lib.load().mlc_comm_destroy(C.c_void_p(self._h))
            self._h = None

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
