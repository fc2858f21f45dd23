"""RCCL failure handling on one GPU (mlcomp_amd/parallel/comm.py, csrc/kernels/rccl_comm.hip).

* A world-2 communicator whose rank 1 never joins: rank 0's non-blocking init is aborted
  at MLC_COMM_INIT_TIMEOUT and raises CommTimeout with the scheduler's restart message,
  instead of hanging in the rendezvous.  It runs in a child process under its own time
  limit, so a regression cannot hang the suite.
* A world-1 communicator through the production path (non-blocking init, watchdog
  registered, step completion watched) still all-reduces, and an abort makes the next
  call raise.
"""
import os
import subprocess
import sys
import time

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_NEVER_JOINS = r'''
import socket, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[1])
from mlcomp_amd.parallel.comm import RcclComm, CommTimeout
from mlcomp_amd.server.supervisor import FATAL_RESTART_MESSAGES
s = socket.socket(); s.bind(('127.0.0.1', 0)); port = s.getsockname()[1]; s.close()
store = dist.TCPStore('127.0.0.1', port, 1, True)
t0 = time.monotonic()
try:
    RcclComm(0, 2, torch.device('cuda', 0), store=store, tag='never', init_timeout=4.0)
except CommTimeout as e:
    dt = time.monotonic() - t0
    assert any(m in str(e) for m in FATAL_RESTART_MESSAGES), str(e)
    print(f'RAISED {dt:.2f} {e}', flush=True)
    sys.exit(0)
print('NO RAISE', flush=True)
sys.exit(3)
'''


def test_peer_that_never_joins_raises_within_init_timeout():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, '-c', _NEVER_JOINS, ROOT], capture_output=True, text=True, timeout=90,
                       env=dict(os.environ, NCCL_DEBUG='WARN'))
    wall = time.monotonic() - t0
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith('RAISED')][0]
    dt = float(line.split()[1])
    assert 4.0 <= dt < 15.0, line
    assert 'communicator init timed out after 4 s on rank 0 of 2' in line
    print(f'init abort after {dt:.2f} s (child wall {wall:.1f} s)')


def test_world1_comm_nonblocking_path_and_abort():
    import torch.distributed as dist
    from mlcomp_amd.parallel.comm import WATCHDOG, CommError, RcclComm
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore('127.0.0.1', port, 1, True)
    comm = RcclComm(0, 1, torch.device('cuda', 0), store=store, tag='wd1', timeout=30)
    assert comm in WATCHDOG.comms and comm._async_error() == 0
    t = torch.arange(4096, device='cuda', dtype=torch.float32)
    comm.all_reduce(t)
    comm.watch_stream(what='test step')
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(4096, device='cuda', dtype=torch.float32))
    assert WATCHDOG.check_once() == [] and comm.failed is None
    comm.fail('RCCL watchdog: injected failure')     # what the watchdog does on an error
    assert comm._h is None and comm not in WATCHDOG.comms
    with pytest.raises(CommError, match='injected failure'):
        comm.all_reduce(t)
