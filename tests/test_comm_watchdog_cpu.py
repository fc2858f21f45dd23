"""The RCCL watchdog's state machine (mlcomp_amd/parallel/comm.py) on a fake communicator
and a fake clock: async errors and timed-out steps abort the communicator once, the next
call raises, and the message is one the scheduler restarts a DAG on."""
import threading

import pytest

from mlcomp_amd.parallel.comm import (WATCHDOG_MESSAGE, CommError, CommTimeout, Watched, Watchdog)
from mlcomp_amd.server.supervisor import FATAL_RESTART_MESSAGES


class FakeComm(Watched):
    def __init__(self, timeout=5.0):
        self.rank, self.world, self.timeout = 1, 4, timeout
        self.state = 0
        self.aborts = 0

    def _async_error(self):
        return self.state

    def _abort(self):
        self.aborts += 1

    def _error_name(self, code):
        return {3: 'ncclInternalError (3)', 6: 'ncclRemoteError (6)'}.get(code, str(code))


class Clock:
    def __init__(self):
        self.t = 100.0

    def __call__(self):
        return self.t


def _restarts(msg):
    return any(m in msg for m in FATAL_RESTART_MESSAGES)


def test_async_error_aborts_once_and_raises():
    wd, c = Watchdog(clock=Clock()), FakeComm()
    wd.comms.append(c)
    assert wd.check_once() == [] and c.failed is None
    c.state = 7                                    # in progress is not an error
    assert wd.check_once() == [] and c.aborts == 0
    c.state = 6
    assert wd.check_once() == [c]
    assert c.aborts == 1 and 'ncclRemoteError' in c.failed and 'rank 1 of 4' in c.failed
    assert wd.check_once() == [] and c.aborts == 1  # a failed comm is not failed again
    with pytest.raises(CommError, match='RCCL watchdog') as e:
        c.check()
    assert not isinstance(e.value, CommTimeout)
    assert c.failed.startswith(WATCHDOG_MESSAGE) and _restarts(c.failed)


def test_step_that_never_completes_times_out():
    clock = Clock()
    wd, c = Watchdog(clock=clock), FakeComm(timeout=5.0)
    wd.comms.append(c)
    done = {'a': False, 'b': False}
    wd.watch(c, lambda: done['a'], 'step 1')
    clock.t += 1
    wd.watch(c, lambda: done['b'], 'step 2')
    clock.t += 3.5                                  # 4.5 s: within the timeout
    assert wd.check_once() == [] and len(wd.pending) == 2
    done['a'] = True                                # step 1 finished, step 2 still running
    clock.t += 1                                    # step 1 would be 5.5 s, step 2 4.5 s
    assert wd.check_once() == [] and len(wd.pending) == 1
    clock.t += 1.0                                  # step 2 at 5.5 s
    assert wd.check_once() == [c]
    assert c.aborts == 1 and len(wd.pending) == 0
    with pytest.raises(CommTimeout, match='step 2 with RCCL collectives not finished after 5.5 s'):
        c.check()
    assert _restarts(c.failed)


def test_completed_work_is_dropped_and_queue_is_bounded():
    clock = Clock()
    wd, c = Watchdog(clock=clock), FakeComm()
    for _ in range(Watchdog.MAX_PENDING + 10):
        wd.watch(c, lambda: True)
    assert len(wd.pending) == Watchdog.MAX_PENDING
    assert wd.check_once() == [] and len(wd.pending) == 0


def test_probe_errors_do_not_kill_the_watchdog():
    clock = Clock()
    wd, c = Watchdog(clock=clock), FakeComm(timeout=1.0)

    def broken():
        raise RuntimeError('event of a destroyed stream')
    wd.watch(c, broken)
    clock.t += 10
    assert wd.check_once() == [] and c.failed is None   # a probe that raises counts as done


def test_watchdog_thread_fails_a_stuck_step():
    """The daemon thread runs the same pass: a step that never completes fails within a few
    polls of its timeout."""
    wd, c = Watchdog(poll=0.01), FakeComm(timeout=0.05)
    wd.register(c)
    fired = threading.Event()
    orig = c._abort

    def abort():
        orig()
        fired.set()
    c._abort = abort
    wd.watch(c, lambda: False)
    assert fired.wait(5.0)
    wd.stop()
    with pytest.raises(CommTimeout):
        c.check()


def test_watchdog_probes_nothing_while_paused():
    """GraphedStep captures inside ``WATCHDOG.paused()``: no event query / async-error probe
    may run on the watchdog thread then (it would invalidate a global-mode capture); probing
    resumes afterwards."""
    import time
    wd, c = Watchdog(poll=0.005), FakeComm(timeout=100.0)
    probes = []
    c._async_error = lambda: probes.append(time.monotonic()) or 0
    wd.register(c)
    with wd.paused():
        t0 = time.monotonic()
        time.sleep(0.1)
        t1 = time.monotonic()
    assert not [t for t in probes if t0 < t < t1]
    time.sleep(0.1)
    wd.stop()
    assert [t for t in probes if t > t1], 'probing did not resume'


def test_torch_comm_has_no_watchdog_hooks():
    """The gloo path keeps torch.distributed's own timeouts (GraphedStep only watches
    communicators with ``watch_stream``)."""
    from mlcomp_amd.parallel.comm import TorchComm
    assert not hasattr(TorchComm(0, 1), 'watch_stream')
