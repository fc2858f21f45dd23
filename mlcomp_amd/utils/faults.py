"""Test-time fault injection ("kill a rank, drop a heartbeat, corrupt a
checkpoint"; the reference has none).

Faults are configured with the ``MLC_FAULTS`` environment variable - a comma-separated
list - so they reach task processes spawned by the worker pool (set it in an executor's
``env:`` block or in the worker's environment):

``kill_rank=R@S``
    the training process of rank R exits abruptly (``os._exit(137)``, as if SIGKILLed)
    when it starts its S-th training batch (1-based, counted over the whole run).
``kill_task=S``
    the task process exits abruptly S seconds after its executor starts work (exercises
    the worker supervisor's dead-process detection: InProgress + gone pid => Failed).
``crash_task=MESSAGE``
    the executor raises ``RuntimeError(MESSAGE)`` before ``work()`` (e.g. a HIP/RCCL fatal
    string, to exercise the scheduler's auto-restart heuristic).
``drop_heartbeat=N``
    the worker supervisor skips its next N heartbeats (queues then look dead to the
    scheduler's 15 s liveness window).
``corrupt_checkpoint``
    every checkpoint file is truncated right after it is written (resume must fall back to
    the other checkpoint or start fresh).

Every hook is a no-op (one dict lookup) when ``MLC_FAULTS`` is unset.
"""
from __future__ import annotations

import os
import threading
from typing import Dict

_LOCK = threading.Lock()
_CACHE: Dict[str, Dict[str, str]] = {}
_COUNTERS: Dict[str, int] = {}


def spec() -> Dict[str, str]:
    raw = os.environ.get('MLC_FAULTS', '')
    if not raw:
        return {}
    out = _CACHE.get(raw)
    if out is None:
        out = {}
        for item in raw.split(','):
            item = item.strip()
            if not item:
                continue
            k, _, v = item.partition('=')
            out[k.strip()] = v.strip()
        _CACHE[raw] = out
    return out


def reset():
    """Forget consumed counters (tests)."""
    with _LOCK:
        _COUNTERS.clear()
        _CACHE.clear()


def maybe_kill_rank(rank: int, step: int):
    v = spec().get('kill_rank')
    if not v:
        return
    r, _, s = v.partition('@')
    if int(r) == int(rank) and int(step) >= int(s or 1):
        os._exit(137)


def arm_task_kill():
    """Start the ``kill_task`` timer for this process (called when an executor starts)."""
    v = spec().get('kill_task')
    if not v:
        return
    t = threading.Timer(float(v), lambda: os._exit(137))
    t.daemon = True
    t.start()


def maybe_crash_task():
    msg = spec().get('crash_task')
    if msg:
        raise RuntimeError(msg)


def heartbeat_dropped() -> bool:
    v = spec().get('drop_heartbeat')
    if not v:
        return False
    with _LOCK:
        n = _COUNTERS.get('drop_heartbeat', int(v))
        if n <= 0:
            return False
        _COUNTERS['drop_heartbeat'] = n - 1
        return True


def after_checkpoint_write(path: str):
    if 'corrupt_checkpoint' not in spec():
        return
    size = os.path.getsize(path)
    with open(path, 'r+b') as f:
        f.truncate(max(0, size // 3))


__all__ = ['spec', 'reset', 'maybe_kill_rank', 'arm_task_kill', 'maybe_crash_task', 'heartbeat_dropped',
           'after_checkpoint_write']
