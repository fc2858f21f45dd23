"""Task transport: named FIFO queues, leased pops with ack/requeue, a keyed result
store and liveness ping.

Replaces Celery-over-Redis (`mlcomp/worker/app.py:1-18`, vendored
`mlcomp/bin/redis-server`).  Two implementations of one interface:

* :class:`BrokerClient` - talks to the native ``mlcomp-broker`` daemon
  (`csrc/broker/broker.cpp`, C++17 epoll server) over TCP;
* :class:`InProcBroker` - thread-safe in-memory broker (tests, single-process runs).

Queue names follow the reference: ``{computer}_{docker}`` (scheduler -> any worker),
``{computer}_{docker}_{index}`` (personal, re-queued multi-stage tasks) and
``{computer}_{docker}_supervisor`` (kill / remove control messages).

Semantics: ``pop`` *leases* a message to the caller; ``ack`` deletes it, ``nack``
(or the consumer's connection dropping) puts it back at the head of its queue, so a
worker that dies mid-dispatch never loses a task.  ``revoke`` removes a pending
message (used when a task is stopped before a worker picked it up).
"""
from __future__ import annotations

import itertools
import json
import logging
import os
import socket
import threading
import time
import uuid
from collections import deque
from typing import Dict, List, Optional, Tuple

Message = Dict


_log = logging.getLogger(__name__)


class Broker:
    def push(self, queue: str, msg: Message) -> str:
        raise NotImplementedError

    def pop(self, queues: List[str], timeout: float = 1.0) -> Optional[Tuple[str, Message]]:
        raise NotImplementedError

    def ack(self, msg_id: str):
        raise NotImplementedError

    def nack(self, msg_id: str):
        raise NotImplementedError

    def has(self, msg_id: str) -> bool:
        """True while the message is queued or leased (not yet acked / revoked)."""
        raise NotImplementedError

    def revoke(self, msg_id: str) -> bool:
        raise NotImplementedError

    def set_result(self, key: str, value):
        raise NotImplementedError

    def get_result(self, key: str, timeout: float = 0.0):
        raise NotImplementedError

    def queue_len(self, queue: str) -> int:
        raise NotImplementedError

    def ping(self) -> bool:
        raise NotImplementedError

    # ---------------------------------------------------------------- helpers
    def send_task(self, queue: str, task: str, *args, reply: bool = False) -> str:
        msg = {'task': task, 'args': list(args)}
        if reply:
            msg['reply'] = 'r:' + uuid.uuid4().hex
        mid = self.push(queue, msg)
        return msg.get('reply', mid) if reply else mid

    def call(self, queue: str, task: str, *args, timeout: float = 30.0):
        key = self.send_task(queue, task, *args, reply=True)
        return self.get_result(key, timeout)


class InProcBroker(Broker):
    def __init__(self):
        self._q: Dict[str, deque] = {}
        self._leased: Dict[str, Tuple[str, Message]] = {}
        self._results: Dict[str, object] = {}
        self._cv = threading.Condition()
        self._ids = itertools.count(1)

    def push(self, queue, msg):
        with self._cv:
            mid = str(next(self._ids))
            m = dict(msg, id=mid)
            self._q.setdefault(queue, deque()).append(m)
            self._cv.notify_all()
            return mid

    def pop(self, queues, timeout=1.0):
        deadline = time.time() + timeout
        with self._cv:
            while True:
                for q in queues:
                    dq = self._q.get(q)
                    if dq:
                        m = dq.popleft()
                        self._leased[m['id']] = (q, m)
                        return q, m
                left = deadline - time.time()
                if left <= 0:
                    return None
                self._cv.wait(left)

    def ack(self, msg_id):
        with self._cv:
            return self._leased.pop(msg_id, None) is not None

    def has(self, msg_id):
        with self._cv:
            return msg_id in self._leased or any(m['id'] == msg_id for dq in self._q.values() for m in dq)

    def nack(self, msg_id):
        with self._cv:
            item = self._leased.pop(msg_id, None)
            if item:
                q, m = item
                self._q.setdefault(q, deque()).appendleft(m)
                self._cv.notify_all()

    def revoke(self, msg_id):
        with self._cv:
            for dq in self._q.values():
                for m in list(dq):
                    if m['id'] == msg_id:
                        dq.remove(m)
                        return True
        return False

    def set_result(self, key, value):
        with self._cv:
            self._results[key] = value
            self._cv.notify_all()

    def get_result(self, key, timeout=0.0):
        deadline = time.time() + timeout
        with self._cv:
            while key not in self._results:
                left = deadline - time.time()
                if left <= 0:
                    return None
                self._cv.wait(left)
            return self._results.pop(key)

    def queue_len(self, queue):
        with self._cv:
            return len(self._q.get(queue, ()))

    def ping(self):
        return True


class BrokerError(RuntimeError):
    pass


class BrokerClient(Broker):
    """Client of the native daemon.  One TCP connection per client object; calls are
    serialised with a lock (use one client per blocking consumer)."""

    def __init__(self, host: str = '127.0.0.1', port: int = 6380, connect_timeout: float = 5.0):
        self.host, self.port = host, port
        self.connect_timeout = connect_timeout
        self._lock = threading.Lock()
        self._sock = None
        self._rf = None

    def _connect(self):
        s = socket.create_connection((self.host, self.port), timeout=self.connect_timeout)
        s.settimeout(None)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s
        self._rf = s.makefile('rb')

    def close(self):
        with self._lock:
            self._drop()

    # safe to re-send after a lost reply: a POP lease dies with the old connection (the
    # broker re-queues it), the others do not change state twice.  PUSH / SET / NACK /
    # REVOKE are retried only when the request never reached the socket.  A re-sent ACK
    # whose first copy never arrived finds the lease gone (re-queued when the connection
    # dropped): the broker answers OK 0 and ack() reports the lost lease.
    IDEMPOTENT = frozenset(('PING', 'POP', 'LEN', 'ACK', 'STATS', 'HAS'))

    def _drop(self):
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
        self._sock = self._rf = None

    def _cmd(self, *parts: str) -> str:
        line = (' '.join(parts) + '\n').encode()
        with self._lock:
            for attempt in (0, 1):
                sent = False
                try:
                    if self._sock is None:
                        self._connect()
                    self._sock.sendall(line)
                    sent = True
                    resp = self._rf.readline()
                    if not resp:
                        raise ConnectionError('broker closed the connection')
                    break
                except (OSError, ConnectionError):
                    self._drop()
                    if attempt or (sent and parts[0] not in self.IDEMPOTENT):
                        raise
        resp = resp.decode().rstrip('\n')
        if resp.startswith('ERR'):
            raise BrokerError(resp[4:])
        return resp

    @staticmethod
    def _check(name: str):
        if not name or any(c.isspace() for c in name):
            raise ValueError(f'bad queue/key name {name!r}')
        return name

    def push(self, queue, msg):
        r = self._cmd('PUSH', self._check(queue), json.dumps(msg, separators=(',', ':')))
        return r.split(' ', 1)[1]

    def pop(self, queues, timeout=1.0):
        r = self._cmd('POP', str(int(timeout * 1000)), *[self._check(q) for q in queues])
        if r == 'NIL':
            return None
        _, q, mid, payload = r.split(' ', 3)
        m = json.loads(payload)
        m['id'] = mid
        return q, m

    def ack(self, msg_id):
        """True when the lease was released; False when the broker had no lease for it
        (it was re-queued after a lost connection: the message will be delivered again,
        and the task status check rejects the duplicate)."""
        ok = self._cmd('ACK', msg_id) == 'OK 1'
        if not ok:
            _log.warning('broker: no lease for message %s at ACK (re-queued after a dropped '
                         'connection; a duplicate delivery follows)', msg_id)
        return ok

    def has(self, msg_id):
        return self._cmd('HAS', msg_id) == 'OK 1'

    def nack(self, msg_id):
        self._cmd('NACK', msg_id)

    def revoke(self, msg_id):
        return self._cmd('REVOKE', msg_id) == 'OK 1'

    def set_result(self, key, value):
        self._cmd('SET', self._check(key), json.dumps(value, separators=(',', ':')))

    def get_result(self, key, timeout=0.0):
        r = self._cmd('GET', self._check(key), str(int(timeout * 1000)))
        if r == 'NIL':
            return None
        return json.loads(r.split(' ', 1)[1])

    def queue_len(self, queue):
        return int(self._cmd('LEN', self._check(queue)).split(' ', 1)[1])

    def ping(self):
        try:
            return self._cmd('PING') == 'PONG'
        except (OSError, BrokerError):
            return False


_DEFAULT: Optional[Broker] = None
_DLOCK = threading.Lock()


def get_broker() -> Broker:
    """Process-wide broker: the daemon at BROKER_HOST:BROKER_PORT, or an in-process
    broker when ``MLCOMP_BROKER=inproc``."""
    global _DEFAULT
    with _DLOCK:
        if _DEFAULT is None:
            if os.environ.get('MLCOMP_BROKER', '') == 'inproc':
                _DEFAULT = InProcBroker()
            else:
                from mlcomp_amd import config
                s = config.get()
                _DEFAULT = BrokerClient(s.BROKER_HOST, s.BROKER_PORT)
        return _DEFAULT


def set_broker(b: Optional[Broker]):
    global _DEFAULT
    with _DLOCK:
        _DEFAULT = b


def new_connection() -> Broker:
    """A fresh connection for a blocking consumer (shares the in-proc broker)."""
    b = get_broker()
    if isinstance(b, BrokerClient):
        return BrokerClient(b.host, b.port)
    return b


def queue_name(computer: str, docker: str = 'default', suffix=None) -> str:
    q = f'{computer}_{docker}'
    return q if suffix is None else f'{q}_{suffix}'


__all__ = ['Broker', 'InProcBroker', 'BrokerClient', 'BrokerError', 'get_broker', 'set_broker',
           'new_connection', 'queue_name']
