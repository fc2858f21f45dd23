"""Transport: the native mlcomp-broker daemon (csrc/broker/broker.cpp) and the
in-process broker obey the same contract (FIFO, blocking pop, lease/ack/requeue on
disconnect, revoke, result store)."""
import contextlib
import os
import socket
import subprocess
import threading
import time

import pytest

from mlcomp_amd.broker import BrokerClient, InProcBroker


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@contextlib.contextmanager
def _broker_daemon(sanitize, tmp_path, journal=None, port=None, compact_every=None):
    """Run the broker daemon; with ``sanitize='asan'`` the AddressSanitizer + UBSan build:
    the test's traffic runs against it, then it is stopped with SIGTERM (clean shutdown
    through its destructors, so LeakSanitizer runs) and must exit 0 with no report."""
    from mlcomp_amd.build import build_broker
    binary = build_broker(sanitize=sanitize)
    port = port or _free_port()
    err = open(tmp_path / f'broker-{sanitize or "plain"}.err', 'a+')
    extra = ['--journal', str(journal)] if journal else []
    if compact_every:
        extra += ['--compact-every', str(compact_every)]
    p = subprocess.Popen([binary, '--host', '127.0.0.1', '--port', str(port)] + extra, stdout=subprocess.PIPE,
                         stderr=err)
    while not p.stdout.readline().startswith(b'mlcomp-broker listening'):
        pass
    try:
        yield port
    finally:
        p.terminate()
        rc = p.wait(timeout=30)
        err.seek(0)
        log = err.read()
        err.close()
    assert rc == 0, (rc, log[-4000:])
    assert 'Sanitizer' not in log and 'runtime error' not in log, log[-4000:]


@pytest.fixture(params=['plain', 'asan'])
def daemon(request, tmp_path):
    with _broker_daemon(None if request.param == 'plain' else request.param, tmp_path) as port:
        yield port


@pytest.fixture(params=['native', 'native-asan', 'inproc'])
def broker_factory(request, tmp_path):
    if request.param == 'inproc':
        b = InProcBroker()
        yield lambda: b
        return
    with _broker_daemon('asan' if request.param == 'native-asan' else None, tmp_path) as port:
        clients = []

        def make():
            c = BrokerClient('127.0.0.1', port)
            clients.append(c)
            return c
        yield make
        for c in clients:
            c.close()


def test_fifo_ack_revoke_results(broker_factory):
    b = broker_factory()
    assert b.ping()
    ids = [b.push('q1', {'task': 'execute', 'args': [i]}) for i in range(3)]
    assert b.queue_len('q1') == 3
    assert b.revoke(ids[1]) is True
    assert b.revoke('999999') is False
    q, m = b.pop(['q0', 'q1'], 0.5)
    assert q == 'q1' and m['args'] == [0] and m['id'] == ids[0]
    assert b.has(m['id']) and b.has(ids[2]) and not b.has(ids[1])   # leased / queued / revoked
    assert b.ack(m['id']) is True
    assert not b.has(m['id'])
    assert b.ack(m['id']) is False        # no lease any more
    q, m = b.pop(['q1'], 0.5)
    assert m['args'] == [2]
    b.nack(m['id'])                       # back to the head
    q, m2 = b.pop(['q1'], 0.5)
    assert m2['args'] == [2]
    b.ack(m2['id'])
    assert b.pop(['q1'], 0.05) is None
    b.set_result('k', {'x': [1, 2]})
    assert b.get_result('k', 0.5) == {'x': [1, 2]}
    assert b.get_result('k', 0.05) is None


def test_blocking_pop_is_woken(broker_factory):
    consumer = broker_factory()
    producer = broker_factory()
    got = []
    t = threading.Thread(target=lambda: got.append(consumer.pop(['w'], 5.0)))
    t.start()
    time.sleep(0.2)
    producer.push('w', {'task': 'kill', 'args': [1]})
    t.join(3)
    assert got and got[0][1]['task'] == 'kill'


def test_rpc_call(broker_factory):
    server = broker_factory()
    client = broker_factory()

    def serve():
        q, m = server.pop(['ctl'], 5.0)
        server.set_result(m['reply'], sum(m['args']))
        server.ack(m['id'])
    t = threading.Thread(target=serve)
    t.start()
    assert client.call('ctl', 'add', 2, 3, timeout=5.0) == 5
    t.join()


def test_lease_requeued_when_consumer_dies(daemon):
    a = BrokerClient('127.0.0.1', daemon)
    a.push('jobs', {'task': 'execute', 'args': [7]})
    consumer = BrokerClient('127.0.0.1', daemon)
    q, m = consumer.pop(['jobs'], 1.0)
    assert a.queue_len('jobs') == 0
    consumer.close()                      # dies without ACK
    deadline = time.time() + 2
    while a.queue_len('jobs') == 0 and time.time() < deadline:
        time.sleep(0.02)
    q, m2 = a.pop(['jobs'], 1.0)
    assert m2['args'] == [7]


def test_dead_consumer_lease_goes_to_blocked_waiter(daemon):
    """A consumer dies holding a lease while another is blocked in POP: the re-queued
    message must reach the waiter immediately, not at the next PUSH or its timeout."""
    a = BrokerClient('127.0.0.1', daemon)
    a.push('jobs2', {'task': 'execute', 'args': [9]})
    dying = BrokerClient('127.0.0.1', daemon)
    assert dying.pop(['jobs2'], 1.0)[1]['args'] == [9]
    waiter = BrokerClient('127.0.0.1', daemon)
    got = []
    t0 = time.time()
    t = threading.Thread(target=lambda: got.append(waiter.pop(['jobs2'], 8.0)))
    t.start()
    time.sleep(0.3)
    dying.close()
    t.join(10)
    assert got and got[0] is not None and got[0][1]['args'] == [9]
    assert time.time() - t0 < 4.0


def test_request_before_half_close_is_served(daemon):
    s = socket.create_connection(('127.0.0.1', daemon))
    s.sendall(b'PUSH half {"task":"x"}\n')
    s.shutdown(socket.SHUT_WR)
    reply = s.makefile('rb').readline()
    s.close()
    assert reply.startswith(b'OK ')
    assert BrokerClient('127.0.0.1', daemon).queue_len('half') == 1


def test_client_does_not_resend_non_idempotent_push(daemon):
    c = BrokerClient('127.0.0.1', daemon)
    c.ping()

    class LostReply:
        """The request reaches the broker, the reply is lost."""
        def __init__(self, sock):
            self.sock = sock

        def sendall(self, data):
            self.sock.sendall(data)

        def close(self):
            self.sock.close()

    real = c._sock
    c._sock = LostReply(real)
    c._rf = type('R', (), {'readline': lambda self: b''})()
    with pytest.raises((ConnectionError, OSError)):
        c.push('once', {'task': 'y'})
    time.sleep(0.1)
    assert BrokerClient('127.0.0.1', daemon).queue_len('once') == 1


def test_half_closed_client_gets_every_reply(daemon):
    """A large pipelined batch followed by shutdown(SHUT_WR): every reply arrives (the
    socket buffer fills, so the broker must keep writing after EOF), and a blocking POP
    sent last is answered when a message arrives, then the connection closes."""
    n = 20000
    s = socket.create_connection(('127.0.0.1', daemon))
    s.sendall(b''.join(b'PUSH big {"task":"x","pad":"%s"}\n' % (b'y' * 200) for _ in range(n))
              + b'POP 5000 halfwait\n')
    s.shutdown(socket.SHUT_WR)
    time.sleep(0.3)
    other = BrokerClient('127.0.0.1', daemon)
    other.push('halfwait', {'task': 'late'})
    f = s.makefile('rb')
    lines = f.read().splitlines()
    s.close()
    assert len(lines) == n + 1 and all(x.startswith(b'OK ') for x in lines[:n])
    assert lines[-1].startswith(b'MSG halfwait')
    # the lease died with the closed connection: the message is queued again
    deadline = time.time() + 2
    while other.queue_len('halfwait') == 0 and time.time() < deadline:
        time.sleep(0.02)
    assert other.queue_len('halfwait') == 1 and other.queue_len('big') == n


def test_journal_survives_broker_restart(tmp_path):
    """--journal: pushed-but-unacked messages (queued or leased) come back after the
    broker process is killed; acked and revoked ones do not; ids keep growing."""
    j = tmp_path / 'broker.journal'
    port = _free_port()
    with _broker_daemon(None, tmp_path, journal=j, port=port):
        c = BrokerClient('127.0.0.1', port)
        ids = [c.push('jq', {'task': 'execute', 'args': [i]}) for i in range(4)]
        c.revoke(ids[1])
        _, m = c.pop(['jq'], 1.0)
        assert c.ack(m['id'])                  # 0 done
        _, leased = c.pop(['jq'], 1.0)         # 2 leased when the broker goes down
        c.close()
    with _broker_daemon('asan', tmp_path, journal=j, port=port):
        c = BrokerClient('127.0.0.1', port)
        assert c.queue_len('jq') == 2
        assert c.has(ids[2]) and c.has(ids[3]) and not c.has(ids[0]) and not c.has(ids[1])
        got = [c.pop(['jq'], 1.0)[1]['args'] for _ in range(2)]
        assert got == [[2], [3]]
        new = c.push('jq', {'task': 'z'})
        assert int(new) > int(ids[-1])
        c.close()


@pytest.mark.parametrize('sanitize', [None, 'asan'])
def test_journal_compaction_at_push_and_ack(tmp_path, sanitize):
    """A compaction triggered by the very line a PUSH / ACK journals (--compact-every 1:
    after every line) rewrites the journal from the live state: the pushed message must
    already be in it, and the acked one must already be gone (journal after
    the state change, not before)."""
    j = tmp_path / 'broker.journal'
    port = _free_port()
    with _broker_daemon(sanitize, tmp_path, journal=j, port=port, compact_every=1):
        c = BrokerClient('127.0.0.1', port)
        ids = [c.push('cq', {'task': 'execute', 'args': [i]}) for i in range(3)]
        _, m = c.pop(['cq'], 1.0)
        assert m['args'] == [0] and c.ack(m['id'])
        c.close()
    with _broker_daemon(sanitize, tmp_path, journal=j, port=port, compact_every=1):
        c = BrokerClient('127.0.0.1', port)
        assert c.queue_len('cq') == 2, j.read_text()
        assert not c.has(ids[0]) and c.has(ids[1]) and c.has(ids[2])
        assert [c.pop(['cq'], 1.0)[1]['args'] for _ in range(2)] == [[1], [2]]
        c.close()
