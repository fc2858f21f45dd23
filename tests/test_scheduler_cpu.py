"""Scheduler GPU placement on synthetic 8-GPU MI355X computers: the
supervisor tick (`mlcomp_amd/server/supervisor.py`, reference
`mlcomp/server/back/supervisor.py:187-343`) is driven against an in-process broker and
the dispatched messages / rank tasks are checked - elastic ``gpu: a-b`` fan-out, DDP rank
``distr_info`` (rank, local_rank, visible GPU set, world size, master port from the
range and its reuse), busy GPUs, the 4+4 multi-branch packing onto NUMA halves, ranks
spanning computers, orphaned Queued tasks and the fatal-restart matcher."""
import datetime

import pytest

from mlcomp_amd.db.enums import TaskStatus, TaskType
from mlcomp_amd.utils.misc import yaml_load


@pytest.fixture
def sched(mlc_root, monkeypatch):
    from mlcomp_amd import broker
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    from mlcomp_amd.server.supervisor import SupervisorBuilder
    b = broker.InProcBroker()
    broker.set_broker(b)
    migrate()
    s = Session.create_session(key='sched-test')
    sup = SupervisorBuilder(session_key='sched-sup', broker=b)
    yield {'sup': sup, 'broker': b, 's': s}
    broker.set_broker(None)
    Session.cleanup()


def _computer(s, name, gpu=8, ip=None, alive=True):
    from mlcomp_amd.db.models import Computer, Docker, now
    s.add(Computer(name=name, gpu=gpu, cpu=128, memory=1536 * 1024, ip=ip or f'10.0.0.{len(name)}',
                   can_process_tasks=True))
    last = now() if alive else now() - datetime.timedelta(minutes=5)
    s.add(Docker(name='default', computer=name, last_activity=last, ports='29500-29502'))
    s.commit()


def _dag(s, executors: dict):
    from mlcomp_amd.dag.standard import dag_standard
    cfg = {'info': {'name': 'sched', 'project': 'p'}, 'executors': executors}
    return dag_standard(s, cfg, upload_files=False, control_reqs=False)


def _tasks(s, **filt):
    from mlcomp_amd.db.models import Task
    s.expire_all()
    q = s.query(Task)
    for k, v in filt.items():
        q = q.filter(getattr(Task, k) == v)
    return q.order_by(Task.id).all()


def _drain(b, queue):
    out = []
    while True:
        item = b.pop([queue], 0.0)
        if item is None:
            return out
        out.append(item[1])


def _ranks(s, parent_id):
    kids = _tasks(s, parent=parent_id)
    return [(k, yaml_load(k.additional_info)['distr_info']) for k in kids]


def test_elastic_distributed_fan_out_on_one_node(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1')
    tid = _dag(s, {'train': {'type': 'bash', 'command': 'true', 'gpu': '1-8', 'distr': True}})['train'][0]
    sup.build()
    ranks = _ranks(s, tid)
    assert len(ranks) == 8
    for r, (k, di) in enumerate(ranks):
        assert k.type == TaskType.Service.value and k.status == TaskStatus.Queued.value
        assert di['rank'] == r and di['world_size'] == 8 and di['master_port'] == 29500
        assert di['master_addr'] == '127.0.0.1' and di['master_computer'] == 'node1'
        # every rank sees the job's 8 GPUs and indexes its own by local_rank
        assert di['visible_gpus'] == '0,1,2,3,4,5,6,7' and di['local_rank'] == di['gpu'] == int(k.gpu_assigned)
    msgs = _drain(b, 'node1_default')
    assert sorted(m['args'][0] for m in msgs) == [k.id for k, _ in ranks]
    assert all(m['task'] == 'execute' for m in msgs)
    assert _tasks(s, id=tid)[0].status == TaskStatus.Queued.value


def test_busy_gpus_shrink_the_elastic_job(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1')
    ids = _dag(s, {'busy': {'type': 'bash', 'command': 'true', 'gpu': 3},
                   'train': {'type': 'bash', 'command': 'true', 'gpu': '2-8', 'distr': True, 'depends': []}})
    busy = _tasks(s, id=ids['busy'][0])[0]
    busy.status, busy.computer_assigned, busy.gpu_assigned = TaskStatus.InProgress.value, 'node1', '0,1,2'
    s.commit()
    sup.build()
    ranks = _ranks(s, ids['train'][0])
    assert sorted(di['gpu'] for _, di in ranks) == [3, 4, 5, 6, 7]
    assert all(di['visible_gpus'] == '3,4,5,6,7' for _, di in ranks)
    assert [di['local_rank'] for _, di in ranks] == [0, 1, 2, 3, 4]
    # nothing is free any more: a second GPU task waits
    more = _dag(s, {'late': {'type': 'bash', 'command': 'true', 'gpu': 1}})['late'][0]
    sup.build()
    assert _tasks(s, id=more)[0].status == TaskStatus.NotRan.value


def test_master_ports_taken_and_reused(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1')
    a = _dag(s, {'a': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': True}})['a'][0]
    c = _dag(s, {'c': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': True}})['c'][0]
    sup.build()
    pa = {di['master_port'] for _, di in _ranks(s, a)}
    pc = {di['master_port'] for _, di in _ranks(s, c)}
    assert pa == {29500} and pc == {29501}
    for k, _ in _ranks(s, a):                      # job a finishes: its port is free again
        k.status = TaskStatus.Success.value
    s.commit()
    sup.build()
    d = _dag(s, {'d': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': True}})['d'][0]
    sup.build()
    assert {di['master_port'] for _, di in _ranks(s, d)} == {29500}
    assert _tasks(s, id=a)[0].status == TaskStatus.Success.value


def test_multi_branch_4_plus_4_packs_numa_halves(sched):
    """BASELINE config 5 (examples/multi_branch): ResNet-50 and BERT ranks side by side,
    each rank set on one half of the node (one socket / NUMA domain)."""
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1')
    ids = _dag(s, {'resnet50': {'type': 'bash', 'command': 'true', 'gpu': 4, 'distr': True, 'single_node': True},
                   'bert': {'type': 'bash', 'command': 'true', 'gpu': 4, 'distr': True, 'single_node': True}})
    sup.build()
    sets = []
    for name in ('resnet50', 'bert'):
        ranks = _ranks(s, ids[name][0])
        assert len(ranks) == 4 and [di['local_rank'] for _, di in ranks] == [0, 1, 2, 3]
        sets.append(sorted(di['gpu'] for _, di in ranks))
        assert ranks[0][1]['visible_gpus'] == ','.join(map(str, sets[-1]))
    assert sorted(sets) == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert len(_drain(b, 'node1_default')) == 8


def test_single_node_job_needs_one_computer(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'a', gpu=4)
    _computer(s, 'b', gpu=4)
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 8, 'distr': True, 'single_node': True}})['t'][0]
    sup.build()
    assert _ranks(s, tid) == [] and _tasks(s, id=tid)[0].status == TaskStatus.NotRan.value


def test_multi_node_ranks_span_computers(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'a', gpu=4, ip='10.1.0.1')
    _computer(s, 'b', gpu=4, ip='10.1.0.2')
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 8, 'distr': True, 'single_node': False}})['t'][0]
    sup.build()
    ranks = _ranks(s, tid)
    assert len(ranks) == 8 and [di['rank'] for _, di in ranks] == list(range(8))
    master = ranks[0][1]['master_computer']
    other = 'b' if master == 'a' else 'a'
    for k, di in ranks:
        assert di['world_size'] == 8 and di['master_computer'] == master
        assert di['visible_gpus'] == '0,1,2,3' and di['local_rank'] == di['gpu']
        if k.computer_assigned == master:
            assert di['master_addr'] == '127.0.0.1'
        else:
            assert di['master_addr'] == ('10.1.0.1' if master == 'a' else '10.1.0.2')
    assert sum(k.computer_assigned == other for k, _ in ranks) == 4
    assert len(_drain(b, 'a_default')) == 4 and len(_drain(b, 'b_default')) == 4


def test_plain_gpu_task_gets_a_half(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1')
    ids = _dag(s, {'x': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': False},
                   'y': {'type': 'bash', 'command': 'true', 'gpu': 3, 'distr': False}})
    sup.build()
    gx = [int(g) for g in _tasks(s, id=ids['x'][0])[0].gpu_assigned.split(',')]
    gy = [int(g) for g in _tasks(s, id=ids['y'][0])[0].gpu_assigned.split(',')]
    assert not set(gx) & set(gy)
    assert len({g // 4 for g in gx}) == 1 and len({g // 4 for g in gy}) == 1   # each inside one half


def test_dead_queue_is_not_a_target(sched):
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'dead', alive=False)
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 1}})['t'][0]
    sup.build()
    assert _tasks(s, id=tid)[0].status == TaskStatus.NotRan.value
    assert b.queue_len('dead_default') == 0


def test_lost_message_requeues_task_and_frees_gpus(sched, monkeypatch):
    """A broker restart without its journal: the Queued task's message is gone.  After
    ORPHAN_SECONDS the task is placed again (new message) instead of holding its GPUs."""
    from mlcomp_amd.server import supervisor as S
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1', gpu=2)
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': False}})['t'][0]
    sup.build()
    t = _tasks(s, id=tid)[0]
    old = t.celery_id
    assert t.status == TaskStatus.Queued.value and b.has(old)
    b.revoke(old)                                   # the broker lost it
    sup.build()                                     # suspect, inside the grace period
    assert _tasks(s, id=tid)[0].celery_id == old
    monkeypatch.setattr(S, 'ORPHAN_SECONDS', 0)
    sup.build()                                     # reset to NotRan, then placed again
    t = _tasks(s, id=tid)[0]
    assert t.status == TaskStatus.Queued.value and t.celery_id != old and b.has(t.celery_id)
    assert t.gpu_assigned == '0,1'


def test_dead_queue_after_dispatch_releases_gpus(sched, monkeypatch):
    from mlcomp_amd.db.models import Docker
    from mlcomp_amd.server import supervisor as S
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'n1', gpu=2)
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 2, 'distr': False}})['t'][0]
    sup.build()
    assert _tasks(s, id=tid)[0].computer_assigned == 'n1'
    d = s.query(Docker).filter(Docker.computer == 'n1').one()
    d.last_activity = d.last_activity - datetime.timedelta(minutes=5)   # n1 dies
    s.commit()
    monkeypatch.setattr(S, 'ORPHAN_SECONDS', 0)
    sup.build()
    t = _tasks(s, id=tid)[0]
    assert t.status == TaskStatus.NotRan.value and t.gpu_assigned is None and t.computer_assigned is None
    assert b.queue_len('n1_default') == 0           # the stale message was revoked
    _computer(s, 'n2', gpu=2)                       # a live node takes it
    sup.build()
    t = _tasks(s, id=tid)[0]
    assert t.status == TaskStatus.Queued.value and t.computer_assigned == 'n2'


def test_lost_rank_message_fails_and_restarts_the_dag(sched, monkeypatch):
    from mlcomp_amd.server import supervisor as S
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1', gpu=2)
    tid = _dag(s, {'t': {'type': 'catalyst', 'gpu': 2, 'distr': True}})['t'][0]
    sup.build()
    ranks = _ranks(s, tid)
    assert len(ranks) == 2
    b.revoke(ranks[1][0].celery_id)
    monkeypatch.setattr(S, 'ORPHAN_SECONDS', 0)
    sup.build()     # rank 1 Failed (orphan); rank 0 is Queued fine
    assert _tasks(s, id=ranks[1][0].id)[0].status == TaskStatus.Failed.value
    sup.build()     # parent Failed -> siblings stopped -> fatal-restart matcher -> start_dag
    sup.build()     # the start command is processed: the parent is NotRan again
    parent = _tasks(s, id=tid)[0]
    info = yaml_load(parent.additional_info)
    assert info.get('auto_restarts') == 1
    assert parent.status in (TaskStatus.NotRan.value, TaskStatus.Queued.value)


@pytest.mark.parametrize('line, restart', [
    ('RCCL version 2.22.3+hip6.4 HEAD:abc', False),
    ('NCCL INFO Using network Socket (RCCL)', False),
    ('RuntimeError: NCCL error in: ProcessGroupNCCL.cpp:1970, ncclSystemError: System call (e.g. socket, '
     'malloc) or external library call failed', True),
    ('Memory access fault by GPU node-2 (Agent handle: 0x5f) on address 0x7f. Reason: Unknown.', True),
    ('HIP error: an illegal memory access was encountered', True),
])
def test_fatal_restart_matches_whole_messages(sched, line, restart):
    from mlcomp_amd.db.enums import ComponentType, LogStatus
    from mlcomp_amd.db.models import Log, now
    s, sup = sched['s'], sched['sup']
    tid = _dag(s, {'t': {'type': 'catalyst', 'gpu': 2, 'distr': True}})['t'][0]
    parent = _tasks(s, id=tid)[0]
    parent.status = TaskStatus.InProgress.value      # a running DDP job ...
    from mlcomp_amd.db.models import Task
    child = Task(name='t', executor='t', status=TaskStatus.Failed.value, type=TaskType.Service.value,
                 parent=tid, dag=parent.dag, gpu=1, gpu_max=1, debug=False, continued=False)   # ... rank died
    s.add(child)
    s.commit()
    s.add(Log(message=line, time=now(), level=LogStatus.Error.value, component=ComponentType.Worker.value,
              task=child.id))
    s.commit()
    sup.build()
    sup.build()
    info = yaml_load(_tasks(s, id=tid)[0].additional_info) or {}
    assert bool(info.get('auto_restarts')) == restart


def test_rank_process_sees_the_job_gpus(sched, monkeypatch):
    """The worker side of the fan-out: each rank's task process gets HIP_VISIBLE_DEVICES =
    the job's GPUs on its computer (mapped through the worker's own mask) and the train
    executor selects its device by local_rank."""
    import os
    from mlcomp_amd.worker.tasks import ExecuteBuilder
    s, sup = sched['s'], sched['sup']
    _computer(s, 'node1')
    tid = _dag(s, {'t': {'type': 'bash', 'command': 'true', 'gpu': 4, 'distr': True}})['t'][0]
    sup.build()
    ranks = _ranks(s, tid)
    k, di = ranks[2]
    monkeypatch.setenv('HIP_VISIBLE_DEVICES', '7,6,5,4,3,2,1,0')     # the worker's own mask
    monkeypatch.setenv('CUDA_VISIBLE_DEVICES', '7,6,5,4,3,2,1,0')
    eb = ExecuteBuilder(k.id)
    eb.create_base()
    want = ','.join('76543210'[int(g)] for g in di['visible_gpus'].split(','))
    assert os.environ['HIP_VISIBLE_DEVICES'] == want and len(want.split(',')) == 4
    assert di['local_rank'] == 2


def test_rccl_transport_summary():
    from mlcomp_amd.parallel.comm import transport_summary
    log = '\n'.join([
        'node:123:456 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC',
        'node:123:456 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC comm 0x1 nRanks 02',
        'node:123:456 [0] NCCL INFO Channel 02/0 : 1[1] -> 0[0] via SHM/direct/direct',
        'node:123:456 [0] NCCL INFO Connected all rings',
        'node:123:456 [0] NCCL INFO RCCL version 2.22.3 via nothing',
    ])
    assert transport_summary(log) == {'P2P/IPC': 2, 'SHM/direct/direct': 1}


def test_straggler_is_marked_before_the_kill_and_not_reported_lost(sched, monkeypatch):
    """A Train parent with one rank finished and one still running (a DDP hang): the
    straggler is Success (and flagged) BEFORE its kill is sent, so the worker that sees its
    process die with a non-zero code does not fail it as a lost process (which would make
    the fatal-restart matcher restart a finished DAG)."""
    from mlcomp_amd.server import supervisor as S
    from mlcomp_amd.worker.daemon import WorkerPool
    from mlcomp_amd.db.models import now
    s, sup, b = sched['s'], sched['sup'], sched['broker']
    _computer(s, 'node1', gpu=2)
    tid = _dag(s, {'t': {'type': 'catalyst', 'gpu': 2, 'distr': True}})['t'][0]
    sup.build()
    (r0, _), (r1, _) = _ranks(s, tid)
    r0.status, r0.finished = TaskStatus.Success.value, now() - datetime.timedelta(minutes=10)
    r1.status, r1.pid = TaskStatus.InProgress.value, 424242
    s.commit()
    monkeypatch.setattr(S, 'STRAGGLER_SECONDS', 0)
    seen = {}

    def call(queue, name, *args, timeout=None):
        seen['status'] = _tasks(s, id=r1.id)[0].status        # the state the dying worker will read
        return True
    monkeypatch.setattr(b, 'call', call, raising=False)
    sup.build()
    assert seen['status'] == TaskStatus.Success.value
    WorkerPool([0])._process_lost(0, r1.id, -9)
    t = _tasks(s, id=r1.id)[0]
    assert t.status == TaskStatus.Success.value
    assert yaml_load(t.additional_info).get('killed_by_supervisor')
    sup.build()
    assert not (yaml_load(_tasks(s, id=tid)[0].additional_info) or {}).get('auto_restarts')
