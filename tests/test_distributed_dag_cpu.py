"""A data-parallel training DAG end to end on CPU (gloo): the reference's
``digit-recognizer/train-distr.yml`` and ``train-distr-stage.yml`` through the real
scheduler -> native broker -> worker pool -> one task process per rank.

The computer reports 2 "GPUs" (MLCOMP_GPU_COUNT), so the scheduler fans the train task out
into one Service child per rank (`mlcomp/server/back/supervisor.py:252-343`); each rank
process finds no HIP device and joins a gloo process group (`catalyst_.py:214-236`).
Checked: distr_info per rank, identical final weights (per-rank digest lines), rank-0-only
checkpoints and report series (`catalyst_.py:349-363`), the stage-2 requeue resuming from
rank 0's checkpoint (`master_task_id = task.id - rank`, `catalyst_.py:407-421`,
`mlcomp/worker/tasks.py:237-258`), the parent reaching Success, and a killed rank failing
the DAG, stopping the straggler and restarting a bounded number of times."""
import os
import random
import re
import shutil
import socket
import subprocess
import threading
import time

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, 'examples', 'digit-recognizer')
SMALL = {'executors/train/params/stages/data_params/max_count': 512,
         'executors/train/params/stages/data_params/batch_size': 64}


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def dcluster(mlc_root, monkeypatch, tmp_path, request):
    world = getattr(request, 'param', 2)
    from mlcomp_amd.build import build_broker
    port = _free_port()
    proc = subprocess.Popen([build_broker(), '--port', str(port)], stdout=subprocess.PIPE)
    proc.stdout.readline()
    base = random.randrange(31000, 60000, 16)
    monkeypatch.setenv('BROKER_PORT', str(port))
    monkeypatch.setenv('MLCOMP_COMPUTER', 'ddphost')
    monkeypatch.setenv('MLCOMP_BROKER', '')
    monkeypatch.setenv('MLCOMP_GPU_COUNT', str(world))
    monkeypatch.setenv('MASTER_PORT_RANGE', f'{base}-{base + 15}')
    monkeypatch.setenv('OMP_NUM_THREADS', '1')
    from mlcomp_amd import config, broker
    config.reset()
    broker.set_broker(None)
    from mlcomp_amd.db.migrate import migrate
    migrate()
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.server.supervisor import SupervisorBuilder
    from mlcomp_amd.worker.daemon import WorkerPool, WorkerSupervisor
    ws = WorkerSupervisor(liveness_period=1.0, grace=1.0)
    ws.heartbeat()
    control = threading.Thread(target=ws._control, daemon=True)   # kill / kill_all requests
    control.start()
    pool = WorkerPool(list(range(world + 1)), poll=0.2).start()
    sup = SupervisorBuilder(session_key='ddp-sup')
    yield {'sup': sup, 'ws': ws, 'tmp': tmp_path, 'world': world}
    ws.stop()
    pool.stop()
    proc.kill()
    proc.wait()
    broker.set_broker(None)
    Session.cleanup()


def _dag(tmp, name, params=None):
    from mlcomp_amd.dag import dag_from_config
    from mlcomp_amd.db.core import Session
    dst = tmp / f'dr_{len(os.listdir(tmp))}'
    if not dst.exists():
        shutil.copytree(EX, dst)
    cfg_path = dst / name
    text = cfg_path.read_text()
    cwd = os.getcwd()
    os.chdir(dst)
    try:
        created = dag_from_config(Session.create_session(key='ddp-client'), yaml.safe_load(text),
                                  config_path=str(cfg_path), config_text=text, params=params)
    finally:
        os.chdir(cwd)
    return [i for d in created for ids in d.values() for i in ids]


def _tick_until(c, ids, timeout, done=None):
    """Run scheduler ticks (and the worker supervisor's heartbeat + liveness scan) until
    every task in ``ids`` is finished, or ``done()`` says so."""
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.providers import TaskProvider
    s = Session.create_session(key='ddp-poll')
    deadline = time.time() + timeout
    while time.time() < deadline:
        c['ws'].heartbeat()
        c['ws'].stop_processes_not_exist()
        c['sup'].build()
        s.expire_all()
        ts = TaskProvider(s).by_ids(ids)
        if done is not None and done(s):
            break
        if done is None and all(t.status >= TaskStatus.Failed.value for t in ts):
            break
        time.sleep(0.3)
    s.expire_all()
    return s, {t.id: TaskStatus(t.status) for t in TaskProvider(s).by_ids(ids)}


def _prepare(c):
    from mlcomp_amd.db.enums import TaskStatus
    ids = _dag(c['tmp'], 'prepare.yml')
    _, res = _tick_until(c, ids, 180)
    assert all(v == TaskStatus.Success for v in res.values()), res


def _children(s, parent):
    from mlcomp_amd.db.providers import TaskProvider
    return sorted(TaskProvider(s).children(parent), key=lambda t: t.id)


def _logs(s, task_id):
    from mlcomp_amd.db.models import Log
    return [l.message for l in s.query(Log).filter(Log.task == task_id).order_by(Log.id)]


def _digests(s, task_id):
    out = {}
    for m in _logs(s, task_id):
        g = re.search(r'rank (\d+) of (\d+): stage (\S+) weights digest ([0-9a-f]+)', m)
        if g:
            out[g.group(3)] = g.group(4)
    return out


def _check_ranks(s, parent, world):
    from mlcomp_amd.db.enums import TaskType
    from mlcomp_amd.utils.misc import yaml_load
    kids = _children(s, parent)
    assert len(kids) == world
    first = kids[0].id
    for r, k in enumerate(kids):
        assert k.type == TaskType.Service.value
        di = yaml_load(k.additional_info)['distr_info']
        assert di['rank'] == r and di['world_size'] == world and di['master_addr'] == '127.0.0.1'
        assert di['local_rank'] == r and di['visible_gpus'] == ','.join(map(str, range(world)))
        assert k.gpu_assigned == str(r)
        assert yaml_load(k.additional_info)['resume']['master_task_id'] == first
    return kids


def _checkpoints(task_id):
    from mlcomp_amd import config
    d = os.path.join(config.get().TASK_FOLDER, str(task_id), 'log', 'checkpoints')
    return os.path.isdir(d) and any(f.endswith('.pth') for f in os.listdir(d))


@pytest.mark.parametrize('dcluster', [2, 4], indirect=True)
def test_distributed_train_dag_runs_on_gloo(dcluster):
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import ReportSeries, Task
    _prepare(dcluster)
    ids = _dag(dcluster['tmp'], 'train-distr.yml', params=SMALL)
    (parent,) = ids
    s, res = _tick_until(dcluster, ids, 300)
    assert res[parent] == TaskStatus.Success, (res, [(k.id, k.status, _logs(s, k.id)[-3:])
                                                   for k in _children(s, parent)])
    world = dcluster['world']
    kids = _check_ranks(s, parent, world)
    assert all(k.status == TaskStatus.Success.value for k in kids)
    ds = [_digests(s, k.id) for k in kids]
    assert ds[0] and all(d == ds[0] for d in ds), ds     # identical weights on every rank
    assert _checkpoints(kids[0].id) and not any(_checkpoints(k.id) for k in kids[1:])
    series = s.query(ReportSeries).filter(ReportSeries.task.in_([parent] + [k.id for k in kids])).all()
    assert {r.task for r in series} == {parent}          # rank 0 reports, onto the parent
    per = {}
    for r in series:
        per[(r.part, r.name, r.epoch)] = per.get((r.part, r.name, r.epoch), 0) + 1
    assert per and max(per.values()) == 1, per            # one row per metric and epoch
    epochs = {r.epoch for r in series if r.name == 'loss'}
    assert len(epochs) == 3
    assert s.get(Task, parent).score is not None


def test_distributed_two_stage_dag_requeues_and_resumes(dcluster):
    from mlcomp_amd.db.enums import TaskStatus
    _prepare(dcluster)
    ids = _dag(dcluster['tmp'], 'train-distr-stage.yml', params=SMALL)
    (parent,) = ids
    s, res = _tick_until(dcluster, ids, 420)
    assert res[parent] == TaskStatus.Success, (res, [(k.id, k.status, _logs(s, k.id)[-3:])
                                                   for k in _children(s, parent)])
    kids = _check_ranks(s, parent, 2)
    d0, d1 = _digests(s, kids[0].id), _digests(s, kids[1].id)
    assert set(d0) == {'stage1', 'stage2'} and d0 == d1, (d0, d1)
    # stage 2 of rank 1 resumed from RANK 0's checkpoint folder
    first = kids[0].id
    resumed = [m for m in _logs(s, kids[1].id) if m.startswith('resuming from')]
    assert resumed and f'/{first}/' in resumed[0], resumed
    assert _checkpoints(first) and not _checkpoints(kids[1].id)
    assert s.get(type(kids[0]), parent).steps == 2


def test_killed_rank_fails_stops_straggler_and_restarts_boundedly(dcluster, monkeypatch):
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import Task
    from mlcomp_amd.server.supervisor import MAX_AUTO_RESTARTS
    from mlcomp_amd.utils.misc import yaml_load
    _prepare(dcluster)
    params = dict(SMALL)
    params['executors/train/env'] = {'MLC_FAULTS': 'kill_rank=1@2'}
    ids = _dag(dcluster['tmp'], 'train-distr.yml', params=params)
    (parent,) = ids

    def all_kids(s):   # every attempt's ranks (a restart marks the earlier ones continued)
        return s.query(Task).filter(Task.parent == parent).order_by(Task.id).all()

    def finished(s):
        t = s.get(Task, parent)
        kids = all_kids(s)
        return t.status == TaskStatus.Failed.value and len(kids) == 2 * (MAX_AUTO_RESTARTS + 1) \
            and all(k.status >= TaskStatus.Failed.value for k in kids)

    s, res = _tick_until(dcluster, ids, 480, done=finished)
    t = s.get(Task, parent)
    assert t.status == TaskStatus.Failed.value, res
    assert (yaml_load(t.additional_info) or {}).get('auto_restarts') == MAX_AUTO_RESTARTS
    kids = all_kids(s)
    assert len(kids) == 2 * (MAX_AUTO_RESTARTS + 1)      # every attempt fanned out again
    for k in kids:
        rank = yaml_load(k.additional_info)['distr_info']['rank']
        if rank == 1:
            assert k.status == TaskStatus.Failed.value
            assert any('task process was lost' in m for m in _logs(s, k.id))
        else:   # rank 0 blocked in a collective: stopped by the scheduler, not left hanging
            assert k.status in (TaskStatus.Stopped.value, TaskStatus.Failed.value), k.status
    # no rank process survives the DAG (the kill requests travel through the broker)
    import psutil

    def alive(pid):
        try:
            return psutil.Process(pid).status() != psutil.STATUS_ZOMBIE
        except psutil.Error:
            return False
    deadline = time.time() + 30
    while time.time() < deadline and any(alive(k.pid) for k in kids if k.pid):
        time.sleep(0.5)
    assert not [k.id for k in kids if k.pid and alive(k.pid)]
