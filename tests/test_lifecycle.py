"""End-to-end DAG lifecycle on CPU: YAML -> DB rows -> scheduler tick -> native broker
-> worker pool -> task process -> executors -> Success/Failed/Skipped, logs and steps.
(The reference has no integration tests; SURVEY.md 7.4 asks for exactly this.)"""
import os
import socket
import subprocess
import time

import pytest
import yaml


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def cluster(mlc_root, monkeypatch, tmp_path):
    from mlcomp_amd.build import build_broker
    port = _free_port()
    proc = subprocess.Popen([build_broker(), '--port', str(port)], stdout=subprocess.PIPE)
    proc.stdout.readline()
    monkeypatch.setenv('BROKER_PORT', str(port))
    monkeypatch.setenv('MLCOMP_COMPUTER', 'testhost')
    monkeypatch.setenv('MLCOMP_BROKER', '')
    from mlcomp_amd import config, broker
    config.reset()
    broker.set_broker(None)
    from mlcomp_amd.db.migrate import migrate
    migrate()
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.worker.daemon import WorkerPool, WorkerSupervisor
    from mlcomp_amd.server.supervisor import SupervisorBuilder
    ws = WorkerSupervisor(liveness_period=1.0, grace=1.0)
    ws.heartbeat()
    pool = WorkerPool([0, 1], poll=0.2).start()
    sup = SupervisorBuilder(session_key='test-sup')
    yield {'sup': sup, 'ws': ws, 'tmp': tmp_path}
    pool.stop()
    proc.kill()
    proc.wait()
    broker.set_broker(None)
    Session.cleanup()


def _submit(tmp, cfg: dict, files=None):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.dag import dag_from_config
    d = tmp / f'proj{time.time_ns()}'
    d.mkdir()
    for name, content in (files or {}).items():
        (d / name).write_text(content)
    path = d / 'config.yml'
    path.write_text(yaml.safe_dump(cfg))
    s = Session.create_session(key='client')
    return dag_from_config(s, cfg, config_path=str(path), config_text=path.read_text())


def _wait(sup, task_ids, timeout=60):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.providers import TaskProvider
    s = Session.create_session(key='poll')
    deadline = time.time() + timeout
    while time.time() < deadline:
        sup.build()
        s.expire_all()
        ts = TaskProvider(s).by_ids(task_ids)
        if all(t.status >= TaskStatus.Failed.value for t in ts):
            return {t.id: TaskStatus(t.status) for t in ts}
        time.sleep(0.2)
    s.expire_all()
    return {t.id: TaskStatus(t.status) for t in TaskProvider(s).by_ids(task_ids)}


def test_bash_success_logs_and_steps(cluster):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.providers import LogProvider, StepProvider
    created = _submit(cluster['tmp'], {'info': {'name': 'bash', 'project': 'examples'},
                                       'executors': {'bash': {'type': 'bash',
                                                              'command': 'echo hello-$who && echo done',
                                                              'who': 'mi355x'}}})
    tid = created[0]['bash'][0]
    st = _wait(cluster['sup'], [tid])
    assert st[tid] == TaskStatus.Success
    s = Session.create_session(key='check')
    msgs = [l['message'] for l in LogProvider(s).get({'task': tid})['data']]
    assert any('hello-mi355x' in m for m in msgs)
    tree = StepProvider(s).get(tid)
    assert tree and tree[0]['name'] == 'main'


def test_failure_skips_dependents_and_grid(cluster):
    from mlcomp_amd.db.enums import TaskStatus
    created = _submit(cluster['tmp'], {
        'info': {'name': 'err', 'project': 'examples'},
        'executors': {
            'bad': {'type': 'bash', 'command': 'python -c "raise SystemExit(3)"'},
            'after': {'type': 'bash', 'command': 'echo never', 'depends': 'bad'},
            'grid': {'type': 'bash', 'command': 'echo $v', 'grid': [{'v': '0-2'}]},
        }})[0]
    ids = created['bad'] + created['after'] + created['grid']
    assert len(created['grid']) == 3
    st = _wait(cluster['sup'], ids)
    assert st[created['bad'][0]] == TaskStatus.Failed
    assert st[created['after'][0]] == TaskStatus.Skipped
    assert all(st[i] == TaskStatus.Success for i in created['grid'])


USER_EXECUTOR = '''
import time
from mlcomp_amd.worker.executors import Executor


@Executor.register
class Steps(Executor):
    def work(self):
        self.step.start(1, 'step 1')
        self.step.start(1, 'step 2')
        self.step.start(2, 'step 2.1')
        for _ in self.tqdm(range(20), interval=0):
            pass
        self.info('user message')
        self.step.end(0)
        return {'ok': 1}
'''


def test_user_executor_hierarchical_steps(cluster):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.providers import StepProvider, TaskProvider
    created = _submit(cluster['tmp'], {'info': {'name': 'steps', 'project': 'examples'},
                                       'executors': {'s': {'type': 'steps'}}},
                      files={'executors.py': USER_EXECUTOR})[0]
    tid = created['s'][0]
    st = _wait(cluster['sup'], [tid])
    assert st[tid] == TaskStatus.Success
    s = Session.create_session(key='check2')
    t = TaskProvider(s).by_id(tid)
    assert yaml.safe_load(t.result) == {'ok': 1}
    assert t.batch_index == 20 and t.batch_total == 20
    tree = StepProvider(s).get(tid)
    names = [c['name'] for c in tree[0]['children']]
    assert names == ['step 1', 'step 2']
    assert tree[0]['children'][1]['children'][0]['name'] == 'step 2.1'


def test_stop_running_task(cluster):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.providers import TaskProvider
    created = _submit(cluster['tmp'], {'info': {'name': 'sleep', 'project': 'examples'},
                                       'executors': {'s': {'type': 'bash', 'command': 'sleep 60'}}})[0]
    tid = created['s'][0]
    s = Session.create_session(key='check3')
    deadline = time.time() + 30
    while time.time() < deadline:
        cluster['sup'].build()
        s.expire_all()
        if TaskProvider(s).by_id(tid).status == TaskStatus.InProgress.value:
            break
        time.sleep(0.2)
    time.sleep(1.0)
    cluster['sup'].stop_tasks([tid])
    cluster['sup'].build()
    s.expire_all()
    assert TaskProvider(s).by_id(tid).status == TaskStatus.Stopped.value
