"""REST API (dispatch + HTTP layer), CLIs and the process manager, on CPU."""
import json
import os
import sys
import time

import pytest
import yaml
from click.testing import CliRunner


@pytest.fixture
def db(mlc_root, monkeypatch):
    monkeypatch.setenv('MLCOMP_COMPUTER', 'apihost')
    from mlcomp_amd import broker, config
    config.reset()
    broker.set_broker(broker.InProcBroker())
    from mlcomp_amd.db.migrate import migrate
    migrate()
    import mlcomp_amd.server.api as api
    api._CTX = None
    yield api
    api._CTX = None
    broker.set_broker(None)
    from mlcomp_amd.db.core import Session
    Session.cleanup()


def _tok():
    from mlcomp_amd import config
    return config.get().TOKEN


def _call(api, name, data=None, token=True):
    st, res = api.dispatch(name, data if data is not None else {}, _tok() if token else 'wrong')
    return st, res


def _make_dag(tmp_path, name='d1'):
    from mlcomp_amd.dag import dag_from_config
    from mlcomp_amd.db.core import Session
    d = tmp_path / name
    d.mkdir()
    (d / 'a.py').write_text('print(1)\n')
    (d / 'sub').mkdir()
    (d / 'sub' / 'b.txt').write_text('hello')
    cfg = {'info': {'name': name, 'project': 'papi', 'layout': 'classify'},
           'executors': {'prep': {'type': 'bash', 'command': 'echo 1'},
                         'train': {'type': 'catalyst', 'depends': 'prep', 'args': {'config': 'x.yml'}}}}
    cwd = os.getcwd()
    os.chdir(d)
    try:
        (d / 'config.yml').write_text(yaml.safe_dump(cfg))
        return dag_from_config(Session.create_session(key='t'), cfg, config_path=str(d / 'config.yml'),
                               config_text=yaml.safe_dump(cfg))
    finally:
        os.chdir(cwd)


def test_auth_and_envelope(db):
    st, res = _call(db, 'projects', {'paginator': {}}, token=False)
    assert st == 401 and res['success'] is False
    assert _call(db, 'token', {'token': 'nope'})[0] == 401
    assert _call(db, 'token', {'token': _tok()})[0] == 200
    st, res = _call(db, 'no/such/endpoint')
    assert st == 404
    st, res = _call(db, 'task/info', {'id': 123456})   # handler error -> 500 + traceback
    assert st == 500 and res['success'] is False and 'Traceback' in res['error']


def test_projects_dags_tasks_code(db, tmp_path):
    _make_dag(tmp_path)
    st, res = _call(db, 'projects', {'paginator': {'page_size': 10}})
    assert st == 200 and res['success'] and any(p['name'] == 'papi' for p in res['data'])
    st, res = _call(db, 'dags', {'paginator': {'page_size': 10}})
    assert st == 200 and res['total'] == 1
    dag_id = res['data'][0]['id']
    st, res = _call(db, 'tasks', {'dag': dag_id, 'paginator': {}})
    assert st == 200 and res['total'] == 2
    tid = res['data'][0]['id']
    assert _call(db, 'task/info', {'id': tid})[1]['id'] == tid
    g = _call(db, 'graph', dag_id)[1]
    assert len(g['nodes']) == 2 and len(g['edges']) == 1
    assert 'executors' in _call(db, 'config', dag_id)[1]['data']
    code = _call(db, 'code', dag_id)[1]['items']
    names = [n['name'] for n in code]
    assert names[0] == 'sub' and 'a.py' in names          # folders first
    sub = code[0]
    assert sub['children'][0]['content'] == 'hello'
    # edit a file in place
    a = [n for n in code if n['name'] == 'a.py'][0]
    assert _call(db, 'update_code', {'file_id': a['id'], 'content': 'print(2)\n', 'dag': dag_id,
                                     'storage': a['storage']})[0] == 200
    code2 = _call(db, 'code', dag_id)[1]['items']
    assert [n for n in code2 if n['name'] == 'a.py'][0]['content'] == 'print(2)\n'
    # stop the DAG: NotRan tasks become Skipped
    st, res = _call(db, 'dag/stop', {'id': dag_id})
    assert st == 200, res
    from mlcomp_amd.server.supervisor import SupervisorBuilder
    db.ctx().supervisor.build()
    st, res = _call(db, 'tasks', {'dag': dag_id, 'paginator': {}})
    assert {t['status'] for t in res['data']} <= {'skipped', 5}
    # restart = copy of the DAG
    st, res = _call(db, 'dag/restart', {'dag': dag_id, 'file_changes': ''})
    assert st == 200
    assert _call(db, 'dags', {'paginator': {}})[1]['total'] == 2


def test_layouts_memory_spaces_reports(db, tmp_path):
    assert 'classify' in [l['name'] for l in _call(db, 'layouts', {'paginator': {}})[1]['data']]
    assert _call(db, 'layout/add', {'name': 'mine'})[0] == 200
    bad = _call(db, 'layout/edit', {'name': 'mine', 'content': 'items: {x: {type: nope}}'})
    assert bad[0] == 500
    ok = _call(db, 'layout/edit', {'name': 'mine', 'content': 'extend: base\nmetric: {name: dice, minimize: false}'})
    assert ok[0] == 200, ok
    assert _call(db, 'layout/remove', {'name': 'mine'})[0] == 200

    assert _call(db, 'memory/add', {'model': 'resnet50', 'memory': 20.5, 'batch_size': 256, 'img_size': 224})[0] == 200
    mem = _call(db, 'memories', {'paginator': {}})[1]['data']
    assert mem[0]['batch_size'] == 256
    _call(db, 'memory/edit', dict(mem[0], batch_size=512))
    assert _call(db, 'memories', {'paginator': {}})[1]['data'][0]['batch_size'] == 512
    _call(db, 'memory/remove', {'id': mem[0]['id']})
    assert _call(db, 'memories', {'paginator': {}})[1]['total'] == 0

    created = _make_dag(tmp_path, 'sp')
    dag_id = _call(db, 'dags', {'paginator': {}})[1]['data'][0]['id']
    _call(db, 'space/add', {'name': 'lr', 'content': 'x.yml:\n  lr: 0.1\n'})
    _call(db, 'space/add', {'name': 'lr2', 'content': 'x.yml:\n  lr: 0.2\n'})
    _call(db, 'space/relation_append', {'parent': 'lr', 'child': 'lr2'})
    _call(db, 'space/tag_add', {'space': 'lr', 'tag': 'sweep'})
    assert _call(db, 'space/tags', {'name': 'sw'})[1]['data'] == ['sweep']
    st, res = _call(db, 'space/run', {'dag': dag_id, 'spaces': [{'logic': 'or', 'value': 'lr'}]})
    assert st == 200 and len(res['dags']) == 2, res          # lr2 (related) + lr itself

    st, res = _call(db, 'report/add_start', {})
    pid = res['projects'][0]['id']
    assert _call(db, 'report/add_end', {'name': 'r1', 'project': pid, 'layout': 'classify'})[0] == 200
    reps = _call(db, 'reports', {'paginator': {}})[1]['data']
    rid = [r for r in reps if r['name'] == 'r1'][0]['id']
    tid = _call(db, 'tasks', {'paginator': {}})[1]['data'][0]['id']
    _call(db, 'task/toogle_report', {'id': tid, 'report': rid})
    det = _call(db, 'report', rid)[1]
    assert det['layout_name'] == 'classify' and len(det['tasks']) == 1
    assert 'scheduler' in json.dumps(_call(db, 'auxiliary')[1]) or _call(db, 'auxiliary')[0] == 200


def test_http_layer(db, tmp_path):
    from fastapi.testclient import TestClient
    c = TestClient(db.create_app())
    assert c.post('/api/projects', json={'paginator': {}}).status_code == 401
    r = c.post('/api/projects', json={'paginator': {}}, headers={'Authorization': _tok()})
    assert r.status_code == 200 and r.json()['success']
    assert c.post('/api/token', json={'token': _tok()}).status_code == 200
    html = c.get('/').text
    assert '<title>mlcomp_amd</title>' in html
    _make_dag(tmp_path, 'zz')
    dag_id = c.post('/api/dags', json={'paginator': {}}, headers={'Authorization': _tok()}).json()['data'][0]['id']
    z = c.get(f'/api/code_download?id={dag_id}', headers={'Authorization': _tok()})
    assert z.status_code == 200 and z.content[:2] == b'PK'


def test_cli_commands(mlc_root, monkeypatch, tmp_path):
    monkeypatch.setenv('MLCOMP_COMPUTER', 'clihost')
    from mlcomp_amd import broker, config
    config.reset()
    broker.set_broker(broker.InProcBroker())
    from mlcomp_amd.__main__ import main
    r = CliRunner()
    assert r.invoke(main, ['migrate']).exit_code == 0
    out = r.invoke(main, ['status'])
    assert 'database' in out.output and 'ok' in out.output
    d = tmp_path / 'proj'
    d.mkdir()
    (d / 'config.yml').write_text(yaml.safe_dump(
        {'info': {'name': 'cli', 'project': 'pcli'},
         'executors': {'a': {'type': 'bash', 'command': f'echo $msg > {d / "out.txt"}', 'msg': 'hi'}}}))
    res = r.invoke(main, ['dag', str(d / 'config.yml'), '--params', 'executors/a/msg:yo'])
    assert res.exit_code == 0, res.output
    res = r.invoke(main, ['execute', str(d / 'config.yml')])
    assert res.exit_code == 0, (res.output, res.exception)
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.models import Task
    s = Session.create_session(key='clichk')
    ts = s.query(Task).order_by(Task.id).all()
    assert len(ts) == 2 and ts[-1].status == 6, [(t.id, t.status) for t in ts]
    res = r.invoke(main, ['report'])
    assert res.exit_code == 0
    assert os.path.exists(os.path.join(config.get().REPORT_FOLDER, 'report.zip'))
    broker.set_broker(None)
    Session.cleanup()


def test_contrib_split_cli(tmp_path, monkeypatch):
    from mlcomp_amd.contrib.__main__ import main
    img = tmp_path / 'img'
    for lab in ('cat', 'dog'):
        (img / lab).mkdir(parents=True)
        for i in range(6):
            (img / lab / f'{lab}{i}.png').write_bytes(b'x')
    monkeypatch.chdir(tmp_path)
    res = CliRunner().invoke(main, ['split-classify', str(img), '--n_splits', '3'])
    assert res.exit_code == 0, res.output
    import pandas as pd
    df = pd.read_csv(tmp_path / 'fold.csv')
    assert len(df) == 12 and sorted(df['fold'].unique()) == [0, 1, 2]
    res = CliRunner().invoke(main, ['split-test-img', str(img / 'cat')])
    assert res.exit_code == 0
    assert len(pd.read_csv(tmp_path / 'fold_test.csv')) == 6


def test_process_manager_restarts_and_stops(tmp_path):
    import threading
    from mlcomp_amd.utils.procman import Program, ProcessManager, read_status, stop_manager
    flag = tmp_path / 'runs'
    code = f"open({str(flag)!r}, 'a').write('x'); import time; time.sleep(0.3)"
    p = Program('flaky', [sys.executable, '-c', code])
    keep = Program('steady', [sys.executable, '-c', 'import time; time.sleep(60)'])
    pm = ProcessManager([p, keep], str(tmp_path), 'test')
    import signal as _s
    orig = _s.signal
    t = threading.Thread(target=pm.run, kwargs={'poll': 0.1, 'grace': 2.0}, daemon=True)
    # signal handlers can only be installed from the main thread: stub them for the test
    _s.signal = lambda *a, **k: None
    try:
        t.start()
        deadline = time.time() + 15
        while time.time() < deadline and (not flag.exists() or len(flag.read_text()) < 3):
            time.sleep(0.1)
    finally:
        _s.signal = orig
    assert len(flag.read_text()) >= 3          # restarted at least twice
    st = read_status(str(tmp_path), 'test')
    assert st and any(x['name'] == 'steady' and x['alive'] for x in st['programs'])
    pm._stop = True
    t.join(10)
    assert not keep.alive()
    assert read_status(str(tmp_path), 'test') is None
