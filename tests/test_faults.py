"""Fault injection (``mlcomp_amd.utils.faults``) and the recovery paths it
exercises: a killed rank, dropped heartbeats, a corrupt checkpoint, a killed task process
(InProgress + dead pid => Failed), a fatal-error crash string."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from mlcomp_amd.utils import faults


@pytest.fixture(autouse=True)
def _clean(monkeypatch):
    monkeypatch.delenv('MLC_FAULTS', raising=False)
    faults.reset()
    yield
    faults.reset()


def test_spec_parsing_and_noop(monkeypatch):
    assert faults.spec() == {}
    assert not faults.heartbeat_dropped()
    faults.maybe_kill_rank(0, 100)      # no-op without MLC_FAULTS
    monkeypatch.setenv('MLC_FAULTS', 'kill_rank=1@3, drop_heartbeat=2,corrupt_checkpoint')
    assert faults.spec() == {'kill_rank': '1@3', 'drop_heartbeat': '2', 'corrupt_checkpoint': ''}
    assert [faults.heartbeat_dropped() for _ in range(4)] == [True, True, False, False]


def _kill_worker(rank, world, port):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), MLC_FAULTS='kill_rank=1@2')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    for step in range(1, 5):
        faults.maybe_kill_rank(rank, step)
        t = torch.ones(4)
        dist.all_reduce(t)
    dist.destroy_process_group()


def test_kill_rank_terminates_the_job():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    with pytest.raises(mp.ProcessExitedException) as ei:
        mp.spawn(_kill_worker, args=(2, port), nprocs=2)
    assert ei.value.exit_code == 137 and ei.value.error_index == 1


def test_corrupt_checkpoint_falls_back(tmp_path, monkeypatch):
    from mlcomp_amd.train.callbacks import load_checkpoint, save_checkpoint
    good = {'stage': 's', 'checkpoint_data': {'epoch': 1}, 'model_state_dict': {'w': torch.ones(3)}}
    save_checkpoint(good, str(tmp_path / 'best_full.pth'))
    monkeypatch.setenv('MLC_FAULTS', 'corrupt_checkpoint')
    save_checkpoint(dict(good, stage='t'), str(tmp_path / 'last_full.pth'))
    with pytest.warns(UserWarning, match='unreadable checkpoint'):
        path, ck = load_checkpoint(str(tmp_path / 'last_full.pth'), str(tmp_path / 'best_full.pth'))
    assert path.endswith('best_full.pth') and ck['stage'] == 's'
    with pytest.warns(UserWarning):
        assert load_checkpoint(str(tmp_path / 'last_full.pth')) == (None, None)
    assert not [f for f in os.listdir(tmp_path) if '.tmp' in f]    # atomic writes leave no temp files


def test_train_executor_resume_skips_corrupt_last(tmp_path, monkeypatch):
    """fix_resume: a corrupt last_full.pth falls back to best_full.pth."""
    from types import SimpleNamespace
    from mlcomp_amd.train.callbacks import save_checkpoint
    from mlcomp_amd.worker.executors.train import Train
    ck = tmp_path / 'log' / 'checkpoints'
    ck.mkdir(parents=True)
    save_checkpoint({'stage': 'a', 'checkpoint_data': {'epoch': 0}, 'model_state_dict': {}}, str(ck / 'best_full.pth'))
    (ck / 'last_full.pth').write_bytes(b'not a checkpoint')
    msgs = []
    fake = SimpleNamespace(resume={'load_last': True}, info=msgs.append, error=msgs.append, session=None,
                           task=SimpleNamespace(id=1))
    exp = SimpleNamespace(logdir=str(tmp_path / 'log'),
                          stages_config={'a': {'state_params': {'num_epochs': 3}}, 'b': {}})
    with pytest.warns(UserWarning):
        start = Train.fix_resume(fake, exp)
    assert start == 1 and list(exp.stages_config) == ['a', 'b']
    assert fake.resume_path.endswith('best_full.pth') and any('unreadable' in m for m in msgs)


from test_lifecycle import _submit, _wait, cluster  # noqa: E402,F401


def _ids(created):
    c = created[0] if isinstance(created, (list, tuple)) else created
    return [t for ts in c.values() for t in ts]


def test_dropped_heartbeats_then_recover(cluster, monkeypatch):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.models import Docker
    ws = cluster['ws']
    s = Session.create_session(key='hb')
    before = {d.name: d.last_activity for d in s.query(Docker).all()}
    monkeypatch.setenv('MLC_FAULTS', 'drop_heartbeat=2')
    ws.heartbeat()
    ws.heartbeat()
    s.expire_all()
    assert {d.name: d.last_activity for d in s.query(Docker).all()} == before
    ws.heartbeat()                        # third one goes through
    s.expire_all()
    assert {d.name: d.last_activity for d in s.query(Docker).all()} != before


def test_killed_task_process_is_failed_by_liveness(cluster):
    from mlcomp_amd.db.enums import TaskStatus
    cfg = {'info': {'name': 'killme', 'project': 'p_fault'},
           'executors': {'sleepy': {'type': 'bash', 'command': 'sleep 30', 'env': {'MLC_FAULTS': 'kill_task=1'}}}}
    ids = _ids(_submit(cluster['tmp'], cfg))
    import threading
    stop = threading.Event()

    def liveness():
        while not stop.is_set():
            cluster['ws'].stop_processes_not_exist()
            stop.wait(0.5)
    th = threading.Thread(target=liveness, daemon=True)
    th.start()
    try:
        res = _wait(cluster['sup'], ids, timeout=60)
    finally:
        stop.set()
        th.join()
    assert all(v == TaskStatus.Failed for v in res.values()), res


def test_crash_string_fails_task_with_message(cluster):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import Log
    cfg = {'info': {'name': 'crash', 'project': 'p_fault2'},
           'executors': {'x': {'type': 'bash', 'command': 'echo hi',
                               'env': {'MLC_FAULTS': 'crash_task=hipErrorIllegalAddress injected'}}}}
    ids = _ids(_submit(cluster['tmp'], cfg))
    res = _wait(cluster['sup'], ids, timeout=60)
    assert all(v == TaskStatus.Failed for v in res.values()), res
    s = Session.create_session(key='logs')
    assert any('hipErrorIllegalAddress injected' in (r.message or '') for r in s.query(Log).all())
