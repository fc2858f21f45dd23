"""File sync between computers (`mlcomp_amd/worker/sync.py`, reference
`mlcomp/worker/sync.py:20-239`): the rsync/ssh command strings for push, pull and relayed
copies, the per-project folder rewrite, and FileSync pulling the sync folders of Success
tasks computed on another computer exactly once (task_synced bookkeeping).  No network:
the shell commands are recorded instead of run."""
import os
import subprocess

import pytest

from mlcomp_amd.db.enums import TaskStatus


def _comp(name, ip, port=22, user='mlcomp', root='/data/mlcomp', sync=True):
    from mlcomp_amd.db.models import Computer
    return Computer(name=name, gpu=8, cpu=64, memory=1024, ip=ip, port=port, user=user, root_folder=root,
                    can_process_tasks=True, sync_with_this_computer=sync)


def test_rsync_command_push_pull_and_relay():
    from mlcomp_amd.worker.sync import rsync_command
    a, b = _comp('a', '10.0.0.1', 2201, root='/ra'), _comp('b', '10.0.0.2', 2202, user='u', root='/rb')
    excl = ['data/p/tmp', 'data/p', 'models/q/x']
    push = rsync_command(a, b, 'data/p', excl, current='a')
    assert push.startswith('rsync -vhru -e "ssh -p 2202 -o StrictHostKeyChecking=no" /ra/data/p/ u@10.0.0.2:/rb/data/p/')
    assert '--exclude tmp' in push and 'models' not in push.split('--size-only')[1]
    assert '--perms --chmod=777 --size-only' in push
    pull = rsync_command(a, b, 'data/p', excl, current='b')
    assert pull.startswith('rsync -vhru -e "ssh -p 2201 -o StrictHostKeyChecking=no" mlcomp@10.0.0.1:/ra/data/p/ /rb/data/p/')
    relay = rsync_command(a, b, 'data/p', [], current='c')
    assert relay.startswith('ssh -p 2201 mlcomp@10.0.0.1 "rsync -vhru -e \\"ssh -p 2202')
    assert relay.rstrip().endswith('--size-only"')


def test_correct_folders_scopes_data_and_models_to_the_project():
    from mlcomp_amd.worker.sync import correct_folders
    assert correct_folders(['data', 'models', 'data/p/x', 'data/other', 'logs'], 'p') == \
        ['data/p', 'models/p', 'data/p/x', 'data/p/other', 'logs']


@pytest.fixture
def db(mlc_root, monkeypatch):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    monkeypatch.setenv('MLCOMP_COMPUTER', 'me')
    migrate()
    s = Session.create_session(key='sync-test')
    yield s
    Session.cleanup()


def _seed(s, other_sync=True):
    from mlcomp_amd.db.models import Dag, Project, Task
    s.add(_comp('me', '10.0.0.1', root='/rme'))
    s.add(_comp('node2', '10.0.0.2', port=2222, root='/rn2', sync=other_sync))
    p = Project(name='p', sync_folders='data models', ignore_folders='data/p/cache')
    s.add(p)
    s.commit()
    d = Dag(project=p.id, name='d', config='')
    s.add(d)
    s.commit()
    tasks = [Task(name='train', dag=d.id, status=TaskStatus.Success.value, computer_assigned='node2'),
             Task(name='valid', dag=d.id, status=TaskStatus.Success.value, computer_assigned='me'),
             Task(name='infer', dag=d.id, status=TaskStatus.InProgress.value, computer_assigned='node2')]
    s.add_all(tasks)
    s.commit()
    return tasks


def test_file_sync_pulls_other_computers_success_tasks_once(db, monkeypatch):
    from mlcomp_amd.db.models import Computer, TaskSynced
    from mlcomp_amd.worker import sync as S
    ran = []

    def fake_run(cmd, shell, capture_output, text):
        ran.append(cmd)
        return subprocess.CompletedProcess(cmd, 0, '', '')
    monkeypatch.setattr(S.subprocess, 'run', fake_run)
    tasks = _seed(db)
    S.FileSync(db).sync()
    # one pull per sync folder, from node2 (the only other computer with a Success task)
    assert len(ran) == 2, ran
    assert all(c.startswith('rsync -vhru -e "ssh -p 2222') and 'mlcomp@10.0.0.2:' in c for c in ran)
    assert '/rn2/data/p/ /rme/data/p/' in ran[0] and '--exclude cache' in ran[0]
    assert '/rn2/models/p/ /rme/models/p/' in ran[1] and '--exclude' not in ran[1]
    db.expire_all()
    synced = {(r.computer, r.task) for r in db.query(TaskSynced).all()}
    assert synced == {('me', tasks[0].id)}      # not the local task, not the running one
    assert db.get(Computer, 'me').last_synced is not None
    ran.clear()
    S.FileSync(db).sync()
    assert ran == []                            # already synced


def test_file_sync_skips_computers_not_shared_and_raises_on_rsync_error(db, monkeypatch):
    from mlcomp_amd.worker import sync as S
    ran = []
    monkeypatch.setattr(S.subprocess, 'run',
                        lambda cmd, **kw: ran.append(cmd) or subprocess.CompletedProcess(cmd, 0, '', ''))
    _seed(db, other_sync=False)
    S.FileSync(db).sync()
    assert ran == []
    from mlcomp_amd.db.models import Computer
    db.get(Computer, 'node2').sync_with_this_computer = True
    db.commit()
    from mlcomp_amd.db.models import TaskSynced
    db.query(TaskSynced).delete()
    db.commit()
    monkeypatch.setattr(S.subprocess, 'run',
                        lambda cmd, **kw: subprocess.CompletedProcess(cmd, 23, 'partial', ' transfer'))
    with pytest.raises(RuntimeError, match='partial transfer'):
        S.FileSync(db).sync()


def test_copy_remote_local_and_scp(db, tmp_path, monkeypatch):
    from mlcomp_amd.worker import sync as S
    src = tmp_path / 'ckpt.pth'
    src.write_bytes(b'w')
    dst = tmp_path / 'sub' / 'copy.pth'
    assert S.copy_remote(db, 'me', str(src), str(dst)) and dst.read_bytes() == b'w'
    _seed(db)
    cmds = []

    def fake_check_output(cmd, shell):
        cmds.append(cmd)
        open(tmp_path / 'remote.pth', 'wb').close()
        return b''
    monkeypatch.setattr(S.subprocess, 'check_output', fake_check_output)
    assert S.copy_remote(db, 'node2', '/rn2/models/p/best.pth', str(tmp_path / 'remote.pth'))
    assert cmds == [f'scp -P 2222 mlcomp@10.0.0.2:/rn2/models/p/best.pth {tmp_path / "remote.pth"}']
    assert os.path.exists(tmp_path / 'remote.pth')
