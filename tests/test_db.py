"""DB layer: migrations (versions 1..10, seeded layouts), providers, signals, layouts.
Mirrors and extends the reference's only tests (`mlcomp/db/tests/test_project.py`)."""
import datetime

import pytest
import yaml


@pytest.fixture
def session(mlc_root):
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    assert migrate() == 10
    s = Session.create_session(key='test')
    yield s
    Session.cleanup()


def test_migrate_idempotent_and_versioned(session):
    from mlcomp_amd.db.migrate import migrate, current_version, LATEST
    assert current_version(session.get_bind()) == LATEST
    assert migrate() == LATEST
    import sqlalchemy as sa
    names = set(sa.inspect(session.get_bind()).get_table_names())
    for t in ['project', 'dag', 'task', 'task_dependency', 'report_layout', 'space', 'space_tag',
              'dag_tag', 'memory', 'computer_usage', 'report_series', 'report_img', 'migrate_version']:
        assert t in names, t


def test_project_provider(session):
    from mlcomp_amd.db.providers import ProjectProvider
    p = ProjectProvider(session)
    p.add_project('test', class_names={'a': [1]})
    assert p.by_name('test').id == 1
    res = p.get({'name': 'te'})
    assert res['total'] == 1 and res['data'][0]['name'] == 'test'


def test_layouts_seeded_and_extended(session):
    from mlcomp_amd.db.providers import ReportLayoutProvider
    from mlcomp_amd.db.report_info import ReportLayoutInfo
    layouts = ReportLayoutProvider(session).all()
    assert {'base', 'base_time', 'classify', 'img-classify', 'segment'} <= set(layouts)
    cl = ReportLayoutInfo(layouts['classify'])
    assert cl.metric.name == 'accuracy01' and not cl.metric.minimize
    # extend: base_time panel comes first
    assert layouts['classify']['layout'][0]['title'] == 'base'
    ic = ReportLayoutInfo(layouts['img-classify'])
    assert [i.name for i in ic.img_classify] == ['img_classify']


def test_layout_validation():
    from mlcomp_amd.db.report_info import LayoutError, ReportLayoutInfo
    with pytest.raises(LayoutError):
        ReportLayoutInfo({'layout': [{'type': 'series'}]})  # missing source
    with pytest.raises(LayoutError):
        ReportLayoutInfo({'layout': [{'type': 'table', 'source': ['a'], 'bogus': 1}]})


def test_signals_bump_last_activity(session):
    from mlcomp_amd.db.models import Dag, Log, Project, Step, Task, ReportImg
    from mlcomp_amd.db.providers import TaskProvider
    session.add(Project(name='p', class_names='', sync_folders='', ignore_folders=''))
    session.add(Dag(name='d', project=1, config=''))
    parent = session.add(Task(name='parent', dag=1, type=1))
    child = session.add(Task(name='child', dag=1, type=2, parent=parent.id))
    assert parent.last_activity is None
    child.status = 2
    session.commit()
    session.expire_all()
    assert TaskProvider(session).by_id(parent.id).last_activity is not None
    st = session.add(Step(task=child.id, level=0, name='main', started=datetime.datetime.now(), index=0))
    session.add(Log(step=st.id, message='m', level=20, component=2, time=datetime.datetime.now()))
    session.add(ReportImg(dag=1, task=child.id, img=b'1234', group='g', epoch=0))
    session.expire_all()
    assert session.query(Dag).one().img_size > 0


def test_parent_stats_and_dependencies(session):
    from mlcomp_amd.db.enums import TaskStatus
    from mlcomp_amd.db.models import Dag, Project, Task
    from mlcomp_amd.db.providers import TaskProvider
    session.add(Project(name='p', class_names='', sync_folders='', ignore_folders=''))
    session.add(Dag(name='d', project=1, config=''))
    tp = TaskProvider(session)
    p = session.add(Task(name='p', dag=1, type=1, status=TaskStatus.InProgress.value))
    for st in (TaskStatus.Success, TaskStatus.InProgress, TaskStatus.Failed):
        session.add(Task(name='c', dag=1, type=2, parent=p.id, status=st.value))
    stats = tp.parent_tasks_stats()
    assert len(stats) == 1
    t, _, _, counts = stats[0]
    assert counts[TaskStatus.Success] == 1 and counts[TaskStatus.Failed] == 1
    a = session.add(Task(name='a', dag=1, type=0, status=TaskStatus.Success.value))
    b = session.add(Task(name='b', dag=1, type=0))
    tp.add_dependency(b.id, a.id)
    assert tp.dependency_status([b])[b.id] == {TaskStatus.Success.value}
