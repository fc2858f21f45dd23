"""ORM models: the reference's 25 tables with identical table and column names/types
(`mlcomp/db/models/*.py`, `mlcomp/migration/versions/001_init.py`), written for
SQLAlchemy 2.0, so a database created by either framework can be read by the other.

Every model has ``to_dict()`` (the JSON shape the REST API returns).
"""
from __future__ import annotations

import datetime
import sys

import sqlalchemy as sa
from sqlalchemy import ForeignKey
from sqlalchemy.orm import declarative_base, deferred, relationship

from .enums import TaskStatus


def now():
    return datetime.datetime.now()


class _Base:
    def to_dict(self, exclude=()):
        """Loaded column values (deferred/unloaded columns and blobs are skipped)."""
        try:
            unloaded = sa.inspect(self).unloaded
        except Exception:
            unloaded = set()
        out = {}
        for c in self.__table__.columns:
            if c.key in exclude or c.key in unloaded:
                continue
            v = getattr(self, c.key)
            if isinstance(v, (datetime.datetime, datetime.date)):
                v = v.isoformat()
            elif isinstance(v, bytes):
                continue
            out[c.key] = v
        return out

    def __repr__(self):
        pk = [getattr(self, c.key, None) for c in self.__table__.primary_key.columns]
        return f'<{type(self).__name__} {pk}>'


Base = declarative_base(cls=_Base)


class Project(Base):
    __tablename__ = 'project'
    id = sa.Column(sa.Integer, primary_key=True)
    name = sa.Column(sa.String, nullable=False)
    class_names = sa.Column(sa.String, nullable=False, default='{}')
    sync_folders = sa.Column(sa.String, nullable=False, default='')
    ignore_folders = sa.Column(sa.String, nullable=False, default='')


class Computer(Base):
    __tablename__ = 'computer'
    name = sa.Column(sa.String, primary_key=True)
    gpu = sa.Column(sa.Integer, default=0)
    cpu = sa.Column(sa.Integer, default=1)
    memory = sa.Column(sa.Float, default=0.1)
    usage = sa.Column(sa.String)
    ip = sa.Column(sa.String)
    port = sa.Column(sa.Integer)
    user = sa.Column(sa.String)
    last_synced = sa.Column(sa.DateTime)
    disk = sa.Column(sa.Integer)
    syncing_computer = sa.Column(sa.String, ForeignKey('computer.name'))
    root_folder = sa.Column(sa.String)
    can_process_tasks = sa.Column(sa.Boolean)
    sync_with_this_computer = sa.Column(sa.Boolean)
    meta = sa.Column(sa.String)


class ComputerUsage(Base):
    __tablename__ = 'computer_usage'
    id = sa.Column(sa.Integer, primary_key=True)
    computer = sa.Column(sa.String, ForeignKey('computer.name', ondelete='CASCADE'))
    usage = sa.Column(sa.String)
    time = sa.Column(sa.DateTime, default=now)


class Report(Base):
    __tablename__ = 'report'
    id = sa.Column(sa.Integer, primary_key=True)
    config = sa.Column(sa.String)
    time = sa.Column(sa.DateTime, default=now)
    name = sa.Column(sa.String)
    project = sa.Column(sa.Integer, ForeignKey('project.id', ondelete='CASCADE'))
    layout = sa.Column(sa.String)


class Dag(Base):
    __tablename__ = 'dag'
    id = sa.Column(sa.Integer, primary_key=True)
    project = sa.Column(sa.Integer, ForeignKey('project.id', ondelete='CASCADE'))
    created = sa.Column(sa.DateTime, default=now)
    config = sa.Column(sa.String)
    name = sa.Column(sa.String)
    tasks = relationship('Task', lazy='noload', foreign_keys='Task.dag', viewonly=True)
    project_rel = relationship('Project', lazy='noload', viewonly=True)
    docker_img = sa.Column(sa.String)
    img_size = sa.Column(sa.BigInteger, nullable=False, default=0)
    file_size = sa.Column(sa.BigInteger, nullable=False, default=0)
    type = sa.Column(sa.Integer, default=0)
    report = sa.Column(sa.Integer, ForeignKey('report.id', ondelete='CASCADE'))
    report_rel = relationship('Report', lazy='noload', viewonly=True)


class DagTag(Base):
    __tablename__ = 'dag_tag'
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'), primary_key=True)
    tag = sa.Column(sa.String, primary_key=True)


class File(Base):
    __tablename__ = 'file'
    id = sa.Column(sa.Integer, primary_key=True)
    md5 = sa.Column(sa.String)
    created = sa.Column(sa.DateTime, default=now)
    content = sa.Column(sa.LargeBinary)
    project = sa.Column(sa.Integer, ForeignKey('project.id', ondelete='CASCADE'))
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    size = sa.Column(sa.BigInteger, nullable=False, default=0)

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.size = sys.getsizeof(self.content)


class DagStorage(Base):
    __tablename__ = 'dag_storage'
    id = sa.Column(sa.Integer, primary_key=True)
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    file = sa.Column(sa.Integer, ForeignKey('file.id', ondelete='CASCADE'))
    path = sa.Column(sa.String)
    is_dir = sa.Column(sa.Boolean)


class DagLibrary(Base):
    __tablename__ = 'dag_library'
    id = sa.Column(sa.Integer, primary_key=True)
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    library = sa.Column(sa.String)
    version = sa.Column(sa.String)


class Task(Base):
    __tablename__ = 'task'
    id = sa.Column(sa.Integer, primary_key=True)
    name = sa.Column(sa.String)
    started = sa.Column(sa.DateTime)
    finished = sa.Column(sa.DateTime)
    last_activity = sa.Column(sa.DateTime)
    computer = sa.Column(sa.String)
    gpu = sa.Column(sa.Integer, default=0)
    gpu_max = sa.Column(sa.Integer, default=0)
    cpu = sa.Column(sa.Integer, default=1)
    executor = sa.Column(sa.String)
    status = sa.Column(sa.Integer, default=TaskStatus.NotRan.value)
    computer_assigned = sa.Column(sa.String, ForeignKey('computer.name', ondelete='CASCADE'))
    computer_assigned_rel = relationship('Computer', lazy='noload', viewonly=True)
    memory = sa.Column(sa.Float, default=0.1)
    steps = sa.Column(sa.Integer, default=1)
    current_step = sa.Column(sa.String)
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    celery_id = sa.Column(sa.String)
    dag_rel = relationship('Dag', lazy='noload', foreign_keys=[dag], viewonly=True)
    debug = sa.Column(sa.Boolean, default=False)
    pid = sa.Column(sa.Integer)
    worker_index = sa.Column(sa.Integer)
    docker_assigned = sa.Column(sa.String)
    type = sa.Column(sa.Integer)
    score = sa.Column(sa.Float)
    report = sa.Column(sa.Integer, ForeignKey('report.id', ondelete='CASCADE'))
    report_rel = relationship('Report', lazy='noload', viewonly=True)
    gpu_assigned = sa.Column(sa.String)
    parent = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))
    parent_rel = relationship('Task', lazy='noload', remote_side=[id], viewonly=True)
    loss = sa.Column(sa.Float)
    continued = sa.Column(sa.Boolean, default=False)
    batch_index = sa.Column(sa.Integer)
    batch_total = sa.Column(sa.Integer)
    loader_name = sa.Column(sa.String)
    epoch_duration = sa.Column(sa.Integer)
    epoch_time_remaining = sa.Column(sa.Integer)
    result = deferred(sa.Column(sa.String))
    additional_info = deferred(sa.Column(sa.String))


class TaskDependence(Base):
    __tablename__ = 'task_dependency'
    task_id = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'), primary_key=True)
    depend_id = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'), primary_key=True)


class TaskSynced(Base):
    __tablename__ = 'task_synced'
    computer = sa.Column(sa.String, ForeignKey('computer.name', ondelete='CASCADE'), primary_key=True)
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'), primary_key=True)


class Step(Base):
    __tablename__ = 'step'
    id = sa.Column(sa.Integer, primary_key=True)
    level = sa.Column(sa.Integer)
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))
    started = sa.Column(sa.DateTime)
    finished = sa.Column(sa.DateTime)
    name = sa.Column(sa.String)
    task_rel = relationship('Task', lazy='noload', viewonly=True)
    index = sa.Column(sa.Integer)


class Log(Base):
    __tablename__ = 'log'
    id = sa.Column(sa.Integer, primary_key=True)
    step = sa.Column(sa.Integer, ForeignKey('step.id', ondelete='CASCADE'))
    message = sa.Column(sa.String)
    time = sa.Column(sa.DateTime)
    level = sa.Column(sa.Integer)
    component = sa.Column(sa.Integer)
    module = sa.Column(sa.String)
    line = sa.Column(sa.Integer)
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))
    computer = sa.Column(sa.String, ForeignKey('computer.name', ondelete='CASCADE'))


class ReportSeries(Base):
    __tablename__ = 'report_series'
    id = sa.Column(sa.Integer, primary_key=True)
    name = sa.Column(sa.String)
    value = sa.Column(sa.Float)
    epoch = sa.Column(sa.Integer)
    time = sa.Column(sa.DateTime)
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))
    part = sa.Column(sa.String)
    stage = sa.Column(sa.String)
    task_rel = relationship('Task', lazy='noload', viewonly=True)


class ReportImg(Base):
    __tablename__ = 'report_img'
    id = sa.Column(sa.Integer, primary_key=True)
    group = sa.Column(sa.String)
    epoch = sa.Column(sa.Integer)
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))
    img = sa.Column(sa.LargeBinary)
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    part = sa.Column(sa.String)
    project = sa.Column(sa.Integer, ForeignKey('project.id', ondelete='CASCADE'))
    y_pred = sa.Column(sa.Integer)
    y = sa.Column(sa.Integer)
    score = sa.Column(sa.Float)
    size = sa.Column(sa.BigInteger)
    attr1 = sa.Column(sa.Float)
    attr2 = sa.Column(sa.Float)
    attr3 = sa.Column(sa.Float)
    attr4 = sa.Column(sa.Float)
    attr5 = sa.Column(sa.Float)
    attr6 = sa.Column(sa.Float)
    attr7 = sa.Column(sa.Float)
    attr8 = sa.Column(sa.Float)
    attr9 = sa.Column(sa.Float)
    attr1_str = sa.Column(sa.String)
    attr2_str = sa.Column(sa.String)
    attr3_str = sa.Column(sa.String)
    attr4_str = sa.Column(sa.String)
    attr5_str = sa.Column(sa.String)

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.size = sys.getsizeof(self.img)


class ReportTasks(Base):
    __tablename__ = 'report_task'
    id = sa.Column(sa.Integer, primary_key=True)
    report = sa.Column(sa.Integer, ForeignKey('report.id', ondelete='CASCADE'))
    task = sa.Column(sa.Integer, ForeignKey('task.id', ondelete='CASCADE'))


class ReportLayout(Base):
    __tablename__ = 'report_layout'
    name = sa.Column(sa.String, primary_key=True)
    content = sa.Column(sa.String)
    last_modified = sa.Column(sa.TIMESTAMP)


class Docker(Base):
    __tablename__ = 'docker'
    name = sa.Column(sa.String, primary_key=True)
    computer = sa.Column(sa.String, ForeignKey('computer.name', ondelete='CASCADE'), primary_key=True)
    last_activity = sa.Column(sa.DateTime, nullable=False)
    ports = sa.Column(sa.String, nullable=False)


class Model(Base):
    __tablename__ = 'model'
    id = sa.Column(sa.Integer, primary_key=True)
    name = sa.Column(sa.String)
    score_local = sa.Column(sa.Float)
    score_public = sa.Column(sa.Float)
    project = sa.Column(sa.Integer, ForeignKey('project.id', ondelete='CASCADE'))
    dag = sa.Column(sa.Integer, ForeignKey('dag.id', ondelete='CASCADE'))
    created = sa.Column(sa.DateTime)
    equations = sa.Column(sa.String)
    fold = sa.Column(sa.Integer)
    dag_rel = relationship('Dag', lazy='noload', viewonly=True)
    project_rel = relationship('Project', lazy='noload', viewonly=True)


class Auxiliary(Base):
    __tablename__ = 'auxiliary'
    name = sa.Column(sa.String, primary_key=True)
    data = sa.Column(sa.String)


class Memory(Base):
    __tablename__ = 'memory'
    id = sa.Column(sa.Integer, primary_key=True)
    model = sa.Column(sa.String, nullable=False)
    variant = sa.Column(sa.String)
    num_classes = sa.Column(sa.Integer)
    img_size = sa.Column(sa.Integer)
    batch_size = sa.Column(sa.Integer, nullable=False)
    memory = sa.Column(sa.Float, nullable=False)


class Space(Base):
    __tablename__ = 'space'
    name = sa.Column(sa.String, nullable=False, primary_key=True)
    created = sa.Column(sa.DateTime, nullable=False, default=now)
    changed = sa.Column(sa.DateTime, nullable=False, default=now)
    content = sa.Column(sa.String, nullable=False)


class SpaceRelation(Base):
    __tablename__ = 'space_relation'
    parent = sa.Column(sa.String, ForeignKey('space.name', ondelete='CASCADE'), primary_key=True)
    child = sa.Column(sa.String, ForeignKey('space.name', ondelete='CASCADE'), primary_key=True)


class SpaceTag(Base):
    __tablename__ = 'space_tag'
    space = sa.Column(sa.String, ForeignKey('space.name', ondelete='CASCADE'), primary_key=True)
    tag = sa.Column(sa.String, primary_key=True)


ALL_MODELS = [Project, Computer, ComputerUsage, Report, Dag, DagTag, File, DagStorage, DagLibrary,
              Task, TaskDependence, TaskSynced, Step, Log, ReportSeries, ReportImg, ReportTasks,
              ReportLayout, Docker, Model, Auxiliary, Memory, Space, SpaceRelation, SpaceTag]

__all__ = [m.__name__ for m in ALL_MODELS] + ['Base', 'now']
