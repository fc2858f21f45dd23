"""Data-access providers (the query layer used by the API, scheduler, workers and the
DAG builders).  Method names follow the reference's providers
(`mlcomp/db/providers/*.py`) so the call sites read the same; queries are written for
SQLAlchemy 2.0 (the reference's ``case(whens=...)`` form no longer exists).
"""
from __future__ import annotations

import datetime
import json
from collections import defaultdict
from typing import Dict, Iterable, List, Optional, Union

import yaml
from sqlalchemy import case, func
from sqlalchemy.orm import aliased

from .core import PaginatorOptions, Session
from .enums import DagType, LogStatus, TaskStatus, TaskType, to_snake
from .models import (Auxiliary, Computer, ComputerUsage, Dag, DagLibrary, DagStorage, DagTag,
                     Docker, File, Log, Memory, Model, Project, Report, ReportImg, ReportLayout,
                     ReportSeries, ReportTasks, Space, SpaceRelation, SpaceTag, Step, Task,
                     TaskDependence, TaskSynced, now)


def duration_format(seconds: float) -> str:
    seconds = int(seconds or 0)
    d, seconds = divmod(seconds, 86400)
    h, seconds = divmod(seconds, 3600)
    m, s = divmod(seconds, 60)
    if d:
        return f'{d} days {h} hours'
    if h:
        return f'{h} hours {m} min'
    if m:
        return f'{m} min {s} sec'
    return f'{s} sec'


def parse_time(v):
    if isinstance(v, datetime.datetime) or v is None:
        return v
    for fmt in ('%Y-%m-%dT%H:%M:%S.%f', '%Y-%m-%dT%H:%M:%S', '%Y-%m-%d %H:%M:%S', '%Y-%m-%d'):
        try:
            return datetime.datetime.strptime(str(v).replace('Z', ''), fmt)
        except ValueError:
            continue
    raise ValueError(f'bad time {v!r}')


class BaseDataProvider:
    model = None

    def __init__(self, session: Optional[Session] = None):
        self.session = session or Session.create_session()

    def query(self, *args, **kwargs):
        return self.session.query(*args, **kwargs)

    def add(self, obj, commit=True):
        return self.session.add(obj, commit=commit)

    def add_all(self, objs, commit=True):
        self.session.add_all(objs, commit=commit)

    def commit(self):
        self.session.commit()

    def rollback(self):
        self.session.rollback()

    def update(self):
        self.session.commit()

    def by_id(self, id, *_):
        return self.query(self.model).filter(self.model.id == id).one_or_none()

    def all(self):
        return self.query(self.model).all()

    def remove(self, id):
        self.query(self.model).filter(self.model.id == id).delete(synchronize_session=False)
        self.commit()

    def create_or_update(self, obj, *keys):
        q = self.query(type(obj))
        for k in keys:
            q = q.filter(getattr(type(obj), k) == getattr(obj, k))
        cur = q.one_or_none()
        if cur is None:
            return self.add(obj)
        for c in obj.__table__.columns:
            v = getattr(obj, c.key)
            if v is not None:
                setattr(cur, c.key, v)
        self.commit()
        return cur

    def paginator(self, query, options: Optional[PaginatorOptions]):
        if options is None:
            return query
        if options.sort_column:
            col = getattr(self.model, options.sort_column, None)
            if col is not None:
                query = query.order_by(col.desc() if options.sort_descending else col.asc())
        if options.page_size:
            query = query.offset(options.page_size * options.page_number).limit(options.page_size)
        return query

    @staticmethod
    def to_dict(obj, exclude=()):
        return obj.to_dict(exclude=exclude)


# ---------------------------------------------------------------------------- projects
class ProjectProvider(BaseDataProvider):
    model = Project

    def by_name(self, name: str) -> Optional[Project]:
        return self.query(Project).filter(Project.name == name).one_or_none()

    def add_project(self, name: str, class_names=None, sync_folders='', ignore_folders=''):
        p = Project(name=name, class_names=yaml.safe_dump(class_names or {}),
                    sync_folders=sync_folders or '', ignore_folders=ignore_folders or '')
        return self.add(p)

    def get(self, filter: Optional[dict] = None, options: Optional[PaginatorOptions] = None):
        filter = filter or {}
        q = self.query(Project)
        if filter.get('name'):
            q = q.filter(Project.name.like(f"%{filter['name']}%"))
        total = q.count()
        res = []
        for p in self.paginator(q, options).all():
            item = p.to_dict()
            dags = self.query(Dag).filter(Dag.project == p.id)
            item['dag_count'] = dags.count()
            last = dags.order_by(Dag.created.desc()).first()
            item['last_activity'] = last.created.isoformat() if last and last.created else None
            item['file_size'] = sum(d.file_size or 0 for d in dags)
            item['img_size'] = sum(d.img_size or 0 for d in dags)
            res.append(item)
        return {'total': total, 'data': res}

    def edit(self, id, **fields):
        p = self.by_id(id)
        for k, v in fields.items():
            if hasattr(p, k) and v is not None:
                setattr(p, k, v)
        self.commit()
        return p


# ---------------------------------------------------------------------------- tasks
class TaskProvider(BaseDataProvider):
    model = Task

    def _filter(self, q, f: dict):
        if f.get('dag'):
            q = q.filter(Task.dag == f['dag'])
        if f.get('name'):
            q = q.filter(Task.name.like(f"%{f['name']}%"))
        if f.get('status'):
            st = [TaskStatus.from_name(k) for k, v in f['status'].items() if v]
            if st:
                q = q.filter(Task.status.in_(st))
        if f.get('id'):
            q = q.filter(Task.id == f['id'])
        if f.get('id_min'):
            q = q.filter(Task.id >= f['id_min'])
        if f.get('id_max'):
            q = q.filter(Task.id <= f['id_max'])
        if f.get('project'):
            q = q.filter(Dag.project == f['project'])
        if f.get('parent'):
            q = q.filter(Task.parent == f['parent'])
        if f.get('last_activity_min'):
            q = q.filter(Task.last_activity >= parse_time(f['last_activity_min']))
        if f.get('last_activity_max'):
            q = q.filter(Task.last_activity <= parse_time(f['last_activity_max']))
        types = [TaskType.from_name(t) for t in f.get('type', ['User', 'Train'])]
        return q.filter(Task.type.in_(types))

    def get(self, filter: dict, options: Optional[PaginatorOptions] = None):
        q = self.query(Task, Dag, Project.name).join(Dag, Dag.id == Task.dag).join(
            Project, Project.id == Dag.project)
        q = self._filter(q, filter)
        total = q.count()
        res = []
        for t, d, pname in self.paginator(q, options).all():
            item = t.to_dict(exclude=('additional_info', 'result'))
            item['status'] = to_snake(TaskStatus(t.status).name)
            item['type'] = to_snake(TaskType(t.type).name) if t.type is not None else None
            item['dag_rel'] = d.to_dict()
            item['dag_rel']['project'] = {'id': d.project, 'name': pname}
            if t.started is None:
                delta = 0
            elif t.status == TaskStatus.InProgress.value:
                delta = (now() - t.started).total_seconds()
            else:
                delta = ((t.finished or t.last_activity or t.started) - t.started).total_seconds()
            item['duration'] = duration_format(delta)
            res.append(item)
        return {'total': total, 'data': res}

    def by_ids(self, ids) -> List[Task]:
        return self.query(Task).filter(Task.id.in_(list(ids))).all()

    def change_status(self, task: Task, status: TaskStatus):
        if status == TaskStatus.InProgress:
            task.started = now()
        elif status in (TaskStatus.Failed, TaskStatus.Stopped, TaskStatus.Success):
            task.finished = now()
        task.status = status.value
        task.last_activity = now()
        self.commit()

    def change_status_all(self, tasks: List[int], status: TaskStatus):
        upd = {'status': status.value, 'last_activity': now()}
        if status == TaskStatus.InProgress:
            upd['started'] = now()
        elif status in (TaskStatus.Failed, TaskStatus.Stopped, TaskStatus.Success):
            upd['finished'] = now()
        if tasks:
            self.query(Task).filter(Task.id.in_(tasks)).update(upd, synchronize_session=False)
            self.commit()

    def by_status(self, *statuses: TaskStatus, task_docker_assigned=None, worker_index=None,
                  computer_assigned=None, project=None) -> List[Task]:
        q = self.query(Task).filter(Task.status.in_([s.value for s in statuses]))
        if task_docker_assigned:
            q = q.filter(Task.docker_assigned == task_docker_assigned)
        if worker_index is not None:
            q = q.filter(Task.worker_index == worker_index)
        if computer_assigned is not None:
            q = q.filter(Task.computer_assigned == computer_assigned)
        if project:
            q = q.join(Dag, Dag.id == Task.dag).filter(Dag.project == project)
        return q.order_by(Task.id).all()

    def add_dependency(self, task_id: int, depend_id: int):
        self.add(TaskDependence(task_id=task_id, depend_id=depend_id))

    def dependency_status(self, tasks: List[Task]) -> Dict[int, set]:
        res = {t.id: set() for t in tasks}
        if not tasks:
            return res
        rows = self.query(TaskDependence.task_id, Task.status).join(
            Task, Task.id == TaskDependence.depend_id).filter(
            TaskDependence.task_id.in_([t.id for t in tasks])).all()
        for tid, st in rows:
            res[tid].add(st)
        return res

    def update_last_activity(self, task_id: int):
        self.query(Task).filter(Task.id == task_id).update({'last_activity': now()},
                                                          synchronize_session=False)
        self.commit()

    def by_dag(self, dag_id: int) -> List[Task]:
        return self.query(Task).filter(Task.dag == dag_id).order_by(Task.id).all()

    def children(self, ids: Union[int, List[int]]) -> List[Task]:
        if isinstance(ids, int):
            ids = [ids]
        return self.query(Task).filter(Task.parent.in_(ids)).filter(
            (Task.continued.is_(None)) | (Task.continued.is_(False))).order_by(Task.id).all()

    def parent_tasks_stats(self):
        """[(parent task, min child started, max child finished, {status: count})] for
        parents still Queued/InProgress, over their non-continued children."""
        parent, child = aliased(Task), aliased(Task)
        sums = [func.sum(case((child.status == e.value, 1), else_=0)) for e in TaskStatus]
        q = self.query(parent, func.min(child.started), func.max(child.finished), *sums).join(
            child, parent.id == child.parent).filter(
            parent.status.in_([TaskStatus.Queued.value, TaskStatus.InProgress.value])).filter(
            (child.continued.is_(None)) | (child.continued.is_(False))).group_by(parent.id)
        out = []
        for row in q.all():
            t, started, finished, *counts = row
            out.append([t, started, finished, {e: int(c or 0) for e, c in zip(TaskStatus, counts)}])
        return out

    def project(self, task_id: int) -> Project:
        return self.query(Project).join(Dag, Dag.project == Project.id).join(
            Task, Task.dag == Dag.id).filter(Task.id == task_id).one()

    def find_dependents(self, task_id: int) -> List[Task]:
        return self.query(Task).join(TaskDependence, Task.id == TaskDependence.depend_id).filter(
            TaskDependence.task_id == task_id).all()

    def get_dependencies(self, dag_id: int) -> List[TaskDependence]:
        return self.query(TaskDependence).join(Task, Task.id == TaskDependence.task_id).filter(
            Task.dag == dag_id).all()

    def last_succeed_time(self):
        r = self.query(Task.finished).filter(Task.status == TaskStatus.Success.value).order_by(
            Task.finished.desc()).first()
        return r[0] if r else None

    def stop(self, id: int):
        t = self.by_id(id)
        if t is not None:
            self.change_status(t, TaskStatus.Stopped)


# ---------------------------------------------------------------------------- dags
class DagProvider(BaseDataProvider):
    model = Dag

    def get(self, filter: dict, options: Optional[PaginatorOptions] = None):
        q = self.query(Dag, Project.name).join(Project, Project.id == Dag.project)
        if filter.get('project'):
            q = q.filter(Dag.project == filter['project'])
        if filter.get('name'):
            q = q.filter(Dag.name.like(f"%{filter['name']}%"))
        if filter.get('id'):
            q = q.filter(Dag.id == filter['id'])
        if filter.get('type') is not None:
            q = q.filter(Dag.type == filter['type'])
        if filter.get('tags'):
            for tag in filter['tags']:
                q = q.filter(Dag.id.in_(self.query(DagTag.dag).filter(DagTag.tag == tag)))
        total = q.count()
        res = []
        for d, pname in self.paginator(q, options).all():
            item = d.to_dict()
            item['project'] = {'id': d.project, 'name': pname}
            tasks = self.query(Task.status, Task.started, Task.finished, Task.last_activity).filter(
                Task.dag == d.id).filter(Task.type != TaskType.Service.value).all()
            cnt = defaultdict(int)
            started = [t[1] for t in tasks if t[1]]
            ended = [t[2] or t[3] for t in tasks if (t[2] or t[3])]
            for st, *_ in tasks:
                cnt[st] += 1
            item['task_count'] = len(tasks)
            item['task_statuses'] = [{'name': to_snake(e.name), 'count': cnt[e.value]} for e in TaskStatus]
            item['started'] = min(started).isoformat() if started else None
            item['last_activity'] = max(ended).isoformat() if ended else None
            item['tags'] = [t[0] for t in self.query(DagTag.tag).filter(DagTag.dag == d.id)]
            item['type'] = to_snake(DagType(d.type or 0).name)
            res.append(item)
        return {'total': total, 'data': res}

    def graph(self, id: int):
        tasks = self.query(Task).filter(Task.dag == id).filter(
            Task.type != TaskType.Service.value).order_by(Task.id).all()
        ids = {t.id for t in tasks}
        deps = self.query(TaskDependence).filter(TaskDependence.task_id.in_(ids)).all()
        nodes = [{'id': t.id, 'label': f'{t.name} {t.id}', 'name': t.name,
                  'status': to_snake(TaskStatus(t.status).name)} for t in tasks]
        edges = [{'from': d.depend_id, 'to': d.task_id,
                  'status': to_snake(TaskStatus(next(t.status for t in tasks if t.id == d.depend_id)).name)}
                 for d in deps if d.depend_id in ids]
        return {'nodes': nodes, 'edges': edges}

    def config(self, id: int) -> str:
        return self.by_id(id).config

    def add_tag(self, dag: int, tag: str):
        self.add(DagTag(dag=dag, tag=tag))

    def remove_tag(self, dag: int, tag: str):
        self.query(DagTag).filter(DagTag.dag == dag).filter(DagTag.tag == tag).delete(
            synchronize_session=False)
        self.commit()

    def tags(self, name: str = ''):
        q = self.query(DagTag.tag).distinct()
        if name:
            q = q.filter(DagTag.tag.like(f'%{name}%'))
        return [r[0] for r in q.all()]

    def last_by_name(self, project: int, name: str, type_: Optional[int] = None):
        q = self.query(Dag).filter(Dag.project == project).filter(Dag.name == name)
        if type_ is not None:
            q = q.filter(Dag.type == type_)
        return q.order_by(Dag.id.desc()).first()


class DagStorageProvider(BaseDataProvider):
    model = DagStorage

    def by_dag(self, dag: int):
        return self.query(DagStorage, File).outerjoin(File, File.id == DagStorage.file).filter(
            DagStorage.dag == dag).order_by(DagStorage.path).all()


class DagLibraryProvider(BaseDataProvider):
    model = DagLibrary

    def dag(self, dag: int):
        return [(l.library, l.version) for l in self.query(DagLibrary).filter(DagLibrary.dag == dag)]


class FileProvider(BaseDataProvider):
    model = File

    def hashs(self, project: int) -> Dict[str, int]:
        return {md5: id for id, md5 in self.query(File.id, File.md5).filter(File.project == project)}


# ---------------------------------------------------------------------------- computers
class ComputerProvider(BaseDataProvider):
    model = Computer

    def by_name(self, name: str) -> Optional[Computer]:
        return self.query(Computer).filter(Computer.name == name).one_or_none()

    def computers(self) -> Dict[str, dict]:
        return {c.name: {k: v for k, v in c.to_dict().items()} for c in self.query(Computer).all()}

    def get(self, filter: Optional[dict] = None, options=None):
        res = []
        for c in self.query(Computer).order_by(Computer.name).all():
            item = c.to_dict()
            item['usage'] = json.loads(c.usage) if c.usage else None
            item['meta'] = json.loads(c.meta) if c.meta else None
            dockers = self.query(Docker).filter(Docker.computer == c.name).all()
            item['dockers'] = [d.to_dict() for d in dockers]
            res.append(item)
        return {'total': len(res), 'data': res}

    def current_usage(self, name: str, usage: dict):
        c = self.by_name(name)
        if c is not None:
            c.usage = json.dumps(usage)
            self.commit()

    def add_usage(self, name: str, usage: dict):
        self.add(ComputerUsage(computer=name, usage=json.dumps(usage), time=now()))

    def usage_history(self, name: str, min_time: datetime.datetime):
        rows = self.query(ComputerUsage).filter(ComputerUsage.computer == name).filter(
            ComputerUsage.time >= min_time).order_by(ComputerUsage.time).all()
        return [{'time': r.time.isoformat(), **json.loads(r.usage)} for r in rows]

    def all_with_last_activity(self):
        out = []
        for c in self.query(Computer).all():
            last = self.query(func.max(Docker.last_activity)).filter(Docker.computer == c.name).scalar()
            out.append((c, last))
        return out


class DockerProvider(BaseDataProvider):
    model = Docker

    def get(self, computer: str, name: str) -> Optional[Docker]:
        return self.query(Docker).filter(Docker.computer == computer).filter(Docker.name == name).one_or_none()

    def get_online(self, seconds: int = 30) -> List[Docker]:
        min_time = now() - datetime.timedelta(seconds=seconds)
        return self.query(Docker).filter(Docker.last_activity >= min_time).all()

    def queues_online(self, seconds: int = 30):
        return [(d.computer, d.name) for d in self.get_online(seconds)]

    def heartbeat(self, computer: str, name: str, ports: str = None):
        d = self.get(computer, name)
        if d is None:
            from mlcomp_amd import config
            pr = ports or '-'.join(map(str, config.get().MASTER_PORT_RANGE))
            self.add(Docker(name=name, computer=computer, last_activity=now(), ports=pr))
        else:
            d.last_activity = now()
            self.commit()


class TaskSyncedProvider(BaseDataProvider):
    model = TaskSynced

    def for_computer(self, name: str):
        """(project, [task ids]) of Success tasks computed elsewhere, not yet synced here."""
        synced = self.query(TaskSynced.task).filter(TaskSynced.computer == name)
        q = self.query(Task, Project).join(Dag, Dag.id == Task.dag).join(
            Project, Project.id == Dag.project).filter(
            Task.status == TaskStatus.Success.value).filter(
            Task.computer_assigned.isnot(None)).filter(Task.computer_assigned != name).filter(
            Task.id.notin_(synced))
        res = defaultdict(list)
        projects = {}
        for t, p in q.all():
            res[p.id].append(t)
            projects[p.id] = p
        return [(projects[k], v) for k, v in res.items()]


# ---------------------------------------------------------------------------- logs/steps
class LogProvider(BaseDataProvider):
    model = Log

    def get(self, filter: dict, options: Optional[PaginatorOptions] = None):
        q = self.query(Log, Step.name).outerjoin(Step, Step.id == Log.step)
        if filter.get('task'):
            tasks = [filter['task']] + [t.id for t in TaskProvider(self.session).children(filter['task'])]
            q = q.filter(Log.task.in_(tasks))
        if filter.get('dag'):
            q = q.join(Task, Task.id == Log.task).filter(Task.dag == filter['dag'])
        if filter.get('computer'):
            q = q.filter(Log.computer == filter['computer'])
        if filter.get('step'):
            q = q.filter(Log.step == filter['step'])
        if filter.get('components'):
            q = q.filter(Log.component.in_(filter['components']))
        if filter.get('levels'):
            q = q.filter(Log.level.in_([LogStatus.from_name(l) if isinstance(l, str) else l
                                        for l in filter['levels']]))
        if filter.get('message'):
            q = q.filter(Log.message.like(f"%{filter['message']}%"))
        total = q.count()
        q = q.order_by(Log.id.desc())
        if options and options.page_size:
            q = q.offset(options.page_size * options.page_number).limit(options.page_size)
        res = []
        for l, step_name in q.all():
            item = l.to_dict()
            item['level'] = to_snake(LogStatus(l.level).name) if l.level in (10, 20, 30, 40) else l.level
            item['step_name'] = step_name
            res.append(item)
        return {'total': total, 'data': res}

    def last(self, count: int, dag: int = None, task: int = None, levels=None):
        q = self.query(Log)
        if task:
            q = q.filter(Log.task == task)
        if dag:
            q = q.join(Task, Task.id == Log.task).filter(Task.dag == dag)
        if levels:
            q = q.filter(Log.level.in_(levels))
        return q.order_by(Log.id.desc()).limit(count).all()


class StepProvider(BaseDataProvider):
    model = Step

    def last_for_task(self, task: int) -> Optional[Step]:
        return self.query(Step).filter(Step.task == task).order_by(Step.id.desc()).first()

    def unfinished(self, task: int) -> List[Step]:
        return self.query(Step).filter(Step.task == task).filter(Step.finished.is_(None)).order_by(
            Step.id).all()

    def by_task(self, task: int) -> List[Step]:
        return self.query(Step).filter(Step.task == task).order_by(Step.id).all()

    def get(self, task_id: int):
        """Step tree with per-step log-level counts."""
        steps = self.by_task(task_id)
        counts = defaultdict(lambda: defaultdict(int))
        for step, level, c in self.query(Log.step, Log.level, func.count(Log.id)).filter(
                Log.task == task_id).group_by(Log.step, Log.level).all():
            counts[step][level] = c
        nodes, stack = [], []
        for s in steps:
            item = s.to_dict()
            item['log_statuses'] = [{'name': to_snake(e.name), 'count': counts[s.id][e.value]}
                                    for e in LogStatus]
            item['children'] = []
            while stack and stack[-1]['level'] >= s.level:
                stack.pop()
            (stack[-1]['children'] if stack else nodes).append(item)
            stack.append(item)
        return nodes


# ---------------------------------------------------------------------------- reports
class ReportLayoutProvider(BaseDataProvider):
    model = ReportLayout

    def by_name(self, name: str) -> Optional[ReportLayout]:
        return self.query(ReportLayout).filter(ReportLayout.name == name).one_or_none()

    def all(self) -> Dict[str, dict]:
        """{name: parsed layout with ``extend`` inheritance resolved}."""
        from .report_info import union_layouts
        raw = {l.name: yaml.safe_load(l.content) or {} for l in self.query(ReportLayout).all()}
        return union_layouts(raw)

    def get(self, filter=None, options=None):
        rows = self.query(ReportLayout).order_by(ReportLayout.name).all()
        return {'total': len(rows), 'data': [r.to_dict() for r in rows]}

    def change(self, name: str, content: str):
        yaml.safe_load(content)
        l = self.by_name(name)
        l.content = content
        l.last_modified = now()
        self.commit()


class ReportProvider(BaseDataProvider):
    model = Report

    def get(self, filter: dict, options=None):
        q = self.query(Report, Project.name).join(Project, Project.id == Report.project)
        if filter.get('project'):
            q = q.filter(Report.project == filter['project'])
        total = q.count()
        res = []
        for r, pname in self.paginator(q.order_by(Report.id.desc()), options).all():
            item = r.to_dict()
            item['project'] = {'id': r.project, 'name': pname}
            item['tasks'] = self.query(ReportTasks).filter(ReportTasks.report == r.id).count()
            res.append(item)
        return {'total': total, 'data': res}

    def detail(self, id: int):
        """Series of every task in the report, grouped by metric name, plus layout."""
        r = self.by_id(id)
        task_ids = [t[0] for t in self.query(ReportTasks.task).filter(ReportTasks.report == id)]
        tasks = {t.id: t for t in TaskProvider(self.session).by_ids(task_ids)}
        series = self.query(ReportSeries).filter(ReportSeries.task.in_(task_ids)).order_by(
            ReportSeries.epoch).all()
        by_name = defaultdict(lambda: defaultdict(list))
        for s in series:
            by_name[s.name][(s.task, s.part, s.stage)].append(
                {'epoch': s.epoch, 'value': s.value, 'time': s.time.isoformat() if s.time else None})
        out_series = []
        for name, groups in by_name.items():
            for (task, part, stage), pts in groups.items():
                t = tasks.get(task)
                out_series.append({'name': name, 'task': task, 'task_name': t.name if t else None,
                                   'part': part, 'stage': stage, 'x': [p['epoch'] for p in pts],
                                   'y': [p['value'] for p in pts]})
        layouts = ReportLayoutProvider(self.session).all()
        return {'id': r.id, 'name': r.name, 'layout_name': r.layout,
                'layout': layouts.get(r.layout), 'series': out_series,
                'tasks': [{'id': t.id, 'name': t.name, 'score': t.score,
                           'status': to_snake(TaskStatus(t.status).name)} for t in tasks.values()]}

    def add_task(self, report: int, task: int):
        self.add(ReportTasks(report=report, task=task))

    def remove_task(self, report: int, task: int):
        self.query(ReportTasks).filter(ReportTasks.report == report).filter(
            ReportTasks.task == task).delete(synchronize_session=False)
        self.commit()


class ReportSeriesProvider(BaseDataProvider):
    model = ReportSeries

    def by_task(self, task: int, name: str = None):
        q = self.query(ReportSeries).filter(ReportSeries.task == task)
        if name:
            q = q.filter(ReportSeries.name == name)
        return q.order_by(ReportSeries.epoch).all()

    def by_dag(self, dag: int, name: str):
        return self.query(ReportSeries).join(Task, Task.id == ReportSeries.task).filter(
            Task.dag == dag).filter(ReportSeries.name == name).order_by(ReportSeries.epoch).all()


class ReportImgProvider(BaseDataProvider):
    model = ReportImg

    def get(self, filter: dict, options=None):
        q = self.query(ReportImg)
        for k in ('dag', 'task', 'project', 'group', 'part', 'epoch', 'y', 'y_pred'):
            if filter.get(k) is not None:
                q = q.filter(getattr(ReportImg, k) == filter[k])
        if filter.get('score_min') is not None:
            q = q.filter(ReportImg.score >= filter['score_min'])
        if filter.get('score_max') is not None:
            q = q.filter(ReportImg.score <= filter['score_max'])
        total = q.count()
        q = self.paginator(q.order_by(ReportImg.id), options)
        import base64
        data = []
        for r in q.all():
            item = r.to_dict()
            item['content'] = base64.b64encode(r.img).decode() if r.img else None
            data.append(item)
        return {'total': total, 'data': data}

    def remove_lower(self, task_id: int, name: str, epoch: int):
        self.query(ReportImg).filter(ReportImg.task == task_id).filter(
            ReportImg.group == name).filter(ReportImg.epoch < epoch).delete(synchronize_session=False)
        self.commit()


# ---------------------------------------------------------------------------- misc
class ModelProvider(BaseDataProvider):
    model = Model

    def get(self, filter: dict, options=None):
        q = self.query(Model, Project.name).join(Project, Project.id == Model.project)
        if filter.get('project'):
            q = q.filter(Model.project == filter['project'])
        if filter.get('name'):
            q = q.filter(Model.name.like(f"%{filter['name']}%"))
        total = q.count()
        res = []
        for m, pname in self.paginator(q.order_by(Model.id.desc()), options).all():
            item = m.to_dict()
            item['project'] = {'id': m.project, 'name': pname}
            res.append(item)
        return {'total': total, 'data': res}

    def by_project(self, project: int):
        return self.query(Model).filter(Model.project == project).all()


class AuxiliaryProvider(BaseDataProvider):
    model = Auxiliary

    def set(self, name: str, data):
        txt = data if isinstance(data, str) else yaml.safe_dump(data, default_flow_style=False)
        a = self.query(Auxiliary).filter(Auxiliary.name == name).one_or_none()
        if a is None:
            self.add(Auxiliary(name=name, data=txt))
        else:
            a.data = txt
            self.commit()

    def get(self):
        return {a.name: yaml.safe_load(a.data) for a in self.query(Auxiliary).all()}


class MemoryProvider(BaseDataProvider):
    model = Memory

    def find(self, filter: dict) -> List[Memory]:
        q = self.query(Memory)
        for k in ('model', 'variant', 'num_classes', 'img_size'):
            if filter.get(k) is not None:
                q = q.filter(getattr(Memory, k) == filter[k])
        return q.order_by(Memory.batch_size.desc()).all()

    def get(self, filter: dict, options=None):
        rows = self.find(filter or {})
        return {'total': len(rows), 'data': [r.to_dict() for r in rows]}


class SpaceProvider(BaseDataProvider):
    model = Space

    def by_name(self, name: str) -> Optional[Space]:
        return self.query(Space).filter(Space.name == name).one_or_none()

    def get(self, filter: dict, options=None):
        q = self.query(Space)
        if filter.get('name'):
            q = q.filter(Space.name.like(f"%{filter['name']}%"))
        if filter.get('parent'):
            q = q.join(SpaceRelation, SpaceRelation.child == Space.name).filter(
                SpaceRelation.parent == filter['parent'])
        total = q.count()
        res = []
        for s in q.order_by(Space.changed.desc()).all():
            item = s.to_dict()
            item['tags'] = [t[0] for t in self.query(SpaceTag.tag).filter(SpaceTag.space == s.name)]
            res.append(item)
        return {'total': total, 'data': res}

    def related(self, parent: str) -> List[Space]:
        return self.query(Space).join(SpaceRelation, SpaceRelation.child == Space.name).filter(
            SpaceRelation.parent == parent).all()

    def add_relation(self, parent: str, child: str):
        self.add(SpaceRelation(parent=parent, child=child))

    def remove_relation(self, parent: str, child: str):
        self.query(SpaceRelation).filter(SpaceRelation.parent == parent).filter(
            SpaceRelation.child == child).delete(synchronize_session=False)
        self.commit()

    def add_tag(self, space: str, tag: str):
        self.add(SpaceTag(space=space, tag=tag))

    def remove_tag(self, space: str, tag: str):
        self.query(SpaceTag).filter(SpaceTag.space == space).filter(SpaceTag.tag == tag).delete(
            synchronize_session=False)
        self.commit()


__all__ = [n for n in dir() if n.endswith('Provider')] + ['duration_format', 'parse_time']
