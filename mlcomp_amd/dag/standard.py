"""YAML DAG -> Project/Dag/Task/TaskDependence/Report rows.

Schema (unchanged from the reference, `docs/usage.rst:13-63`,
`mlcomp/server/back/create_dags/standard.py:21-341`)::

    info:      {name, project, layout?, expdir?, type?: standard|pipe, docker_img?,
                computer?, seed?}
    executors: {<name>: {type, depends?: str|list, gpu?: int|"a-b", cpu?, memory?,
                         distr?, single_node?, grid?, env?, task_type?, computer?,
                         steps?, ...executor kwargs}}
    grid:      (optional) DAG-level grid -> one DAG per cell (handled by the caller)

Differences: executors are ordered with Kahn's algorithm (cycles are reported instead
of looping forever), the whole schema is validated before any row is written, and all
rows of one DAG are inserted in a single transaction.
"""
from __future__ import annotations

import os
from collections import OrderedDict, deque
from copy import deepcopy
from typing import Dict, List, Optional, Tuple

from mlcomp_amd.db.core import Session
from mlcomp_amd.db.enums import DagType, TaskType
from mlcomp_amd.db.models import Dag, Report, ReportTasks, Task, TaskDependence, now
from mlcomp_amd.db.providers import DagProvider, ProjectProvider, ReportLayoutProvider
from mlcomp_amd.utils.misc import grid_cells, parse_gpu_range, yaml_dump

TRAINABLE = {'catalyst', 'train', 'native_train'}
RESERVED = {'type', 'depends', 'gpu', 'cpu', 'memory', 'distr', 'single_node', 'grid', 'env',
            'task_type', 'computer', 'steps', 'name'}


class DagConfigError(ValueError):
    pass


def validate(config: dict):
    if not isinstance(config, dict):
        raise DagConfigError('config must be a mapping')
    info = config.get('info')
    if not isinstance(info, dict):
        raise DagConfigError('config must have an info section')
    for k in ('name', 'project'):
        if not info.get(k):
            raise DagConfigError(f'info.{k} is required')
    ex = config.get('executors')
    if not isinstance(ex, dict) or not ex:
        raise DagConfigError('config must have a non-empty executors section')
    for name, v in ex.items():
        if not isinstance(v, dict) or 'type' not in v:
            raise DagConfigError(f'executor {name}: a mapping with a "type" is required')
        deps = v.get('depends', [])
        deps = deps if isinstance(deps, list) else [deps]
        for d in deps:
            if d == name:
                raise DagConfigError(f'Executor {name} depends on itself')
            if d not in ex:
                raise DagConfigError(f'Executor {name} depends on {d} which does not exist')
        try:
            g, gmax = parse_gpu_range(v.get('gpu', 0))
        except ValueError:
            raise DagConfigError(f'executor {name}: bad gpu spec {v.get("gpu")!r}')
        if g == 0 and gmax > 0:
            raise DagConfigError(f"Executor {name}: gpu_max can't be > 0 when gpu = 0")
        if gmax < g:
            raise DagConfigError(f'executor {name}: gpu range {v.get("gpu")} is reversed')


def topo_order(executors: dict) -> List[str]:
    deps = {k: (v.get('depends', []) if isinstance(v.get('depends', []), list) else [v['depends']])
            for k, v in executors.items()}
    indeg = {k: len(set(d)) for k, d in deps.items()}
    users = {k: [] for k in executors}
    for k, d in deps.items():
        for x in set(d):
            users[x].append(k)
    q = deque(k for k in executors if indeg[k] == 0)
    order = []
    while q:
        k = q.popleft()
        order.append(k)
        for u in users[k]:
            indeg[u] -= 1
            if indeg[u] == 0:
                q.append(u)
    if len(order) != len(executors):
        raise DagConfigError(f'dependency cycle among {sorted(set(executors) - set(order))}')
    return order


class DagStandardBuilder:
    def __init__(self, session: Session, config: dict, debug: bool = False, config_text: str = None,
                 upload_files: bool = True, copy_files_from: int = None, config_path: str = None,
                 control_reqs: bool = True, logger=None, component=None,
                 grid_cell: Optional[Tuple[dict, str]] = None):
        validate(config)
        self.session = session
        self.config = config
        self.debug = debug
        self.config_text = config_text
        self.upload_files = upload_files
        self.copy_files_from = copy_files_from
        self.config_path = config_path
        self.control_reqs = control_reqs
        self.logger = logger
        self.component = component
        self.grid_cell = grid_cell
        self.info = config['info']
        self.layout_name = self.info.get('layout')
        self.created: Dict[str, List[int]] = OrderedDict()

    def _log(self, msg):
        if self.logger:
            self.logger.info(msg, self.component)

    def load_base(self):
        pp = ProjectProvider(self.session)
        project = pp.by_name(self.info['project']) or pp.add_project(self.info['project'])
        self.project = project.id
        self.layouts = ReportLayoutProvider(self.session).all()
        if self.layout_name and self.layout_name not in self.layouts:
            raise DagConfigError(f'Unknown layout = {self.layout_name}')

    def create_report(self):
        self.dag_report_id = None
        if self.layout_name:
            r = Report(config=yaml_dump(self.layouts[self.layout_name]), name=self.info['name'],
                       project=self.project, layout=self.layout_name, time=now())
            self.session.add(r, commit=False)
            self.session.flush()
            self.dag_report_id = r.id

    def create_dag(self):
        name = self.info['name']
        if self.grid_cell:
            name = f'{name} {self.grid_cell[1]}'
        dag = Dag(config=self.config_text or yaml_dump(self.config), project=self.project, name=name,
                  docker_img=self.info.get('docker_img'),
                  type=DagType.Pipe.value if self.info.get('type') == 'pipe' else DagType.Standard.value,
                  created=now(), report=self.dag_report_id, file_size=0, img_size=0)
        self.session.add(dag, commit=False)
        self.session.flush()
        self.dag = dag

    def upload(self):
        from mlcomp_amd.worker.storage import Storage
        storage = Storage(self.session, logger=self.logger, component=self.component)
        if self.upload_files and self.config_path:
            folder = os.path.dirname(os.path.abspath(self.config_path))
            if 'expdir' in self.info:
                folder = os.path.abspath(os.path.join(folder, self.info['expdir']))
            storage.upload(folder, self.dag, control_reqs=self.control_reqs)
        elif self.copy_files_from:
            storage.copy_from(self.copy_files_from, self.dag)

    def _task(self, k: str, v: dict, name: str, info: dict, cell: dict):
        v = deepcopy(v)
        ttype = TaskType.Train.value if (v.get('task_type') == 'train'
                                          or str(v['type']).lower() in TRAINABLE) else TaskType.User.value
        gpu, gpu_max = parse_gpu_range(v.get('gpu', 0))
        v.update(cell or {})
        info = dict(info)
        info['executor'] = v
        report = None
        if self.layout_name and ttype == TaskType.Train.value:
            info['report_config'] = self.layouts[self.layout_name]
            report = Report(config=yaml_dump(self.layouts[self.layout_name]), name=name,
                            project=self.project, layout=self.layout_name, time=now())
        t = Task(name=name, executor=k, computer=self.info.get('computer') or v.get('computer'),
                 gpu=gpu, gpu_max=gpu_max, cpu=int(v.get('cpu', 1)), memory=float(v.get('memory', 0.1)),
                 dag=self.dag.id, debug=self.debug, steps=int(v.get('steps', 1)), type=ttype,
                 status=0, continued=False, additional_info=yaml_dump(info))
        return t, report

    def create_tasks(self):
        executors = self.config['executors']
        order = topo_order(executors)
        created: Dict[str, List[Task]] = OrderedDict()
        deps = []
        for k in order:
            v = deepcopy(executors[k])
            if self.grid_cell:
                v.update(self.grid_cell[0])
            if 'grid' in v:
                grid = v.pop('grid')
                cells = [(c, n, {'grid_cell': i}) for i, (c, n) in enumerate(grid_cells(grid))]
            else:
                cells = [({}, v.get('name', k), {})]
            ktasks = []
            for cell, name, info in cells:
                t, rep = self._task(k, v, name, info, cell)
                if rep is not None:
                    self.session.add(rep, commit=False)
                    self.session.flush()
                    t.report = rep.id
                self.session.add(t, commit=False)
                self.session.flush()
                if rep is not None:
                    self.session.add(ReportTasks(report=rep.id, task=t.id), commit=False)
                if self.dag_report_id is not None and rep is not None:
                    self.session.add(ReportTasks(report=self.dag_report_id, task=t.id), commit=False)
                ktasks.append(t)
                d = v.get('depends', [])
                for dn in (d if isinstance(d, list) else [d]):
                    deps.extend((t.id, dd.id) for dd in created[dn])
            created[k] = ktasks
        self.session.add_all([TaskDependence(task_id=a, depend_id=b) for a, b in deps], commit=False)
        self.created = OrderedDict((k, [t.id for t in v]) for k, v in created.items())

    def build(self) -> Dict[str, List[int]]:
        try:
            self.load_base()
            self.create_report()
            self.create_dag()
            self.upload()
            self.create_tasks()
            self.session.commit()
        except Exception:
            self.session.rollback()
            raise
        self._log(f'dag {self.dag.id} created: {dict(self.created)}')
        return self.created


def dag_standard(session: Session, config: dict, debug: bool = False, config_text: str = None,
                 upload_files: bool = True, copy_files_from: int = None, config_path: str = None,
                 control_reqs: bool = True, logger=None, component=None, grid_cell=None):
    return DagStandardBuilder(session, config, debug, config_text, upload_files, copy_files_from,
                              config_path, control_reqs, logger, component, grid_cell).build()


def dag_from_config(session: Session, config: dict, config_path: str = None, config_text: str = None,
                    debug: bool = False, params: dict = None, logger=None, component=None,
                    control_reqs: bool = True) -> List[Dict[str, List[int]]]:
    """Top-level entry used by ``mlcomp dag``: applies ``--params`` overrides and the
    DAG-level ``grid`` (one DAG per cell, `mlcomp/__main__.py:37-75`)."""
    from mlcomp_amd.utils.misc import merge_dicts_smart
    if params:
        config = merge_dicts_smart(config, params)
        config_text = yaml_dump(config)
    if config.get('info', {}).get('type') == 'pipe':
        from .pipe import dag_pipe
        return [dag_pipe(session, config, config_text)]
    grid = config.get('grid')
    if not grid:
        return [dag_standard(session, config, debug, config_text, config_path=config_path,
                             logger=logger, component=component, control_reqs=control_reqs)]
    cfg = {k: v for k, v in config.items() if k != 'grid'}
    out = []
    for cell in grid_cells(grid):
        out.append(dag_standard(session, deepcopy(cfg), debug, yaml_dump(cfg), config_path=config_path,
                                logger=logger, component=component, grid_cell=cell,
                                control_reqs=control_reqs))
    return out


__all__ = ['DagStandardBuilder', 'dag_standard', 'dag_from_config', 'validate', 'topo_order',
           'DagConfigError']
