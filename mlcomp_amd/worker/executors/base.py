"""Executor ABC, registry, hierarchical steps and DB progress
(`mlcomp/worker/executors/base/executor.py:16-230`, `.../base/step.py:8-131`).

User code subclasses :class:`Executor`, decorates it with ``@Executor.register`` and
implements ``work()``; inside, ``self.step.start(level, name)`` / ``self.step.end(level)``
build the step tree (level 0 "main", 1 stage, 2 epoch, deeper user levels),
``self.info(...)`` logs against the current step, ``self.tqdm(it)`` writes progress into
the task row every ``interval`` seconds, and ``self.dependent_results()`` returns the
YAML results of upstream tasks.
"""
from __future__ import annotations

import time
from abc import ABC, abstractmethod
from typing import Dict, Optional

from mlcomp_amd import config
from mlcomp_amd.db.enums import ComponentType, to_snake
from mlcomp_amd.db.models import Dag, Step, Task, now
from mlcomp_amd.db.providers import StepProvider, TaskProvider, TaskSyncedProvider
from mlcomp_amd.utils.misc import yaml_dump, yaml_load


class StepWrap:
    def __init__(self, session, logger, logger_db, task: Task, task_provider: TaskProvider):
        self.step_provider = StepProvider(session)
        self.task_provider = task_provider
        self.task = task
        self.children = []
        self.step: Optional[Step] = None
        self.logger = logger
        self.logger_db = logger_db or logger

    @property
    def id(self):
        return self.step.id if self.step else None

    def _owner(self) -> Task:
        # ranks of a distributed task log into the parent's step tree
        if self.task.parent:
            return self.task_provider.by_id(self.task.parent)
        return self.task

    def enter(self):
        owner = self._owner()
        self.children = self.step_provider.unfinished(owner.id)
        if not self.children:
            self.step = self.start(0, 'main', 0)
        else:
            self.step = self.children[-1]

    def _finish_one(self):
        if not self.children:
            return
        st = self.children.pop()
        st.finished = now()
        self.step_provider.commit()
        self.step = self.children[-1] if self.children else st

    def finish(self):
        while self.children:
            self._finish_one()

    def start(self, level: int, name: str = None, index: int = None):
        if any(c.level == level and c.index == index and c.name == name for c in self.children):
            return None
        owner = self._owner()
        if index is None and owner.current_step:
            parts = owner.current_step.split('.')
            if 0 < level <= len(parts):
                index = int(parts[level - 1])
        if self.step is not None and self.children:
            diff = level - self.step.level
            assert level > 0, 'level must be positive'
            assert diff <= 1, f'level {level} can not be started after {self.step.level}'
            for _ in range(max(0, -diff + 1)):
                self._finish_one()
        st = Step(level=level, name=name or '', started=now(), task=owner.id, index=index or 0)
        self.step_provider.add(st)
        self.children.append(st)
        self.step = st
        owner.current_step = '.'.join(str(c.index + 1) for c in self.children[1:])
        self.task_provider.commit()
        return st

    def end(self, level: int):
        diff = level - self.step.level
        assert diff <= 0, 'you can end only the current step or an enclosing one'
        for _ in range(-diff + 1):
            self._finish_one()

    def _log(self, fn, message, db):
        logger = self.logger_db if db else self.logger
        if logger is None:
            print(message)
            return
        getattr(logger, fn)(message, ComponentType.Worker, self.task.computer_assigned, self.task.id,
                            self.id)

    def debug(self, m, db=False):
        self._log('debug', m, db)

    def info(self, m, db=False):
        self._log('info', m, db)

    def warning(self, m, db=False):
        self._log('warning', m, db)

    def error(self, m, db=False):
        self._log('error', m, db)


class TqdmWrapper:
    """Iterates like tqdm and writes loader_name/batch_index/batch_total/epoch_duration/
    epoch_time_remaining into the task row at most once per ``interval`` seconds."""

    def __init__(self, executor: 'Executor', iterable=None, desc='progress', interval=10, total=None):
        self.executor = executor
        self.iterable = iterable
        self.desc = desc
        self.interval = interval
        self.total = total if total is not None else (len(iterable) if hasattr(iterable, '__len__') else None)
        self.n = 0
        self.start_t = time.time()

    def refresh(self):
        t = self.executor.task
        t.loader_name = self.desc
        t.batch_index = self.n
        t.batch_total = self.total
        t.epoch_duration = int(time.time() - self.start_t)
        if self.n > 0 and self.total:
            t.epoch_time_remaining = int(t.epoch_duration * (self.total - self.n) / self.n)
        self.executor.task_provider.commit()
        return time.time()

    def set_description(self, desc=None, refresh=True):
        self.desc = desc or ''
        if refresh:
            self.refresh()

    def __iter__(self):
        last = self.refresh()
        for item in self.iterable:
            yield item
            self.n += 1
            if time.time() - last > self.interval:
                last = self.refresh()
        self.refresh()

    def __len__(self):
        return self.total or 0


class Executor(ABC):
    _child: Dict[str, type] = {}

    session = None
    task_provider: TaskProvider = None
    logger = None
    logger_db = None
    step: StepWrap = None
    task: Task = None
    dag: Dag = None

    def __init__(self, **kwargs):
        self.kwargs = kwargs

    # ------------------------------------------------------------------ logging
    def debug(self, m, db=False):
        self.step.debug(m, db) if self.step else print(m)

    def info(self, m, db=False):
        self.step.info(m, db) if self.step else print(m)

    def warning(self, m, db=False):
        self.step.warning(m, db) if self.step else print(m)

    def error(self, m, db=False):
        self.step.error(m, db) if self.step else print(m)

    # stdout sink (click executor redirects user prints here)
    def write(self, message: str):
        if message.strip():
            self.info(message.rstrip('\n'), db=True)

    def flush(self):
        pass

    def add_child_process(self, pid: int):
        info = yaml_load(self.task.additional_info) or {}
        info['child_processes'] = info.get('child_processes', []) + [pid]
        self.task.additional_info = yaml_dump(info)
        self.task_provider.commit()

    # ------------------------------------------------------------------ lifecycle
    def __call__(self, *, task: Task, task_provider: TaskProvider, dag: Dag) -> dict:
        self.task_provider = task_provider
        self.task = task
        self.dag = dag
        self.step = StepWrap(self.session, self.logger, self.logger_db, task, task_provider)
        self.step.enter()
        if not task.debug and config.get().FILE_SYNC_INTERVAL:
            self.wait_data_sync()
        from mlcomp_amd.utils import faults
        faults.arm_task_kill()
        faults.maybe_crash_task()
        res = self.work()
        self.task_provider.commit()
        return res

    @abstractmethod
    def work(self) -> dict:
        ...

    @classmethod
    def _from_config(cls, executor: dict, config_: dict, additional_info: dict) -> 'Executor':
        kw = {k: v for k, v in executor.items() if k not in ('type', 'depends', 'gpu', 'cpu',
                                                              'memory', 'distr', 'single_node',
                                                              'grid', 'env', 'task_type',
                                                              'computer', 'steps', 'slot')}
        return cls(**kw)

    @staticmethod
    def from_config(*, executor: str, config: dict, additional_info: dict, session, logger,
                    logger_db) -> 'Executor':
        if executor not in config.get('executors', {}):
            raise ModuleNotFoundError(f'Executor {executor} has not been found')
        ex = additional_info.get('executor') or config['executors'][executor]
        t = ex['type']
        if t not in Executor._child:
            raise ModuleNotFoundError(f'Executor type {t} is not registered')
        res = Executor._child[t]._from_config(ex, config, additional_info)
        res.session = session
        res.logger = logger
        res.logger_db = logger_db
        return res

    @staticmethod
    def register(cls):
        for n in (cls.__name__, cls.__name__.lower(), to_snake(cls.__name__)):
            Executor._child[n] = cls
        return cls

    @staticmethod
    def is_registered(name: str) -> bool:
        return name in Executor._child

    @staticmethod
    def is_trainable(type_: str) -> bool:
        return type_.lower() in ('catalyst', 'train', 'native_train')

    def wait_data_sync(self):
        self.info('Start data sync')
        while True:
            provider = TaskSyncedProvider(self.session)
            if not any(p.id == self.dag.project for p, _ in provider.for_computer(self.task.computer_assigned)):
                break
            time.sleep(1)
        self.info('Finish data sync')

    def tqdm(self, iterable=None, desc='progress', interval=10, **kwargs):
        return TqdmWrapper(self, iterable, desc=desc, interval=interval, total=kwargs.get('total'))

    def dependent_results(self) -> dict:
        return {t.id: yaml_load(t.result) for t in self.task_provider.find_dependents(self.task.id)}


__all__ = ['Executor', 'StepWrap', 'TqdmWrapper']
