"""Task lifecycle on a worker (`mlcomp/worker/tasks.py:31-306` equivalent).

``execute_by_id`` runs ONE task in the current process: load task+dag, seed, map the
task's assigned GPU indices through any inherited device mask (``HIP_VISIBLE_DEVICES``
/ ``CUDA_VISIBLE_DEVICES`` - both are set so PyTorch-ROCm and raw HIP agree), apply the
executor's ``env``, guard against duplicate delivery, mark InProgress, materialise the
code, import the executor (framework executors first, then the task folder), run it,
store its result and mark Success - or log the traceback and mark Failed.  A
multi-stage executor that returns ``{stage, stages}`` with stages left is re-queued to
the worker's personal queue (stage-granular continuation of DDP training).

The worker pool (`mlcomp_amd.worker.pool`) launches each task in a fresh child
process, so every task gets a clean HIP context; the control-queue handlers
(``kill``, ``kill_all``, ``remove``) run in the worker-supervisor daemon.
"""
from __future__ import annotations

import os
import shutil
import signal
import socket
import sys
import time
import traceback

from mlcomp_amd import config
from mlcomp_amd.broker import get_broker, queue_name
from mlcomp_amd.db.core import Session
from mlcomp_amd.db.enums import ComponentType, TaskStatus
from mlcomp_amd.db.providers import DagLibraryProvider, DagProvider, TaskProvider
from mlcomp_amd.utils.logging import create_logger
from mlcomp_amd.utils.misc import (kill_child_processes, kill_pid, set_global_seed, yaml_dump,
                                   yaml_load)


def hostname() -> str:
    return os.environ.get('MLCOMP_COMPUTER') or socket.gethostname()


def map_visible_devices(gpu_assigned: str, inherited: str) -> str:
    """Indices assigned by the scheduler are relative to the worker's own device mask."""
    gpu_assigned = gpu_assigned or ''
    idx = [int(g) for g in gpu_assigned.split(',') if g.strip() != '']
    if inherited.strip():
        base = [d.strip() for d in inherited.split(',')]
        return ','.join(base[i] for i in idx)
    return ','.join(map(str, idx))


class ExecuteBuilder:
    def __init__(self, task_id: int, repeat_count: int = 1, exit_process: bool = False):
        self.session = Session.create_session(key='ExecuteBuilder')
        self.id = task_id
        self.repeat_count = repeat_count
        self.exit_process = exit_process
        self.logger = create_logger(self.session, 'ExecuteBuilder')
        self.logger_db = create_logger(self.session, 'ExecuteBuilder.db', console=False)
        self.executor = None
        self.task = None

    def _log(self, level, msg, step=None):
        getattr(self.logger, level)(msg, ComponentType.Worker, hostname(), self.id, step)

    def create_base(self):
        s = config.get()
        self.provider = TaskProvider(self.session)
        self.task = self.provider.by_id(self.id)
        if self.task is None:
            raise RuntimeError(f'task {self.id} not found')
        self.dag = DagProvider(self.session).by_id(self.task.dag)
        self.config = yaml_load(self.dag.config) or {}
        set_global_seed(self.config.get('info', {}).get('seed', 0))
        self.executor_cfg = self.config['executors'][self.task.executor]
        self.executor_type = self.executor_cfg['type']
        self.worker_index = s.WORKER_INDEX
        self.queue_personal = queue_name(hostname(), s.DOCKER_IMG, self.worker_index)
        inherited = os.environ.get('HIP_VISIBLE_DEVICES') or os.environ.get('CUDA_VISIBLE_DEVICES', '')
        # a DDP rank sees every GPU of its job on this computer (distr_info.visible_gpus) and
        # selects its own by local_rank, so RCCL can connect the ranks peer-to-peer over xGMI
        di = (yaml_load(self.task.additional_info) or {}).get('distr_info') or {}
        assigned = di.get('visible_gpus') if di.get('visible_gpus') is not None else self.task.gpu_assigned
        if assigned is not None or inherited:
            vis = map_visible_devices(assigned or '', inherited)
            env = {'HIP_VISIBLE_DEVICES': vis, 'CUDA_VISIBLE_DEVICES': vis}
        else:
            env = {}
        env.update({'MKL_NUM_THREADS': os.environ.get('MKL_NUM_THREADS', '1'),
                    'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS', '1')})
        env.update({k: str(v) for k, v in (self.executor_cfg.get('env') or {}).items()})
        for k, v in env.items():
            os.environ[k] = str(v)
        self._log('debug', f'env {env}')

    def check_status(self) -> bool:
        if self.task.status >= TaskStatus.InProgress.value:
            self._log('error', f'task {self.id} has status {TaskStatus(self.task.status).name} '
                               f'before execution (duplicate delivery?)')
            return False
        return True

    def change_status(self):
        t = self.task
        t.computer_assigned = hostname()
        t.pid = os.getpid()
        t.worker_index = self.worker_index
        t.docker_assigned = config.get().DOCKER_IMG
        self.provider.change_status(t, TaskStatus.InProgress)

    def download(self):
        from mlcomp_amd.worker.executors import Executor, load_builtin_executors
        from mlcomp_amd.worker.storage import Storage
        load_builtin_executors(self.executor_type)
        if self.task.debug:
            folder = os.getcwd()
        else:
            folder = Storage(self.session).download(self.id)
        os.chdir(folder)
        if folder not in sys.path:
            sys.path.insert(0, folder)
        if not Executor.is_registered(self.executor_type):
            libs = DagLibraryProvider(self.session).dag(self.task.dag)
            found, _ = Storage(self.session, logger=self.logger,
                               component=ComponentType.Worker).import_executor(folder, self.executor_type, libs)
            if not found or not Executor.is_registered(self.executor_type):
                raise ModuleNotFoundError(f'Executor {self.executor_type} not found')

    def create_executor(self):
        from mlcomp_amd.worker.executors import Executor
        # again now that the executor's modules are imported (torch, if it uses it)
        set_global_seed(self.config.get('info', {}).get('seed', 0))
        info = yaml_load(self.task.additional_info) or {}
        self.executor = Executor.from_config(executor=self.task.executor, config=self.config,
                                             additional_info=info, session=self.session,
                                             logger=self.logger, logger_db=self.logger_db)

    def execute(self):
        res = self.executor(task=self.task, task_provider=self.provider, dag=self.dag) or {}
        self.task.result = yaml_dump(res)
        self.provider.commit()
        if 'stage' in res and 'stages' in res:
            i = res['stages'].index(res['stage'])
            if i < len(res['stages']) - 1:
                self.executor.info(f'stage {res["stage"]} done, next {res["stages"][i + 1]}')
                self.task.status = TaskStatus.Queued.value
                self.provider.commit()
                mid = get_broker().send_task(self.queue_personal, 'execute', self.id)
                # the scheduler's orphan pass checks the broker for task.celery_id: point it
                # at the continuation message (the stage's own message is acked by now)
                self.task.celery_id = mid
                self.provider.commit()
                return
        self.executor.step.finish()
        self.provider.change_status(self.task, TaskStatus.Success)

    def build(self):
        try:
            self.create_base()
            if not self.check_status():
                return
            self.change_status()
            self.download()
            self.create_executor()
            self.execute()
        except BaseException as e:
            step = self.executor.step.id if (self.executor and self.executor.step) else None
            if Session.sqlalchemy_error(e):
                Session.cleanup('ExecuteBuilder')
                self.session = Session.create_session(key='ExecuteBuilder')
                self.logger = create_logger(self.session, 'ExecuteBuilder')
                self.provider = TaskProvider(self.session)
                self.task = self.provider.by_id(self.id)
            self._log('error', traceback.format_exc(), step)
            if self.task is not None and self.task.status <= TaskStatus.InProgress.value:
                self.provider.change_status(self.task, TaskStatus.Failed)
            if not isinstance(e, Exception):
                raise
        finally:
            if self.exit_process:
                sys.stdout.flush()
                os._exit(0)


def execute_by_id(task_id: int, repeat_count: int = 1, exit_process: bool = False):
    ExecuteBuilder(task_id, repeat_count, exit_process).build()


# ---------------------------------------------------------------------------- control
def kill(pid: int) -> bool:
    kill_child_processes(pid)
    return kill_pid(pid)


def kill_all(pids):
    return [kill(p) for p in pids]


def remove(path: str) -> bool:
    if os.path.isdir(path):
        shutil.rmtree(path, ignore_errors=True)
        return True
    if os.path.exists(path):
        os.remove(path)
        return True
    return False


CONTROL_TASKS = {'kill': kill, 'kill_all': kill_all, 'remove': remove}


def remove_from_all(session, path: str):
    """Ask every online computer's supervisor queue to delete ``path`` (fire-and-forget)."""
    from mlcomp_amd.broker import get_broker, queue_name
    from mlcomp_amd.db.providers import DockerProvider
    b = get_broker()
    for d in DockerProvider(session).get_online():
        try:
            b.send_task(queue_name(d.computer, d.name or 'default', 'supervisor'), 'remove', path)
        except Exception:
            pass
    remove(path) if os.path.exists(path) else None


def remove_model_files(session, project_name: str, model_name: str):
    s = config.get()
    for suffix in ('.pth', '_weight.pth'):
        remove_from_all(session, os.path.join(s.MODEL_FOLDER, project_name, model_name + suffix))


def remove_task_files(session, task_id: int):
    remove_from_all(session, os.path.join(config.get().TASK_FOLDER, str(task_id)))


def remove_dag_files(session, dag_id: int):
    from mlcomp_amd.db.providers import TaskProvider
    for t in TaskProvider(session).by_dag(dag_id):
        remove_task_files(session, t.id)


if __name__ == '__main__':  # python -m mlcomp_amd.worker.tasks <task_id>
    execute_by_id(int(sys.argv[1]), exit_process=False)
