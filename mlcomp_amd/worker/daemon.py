"""Per-computer worker runtime: the worker pool and the worker-supervisor daemon.

``WorkerPool`` (``mlcomp-worker worker N``) - one consumer per worker slot popping
``{host}_{docker}_{N}`` (personal) then ``{host}_{docker}`` (shared) and running each
task in a FRESH child process (``python -m mlcomp_amd.worker.tasks <id>``): process-per-
task isolation like the reference's ``os._exit`` + supervisord restart
(`mlcomp/worker/tasks.py:299-301`), without re-exec'ing a process that touched the GPU.
The message is acked only after the child exits, so a pool that dies mid-task hands the
message back to the broker (duplicate delivery is rejected by the task status check).

``WorkerSupervisor`` (``mlcomp-worker worker-supervisor``,
`mlcomp/worker/__main__.py:41-161,181-219`) - registers the Computer/Docker rows,
heartbeats, samples usage (psutil + amdsmi for MI355X util / VRAM / power /
temperature), fails InProgress tasks whose process died (pid gone and idle > 30 s),
kills orphaned task processes whose task was stopped, serves the control queue
``{host}_{docker}_supervisor`` (kill / kill_all / remove) and runs file sync.
"""
from __future__ import annotations

import datetime
import json
import os
import subprocess
import sys
import threading
import time
import traceback
from typing import List, Optional

import psutil

from mlcomp_amd import config
from mlcomp_amd.broker import new_connection, queue_name
from mlcomp_amd.db.core import Session
from mlcomp_amd.db.enums import ComponentType, TaskStatus
from mlcomp_amd.db.models import Computer, now
from mlcomp_amd.db.providers import ComputerProvider, DockerProvider, TaskProvider
from mlcomp_amd.utils.logging import create_logger
from mlcomp_amd.utils.misc import kill_child_processes, kill_pid, yaml_load
from .tasks import CONTROL_TASKS, hostname


# ---------------------------------------------------------------------------- GPU info
class GpuInfo:
    """MI355X metrics through amdsmi (no HIP context is created)."""

    def __init__(self):
        self.handles = []
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi = amdsmi
            self.handles = amdsmi.amdsmi_get_processor_handles()
        except Exception:
            self.smi = None

    def count(self) -> int:
        if self.handles:
            return len(self.handles)
        env = os.environ.get('MLCOMP_GPU_COUNT')
        return int(env) if env else 0

    def sample(self) -> List[dict]:
        out = []
        for i, h in enumerate(self.handles):
            d = {'index': i}
            try:
                d['load'] = float(self.smi.amdsmi_get_gpu_activity(h)['gfx_activity'])
            except Exception:
                pass
            try:
                v = self.smi.amdsmi_get_gpu_vram_usage(h)
                d['memory'] = 100.0 * v['vram_used'] / max(1, v['vram_total'])
                d['memory_total_mb'] = v['vram_total']
            except Exception:
                pass
            try:
                d['power'] = float(self.smi.amdsmi_get_power_info(h).get('socket_power', 0))
            except Exception:
                pass
            out.append(d)
        return out


def usage_snapshot(gpu: GpuInfo) -> dict:
    vm = psutil.virtual_memory()
    du = psutil.disk_usage(config.get().ROOT_FOLDER)
    return {'cpu': psutil.cpu_percent(), 'memory': vm.percent, 'disk': du.percent,
            'gpu': gpu.sample()}


def register_computer(session, gpu: GpuInfo, can_process: Optional[bool] = None):
    s = config.get()
    name = hostname()
    cp = ComputerProvider(session)
    c = Computer(name=name, gpu=gpu.count(), cpu=psutil.cpu_count(),
                 memory=psutil.virtual_memory().total / 2 ** 20, ip=s.IP, port=s.PORT,
                 user=os.environ.get('USER', ''), disk=int(psutil.disk_usage(s.ROOT_FOLDER).total / 2 ** 30),
                 root_folder=s.ROOT_FOLDER,
                 can_process_tasks=s.CAN_PROCESS_TASKS if can_process is None else can_process,
                 sync_with_this_computer=s.SYNC_WITH_THIS_COMPUTER)
    cp.create_or_update(c, 'name')
    DockerProvider(session).heartbeat(name, s.DOCKER_IMG, '-'.join(map(str, s.MASTER_PORT_RANGE)))
    return name


# ---------------------------------------------------------------------------- pool
# the log line of a task whose process died (the scheduler's bounded restart matches it)
PROCESS_LOST_MESSAGE = 'task process was lost'


class WorkerPool:
    def __init__(self, indices: List[int], docker: Optional[str] = None, poll: float = 1.0):
        self.indices = indices
        self.docker = docker or config.get().DOCKER_IMG
        self.poll = poll
        self._stop = threading.Event()
        self.threads = []
        self.running = {}

    def _slot(self, index: int):
        host = hostname()
        queues = [queue_name(host, self.docker, index), queue_name(host, self.docker)]
        broker = new_connection()
        while not self._stop.is_set():
            try:
                item = broker.pop(queues, self.poll)
            except Exception:
                time.sleep(1)
                continue
            if item is None:
                continue
            _, msg = item
            try:
                if msg.get('task') == 'execute':
                    env = dict(os.environ, WORKER_INDEX=str(index))
                    p = subprocess.Popen([sys.executable, '-m', 'mlcomp_amd.worker.tasks',
                                          str(msg['args'][0])], env=env)
                    self.running[index] = p
                    rc = p.wait()
                    self.running.pop(index, None)
                    if rc != 0:
                        self._process_lost(index, int(msg['args'][0]), rc)
                elif msg.get('task') in CONTROL_TASKS:
                    res = CONTROL_TASKS[msg['task']](*msg.get('args', []))
                    if msg.get('reply'):
                        broker.set_result(msg['reply'], res)
            finally:
                try:
                    broker.ack(msg['id'])
                except Exception:
                    pass  # broker gone: the lease is re-queued by the broker itself

    def _process_lost(self, index: int, task_id: int, rc: int):
        """A task process that exited abnormally while its task is still InProgress (killed:
        OOM killer, a crashed driver, an injected fault) is failed at once - the liveness
        scan of the worker supervisor would only see the missing pid after its grace."""
        try:
            session = Session.create_session(key=f'WorkerPool-{index}')
            session.expire_all()
            tp = TaskProvider(session)
            t = tp.by_id(task_id)
            # only a task still InProgress is failed here.  A straggler rank the scheduler
            # stops on purpose is set Success before its kill (supervisor: parent finished),
            # so the status test already covers it; the killed_by_supervisor mark is checked
            # first anyway, so a kill that races the status write is never reported as lost
            info = yaml_load(t.additional_info) or {} if t is not None else {}
            if t is None or info.get('killed_by_supervisor') or t.status != TaskStatus.InProgress.value:
                return
            for pid in info.get('child_processes', []):
                kill_pid(pid)
            create_logger(session, 'WorkerPool', console=False).error(
                f'{PROCESS_LOST_MESSAGE} (task {task_id}, exit code {rc})', ComponentType.Worker, hostname(), task_id)
            tp.change_status(t, TaskStatus.Failed)
        except Exception:
            traceback.print_exc()

    def start(self):
        for i in self.indices:
            t = threading.Thread(target=self._slot, args=(i,), daemon=True, name=f'worker-{i}')
            t.start()
            self.threads.append(t)
        return self

    def stop(self, timeout: float = 5.0):
        self._stop.set()
        for p in list(self.running.values()):
            try:
                p.terminate()
            except Exception:
                pass
        for t in self.threads:
            t.join(timeout)

    def join(self):
        for t in self.threads:
            t.join()


# ---------------------------------------------------------------------------- supervisor
class WorkerSupervisor:
    def __init__(self, session_key='WorkerSupervisor', liveness_period=10.0, grace=30.0):
        self.session = Session.create_session(key=session_key)
        self.logger = create_logger(self.session, 'WorkerSupervisor', console=False)
        self.gpu = GpuInfo()
        self.liveness_period = liveness_period
        self.grace = grace
        self._stop = threading.Event()
        self._usage: List[dict] = []
        self.name = register_computer(self.session, self.gpu)

    # liveness: InProgress tasks of this computer whose process is gone
    def stop_processes_not_exist(self):
        tp = TaskProvider(self.session)
        self.session.expire_all()
        for t in tp.by_status(TaskStatus.InProgress, computer_assigned=self.name):
            if t.pid is None or psutil.pid_exists(t.pid):
                continue
            if t.last_activity and (now() - t.last_activity).total_seconds() < self.grace:
                continue
            info = yaml_load(t.additional_info) or {}
            for p in info.get('child_processes', []):
                kill_pid(p)
            self.logger.error(f'{PROCESS_LOST_MESSAGE} (task {t.id}: process {t.pid} is gone)',
                              ComponentType.WorkerSupervisor, self.name, t.id)
            tp.change_status(t, TaskStatus.Failed)
        # orphans: live task processes whose task was stopped/failed/skipped
        for t in tp.by_status(TaskStatus.Stopped, TaskStatus.Failed, TaskStatus.Skipped,
                              computer_assigned=self.name):
            if t.pid and psutil.pid_exists(t.pid) and t.finished and \
                    (now() - t.finished).total_seconds() < 3600:
                try:
                    cmd = ' '.join(psutil.Process(t.pid).cmdline())
                except psutil.Error:
                    continue
                if 'mlcomp_amd.worker.tasks' in cmd:
                    kill_child_processes(t.pid)
                    kill_pid(t.pid)

    def heartbeat(self):
        from mlcomp_amd.utils import faults
        if faults.heartbeat_dropped():
            return
        s = config.get()
        u = usage_snapshot(self.gpu)
        self._usage.append(u)
        cp = ComputerProvider(self.session)
        cp.current_usage(self.name, u)
        DockerProvider(self.session).heartbeat(self.name, s.DOCKER_IMG)
        if len(self._usage) >= 6:
            n = len(self._usage)
            mean = {k: sum(x[k] for x in self._usage) / n for k in ('cpu', 'memory', 'disk')}
            # per-GPU load / memory averaged over the window like the host counters
            mean['gpu'] = [{'index': g.get('index', i),
                            **{k: sum((x['gpu'][i].get(k) or 0) for x in self._usage if i < len(x['gpu'])) / n
                               for k in ('load', 'memory') if k in g}}
                           for i, g in enumerate(u['gpu'])]
            cp.add_usage(self.name, mean)
            self._usage = []

    def _loop(self, fn, period):
        while not self._stop.is_set():
            try:
                fn()
            except Exception:
                try:
                    self.session.rollback()
                    self.logger.error(traceback.format_exc(), ComponentType.WorkerSupervisor, self.name)
                except Exception:
                    pass
            self._stop.wait(period)

    def _control(self):
        broker = new_connection()
        q = queue_name(self.name, config.get().DOCKER_IMG, 'supervisor')
        while not self._stop.is_set():
            try:
                item = broker.pop([q], 1.0)
            except Exception:
                time.sleep(1)
                continue
            if item is None:
                continue
            _, msg = item
            try:
                fn = CONTROL_TASKS.get(msg.get('task'))
                res = fn(*msg.get('args', [])) if fn else None
                if msg.get('reply'):
                    broker.set_result(msg['reply'], res)
            finally:
                try:
                    broker.ack(msg['id'])
                except Exception:
                    pass

    def start(self):
        s = config.get()
        threads = [threading.Thread(target=self._loop, args=(self.heartbeat, min(5, s.WORKER_USAGE_INTERVAL)),
                                    daemon=True),
                   threading.Thread(target=self._loop, args=(self.stop_processes_not_exist,
                                                             self.liveness_period), daemon=True),
                   threading.Thread(target=self._control, daemon=True)]
        if s.FILE_SYNC_INTERVAL:
            from .sync import FileSync
            fs = FileSync(self.session)
            threads.append(threading.Thread(target=self._loop, args=(fs.sync, s.FILE_SYNC_INTERVAL),
                                            daemon=True))
        for t in threads:
            t.start()
        self.threads = threads
        return self

    def stop(self):
        self._stop.set()


__all__ = ['PROCESS_LOST_MESSAGE', 'WorkerPool', 'WorkerSupervisor', 'GpuInfo', 'register_computer', 'usage_snapshot']
