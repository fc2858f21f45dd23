"""The scheduler ("supervisor"): one tick per second matches runnable tasks to free
CPU/GPU/memory on live computers and dispatches them through the broker.

Behaviour follows `mlcomp/server/back/supervisor.py:24-690`:
tick = create_base (live queues = docker heartbeats < 15 s) -> stop requests -> start
requests -> parent aggregation -> load tasks (NotRan sorted by GPU demand, dependency
status) -> resource ledger -> dependency gating + placement + dispatch -> auxiliary
snapshot for the UI.  Distributed tasks (``gpu_max > 1`` and ``distr``) fan out into one
Service child task per rank carrying ``distr_info`` (master addr/port, rank,
local_rank = GPU index, world size).

MI355X-first changes:
* placement is best-fit over computers (fewest free GPUs that still fit) so large
  multi-GPU jobs keep finding whole free blocks; inside a node a rank set is taken
  from one half of the 8 GPUs (one CPU socket / NUMA domain) when it fits there -
  every MI355X pair is directly xGMI-connected, so that is the only locality left;
* stop/start requests come from API threads through a thread-safe command queue
  (the reference appended to plain lists from other threads);
* the reference's quirks are fixed (`SURVEY.md` 7.6): the single-node sort uses the
  right loop variable, memory is compared in MB on both sides;
* the fatal-error auto-restart matches HIP/RCCL messages and is bounded.
"""
from __future__ import annotations

import datetime
import os
import queue as _queue
import threading
import time
import traceback
from typing import Dict, List, Optional

from mlcomp_amd.broker import get_broker, queue_name
from mlcomp_amd.db.core import Session
from mlcomp_amd.db.enums import ComponentType, TaskStatus, TaskType
from mlcomp_amd.db.models import Auxiliary, Task, now
from mlcomp_amd.db.providers import (AuxiliaryProvider, ComputerProvider, DagProvider,
                                     DockerProvider, LogProvider, TaskProvider)
from mlcomp_amd.utils.logging import create_logger
from mlcomp_amd.utils.misc import yaml_dump, yaml_load

# complete fatal-error strings of a crashed rank's last log line that make the DAG restart
# from its last checkpoint (`mlcomp/server/back/supervisor.py:400-407` lists the CUDA/cuDNN
# ones); a bare library name would also match harmless lines that merely mention it
ORPHAN_MESSAGE = 'task message lost before the task started'
FATAL_RESTART_MESSAGES = (
    'hipErrorIllegalAddress', 'an illegal memory access was encountered',
    'device-side assert triggered', 'Memory access fault by GPU', 'GPU Hang', 'HW Exception by GPU',
    'hipErrorLaunchFailure', 'ncclUnhandledCudaError', 'ncclSystemError: System call',
    'unhandled system error', 'ncclRemoteError', 'MIOPEN_STATUS_INTERNAL_ERROR',
    # the framework's own RCCL communicator: a timed-out / failed collective or rendezvous
    # (parallel/comm.py WATCHDOG_MESSAGE; torch's NCCL watchdog gives the reference the same)
    'RCCL watchdog:',
    ORPHAN_MESSAGE,
    # a rank whose process died (SIGKILL, OOM killer): worker/daemon.PROCESS_LOST_MESSAGE
    'task process was lost',
)
MAX_AUTO_RESTARTS = 3
# a DDP rank still InProgress this long after a sibling rank succeeded is taken to hang in a
# collective and is killed (its training finished with the others)
STRAGGLER_SECONDS = float(os.environ.get('MLC_STRAGGLER_SECONDS', 60))
ALIVE_SECONDS = 15
# a Queued task whose broker message is gone (broker restarted without its journal) or
# whose queue has been dead this long is taken back: its GPUs return to the ledger
ORPHAN_SECONDS = 30


class SupervisorBuilder:
    def __init__(self, session_key: str = 'SupervisorBuilder', broker=None):
        self.session_key = session_key
        self.session = Session.create_session(key=session_key)
        self.logger = create_logger(self.session, 'SupervisorBuilder', console=False)
        self.broker = broker or get_broker()
        self.commands: _queue.Queue = _queue.Queue()
        self.auxiliary: dict = {}
        self.sent_tasks = 0
        self._suspect: Dict[int, float] = {}   # Queued task id -> first tick it looked orphaned
        self._providers()

    def _providers(self):
        s = self.session
        self.provider = TaskProvider(s)
        self.computer_provider = ComputerProvider(s)
        self.docker_provider = DockerProvider(s)
        self.auxiliary_provider = AuxiliaryProvider(s)
        self.dag_provider = DagProvider(s)
        self.log_provider = LogProvider(s)

    # ------------------------------------------------------------------ commands (thread-safe)
    def stop_tasks(self, tasks: List[Task]):
        self.commands.put(('stop', [t.id if isinstance(t, Task) else int(t) for t in tasks]))

    def start_dag(self, dag_id: int):
        self.commands.put(('start', int(dag_id)))

    # ------------------------------------------------------------------ tick
    def create_base(self):
        self.session.commit()
        self.session.expire_all()
        min_time = now() - datetime.timedelta(seconds=ALIVE_SECONDS)
        self.queues = [queue_name(d.computer, d.name) for d in self.docker_provider.all()
                       if d.last_activity and d.last_activity >= min_time]
        self.auxiliary['queues'] = self.queues

    def process_commands(self):
        stop, start = [], []
        while True:
            try:
                kind, arg = self.commands.get_nowait()
            except _queue.Empty:
                break
            (stop.extend(arg) if kind == 'stop' else start.append(arg))
        if stop:
            self.process_stop_tasks(stop)
        if start:
            self.process_start_dags(start)

    def process_stop_tasks(self, ids: List[int]):
        tasks = self.provider.by_ids(ids)
        tasks += self.provider.children([t.id for t in tasks])
        not_ran = [t for t in tasks if t.status in (TaskStatus.NotRan.value, TaskStatus.Queued.value)]
        started = [t for t in tasks if t.status == TaskStatus.InProgress.value]
        for t in not_ran:
            if t.celery_id:
                self.broker.revoke(t.celery_id)
        self.provider.change_status_all([t.id for t in not_ran], TaskStatus.Skipped)
        by_queue: Dict[str, List[int]] = {}
        for t in started:
            pids = [t.pid] if t.pid else []
            pids += (yaml_load(t.additional_info) or {}).get('child_processes', [])
            if t.computer_assigned and pids:
                q = queue_name(t.computer_assigned, t.docker_assigned or 'default', 'supervisor')
                by_queue.setdefault(q, []).extend(pids)
        for q, pids in by_queue.items():
            self.broker.send_task(q, 'kill_all', pids)
        self.provider.change_status_all([t.id for t in started], TaskStatus.Stopped)

    def _find_resume(self, task: Task, children: List[Task]) -> dict:
        kids = sorted([c for c in children if c.parent == task.id], key=lambda c: -c.id)
        for c in kids:
            info = yaml_load(c.additional_info) or {}
            if info.get('distr_info', {}).get('rank') == 0:
                return {'master_computer': c.computer_assigned, 'master_task_id': c.id, 'load_last': True}
        if kids:
            c = kids[0]
            return {'master_computer': c.computer_assigned, 'master_task_id': c.id, 'load_last': True}
        return {'master_computer': task.computer_assigned, 'master_task_id': task.id, 'load_last': True}

    def process_start_dags(self, dag_ids: List[int]):
        restartable = (TaskStatus.Failed.value, TaskStatus.Skipped.value, TaskStatus.Stopped.value)
        for dag_id in dag_ids:
            tasks = self.provider.by_dag(dag_id)
            children = self.provider.children([t.id for t in tasks])
            for t in tasks:
                if t.parent:
                    t.continued = True
                    continue
                if t.status not in restartable:
                    continue
                if t.type == TaskType.Train.value:
                    info = yaml_load(t.additional_info) or {}
                    info['resume'] = self._find_resume(t, children)
                    t.additional_info = yaml_dump(info)
                t.status = TaskStatus.NotRan.value
                t.pid = t.started = t.finished = t.computer_assigned = None
                t.celery_id = t.worker_index = t.docker_assigned = t.gpu_assigned = None
        self.provider.commit()

    def _kill_stragglers(self, task: Task, counts: dict):
        """A Train parent whose ranks partly finished while the rest still run is a DDP
        hang (one rank exited, the others block in a collective): kill the rest."""
        if task.type != TaskType.Train.value:
            return
        succ, prog = counts[TaskStatus.Success], counts[TaskStatus.InProgress]
        if succ > 0 and prog > 0 and succ + prog == sum(counts.values()):
            kids = self.provider.children(task.id)
            # ranks finish a few seconds apart (checkpoint, digest, process-group teardown):
            # only a rank still running STRAGGLER_SECONDS after the first one finished hangs
            done = [c.finished for c in kids if c.status == TaskStatus.Success.value and c.finished]
            if done and (now() - min(done)).total_seconds() < STRAGGLER_SECONDS:
                return
            # mark first, kill after: the killed rank's worker sees a non-zero exit code and
            # must find the task already terminal (and flagged), or it would record a lost
            # process - a Failed rank whose log line triggers _restart_on_fatal on a DAG
            # whose training finished
            victims = [c for c in kids if c.status == TaskStatus.InProgress.value and c.pid and c.computer_assigned]
            for c in victims:
                info = yaml_load(c.additional_info) or {}
                info['killed_by_supervisor'] = True
                c.additional_info = yaml_dump(info)
                c.status = TaskStatus.Success.value
            self.provider.commit()
            for c in victims:
                q = queue_name(c.computer_assigned, c.docker_assigned or 'default', 'supervisor')
                try:
                    self.broker.call(q, 'kill', c.pid, timeout=10.0)
                except Exception:
                    pass   # the worker supervisor's liveness scan reaps it

    def _restart_on_fatal(self, task: Task):
        if task.type != TaskType.Train.value:
            return
        info = yaml_load(task.additional_info) or {}
        if info.get('auto_restarts', 0) >= MAX_AUTO_RESTARTS:
            return
        for c in sorted(self.provider.children(task.id), key=lambda x: -x.id):
            if c.status != TaskStatus.Failed.value:
                continue
            logs = self.log_provider.last(1, task=c.id)
            hit = [m for m in FATAL_RESTART_MESSAGES if logs and m in (logs[0].message or '')]
            if hit:
                info['auto_restarts'] = info.get('auto_restarts', 0) + 1
                task.additional_info = yaml_dump(info)
                self.provider.commit()
                self.logger.info(f'restart dag {task.dag} ({info["auto_restarts"]} of {MAX_AUTO_RESTARTS}): '
                                 f'task {c.id} failed with "{hit[0]}"', ComponentType.Supervisor, None, task.id)
                self.start_dag(task.dag)
                return

    def process_parent_tasks(self):
        stats = self.provider.parent_tasks_stats()
        changed = False
        for task, started, finished, counts in stats:
            self._kill_stragglers(task, counts)
            status = task.status
            for st in (TaskStatus.Failed, TaskStatus.Skipped, TaskStatus.Queued,
                       TaskStatus.InProgress, TaskStatus.Success):
                if counts[st] > 0:
                    status = st.value
                    break
            if status != task.status:
                if status == TaskStatus.InProgress.value:
                    task.started = started
                elif status >= TaskStatus.Failed.value:
                    task.started, task.finished = started, finished
                    if status != TaskStatus.Success.value:
                        self.process_stop_tasks([c.id for c in self.provider.children(task.id)
                                                 if c.status <= TaskStatus.InProgress.value])
                task.status = status
                changed = True
                if status == TaskStatus.Failed.value:
                    self.provider.commit()
                    self._restart_on_fatal(task)
        if changed:
            self.provider.commit()
        self.auxiliary['parent_tasks_stats'] = [
            {'id': t.id, 'name': t.name, 'statuses': {k.name: v for k, v in c.items()}}
            for t, _, _, c in stats[:5]]

    def load_tasks(self):
        self.tasks = self.provider.by_status(TaskStatus.NotRan, TaskStatus.InProgress, TaskStatus.Queued)
        not_ran = [t for t in self.tasks if t.status == TaskStatus.NotRan.value and not t.debug
                   and t.type != TaskType.Service.value]
        # largest GPU demand first so big DDP jobs are not starved by small ones
        self.not_ran_tasks = sorted(not_ran, key=lambda t: (-(t.gpu or 0), t.id))
        self.dep_status = self.provider.dependency_status(self.not_ran_tasks)
        self.auxiliary['not_ran_tasks'] = [
            {'id': t.id, 'name': t.name,
             'dep_status': sorted(TaskStatus(s).name for s in self.dep_status.get(t.id, ()))}
            for t in self.not_ran_tasks[:5]]

    def process_orphans(self):
        """Queued tasks nobody will run: the message is no longer in the broker (queued or
        leased - a broker restart without ``--journal``), or the target queue has had no
        heartbeat for ``ORPHAN_SECONDS``.  After ``ORPHAN_SECONDS`` of that (a worker that
        just popped the message holds a lease, so a live hand-off never looks orphaned) a
        plain task goes back to NotRan and is placed again, which also frees its GPUs in the
        ledger; a DDP rank task is failed with ``ORPHAN_MESSAGE`` - its parent fails, the
        other ranks are stopped and the bounded fatal-restart resumes the DAG."""
        t_now = time.time()
        seen = set()
        for t in self.tasks:
            if t.status != TaskStatus.Queued.value or not t.celery_id or not t.computer_assigned:
                continue
            q = queue_name(t.computer_assigned, t.docker_assigned or 'default')
            try:
                lost = not self.broker.has(t.celery_id)
            except NotImplementedError:
                lost = False
            if not lost and q in self.queues:
                continue
            seen.add(t.id)
            first = self._suspect.setdefault(t.id, t_now)
            if t_now - first < ORPHAN_SECONDS:
                continue
            self._suspect.pop(t.id, None)
            why = 'its broker message is gone' if lost else f'queue {q} is dead'
            self.broker.revoke(t.celery_id)
            if t.type == TaskType.Service.value and t.parent:
                self.logger.error(f'task {t.id}: {ORPHAN_MESSAGE} ({why})', ComponentType.Supervisor,
                                  t.computer_assigned, t.id)
                self.provider.change_status(t, TaskStatus.Failed)
                continue
            self.logger.warning(f'task {t.id} re-queued: {why}', ComponentType.Supervisor, t.computer_assigned, t.id)
            t.status = TaskStatus.NotRan.value
            t.computer_assigned = t.docker_assigned = t.celery_id = t.gpu_assigned = None
            self.provider.commit()
        for tid in list(self._suspect):
            if tid not in seen:
                del self._suspect[tid]

    def load_computers(self):
        comps = {}
        for name, c in self.computer_provider.computers().items():
            comps[name] = {**c, 'gpu': [0] * int(c.get('gpu') or 0), 'ports': set(),
                           'cpu_total': c.get('cpu') or 0, 'memory_total': c.get('memory') or 0,
                           'cpu': c.get('cpu') or 0, 'memory': c.get('memory') or 0}
        for t in self.tasks:
            if t.status not in (TaskStatus.InProgress.value, TaskStatus.Queued.value):
                continue
            c = comps.get(t.computer_assigned)
            if c is None:
                continue
            if t.type == TaskType.Service.value or not self.provider.children(t.id):
                c['cpu'] -= t.cpu or 0
                c['memory'] -= (t.memory or 0) * 1024
            if t.gpu_assigned:
                for g in str(t.gpu_assigned).split(','):
                    if g.strip() != '' and int(g) < len(c['gpu']):
                        c['gpu'][int(g)] = t.id
            info = yaml_load(t.additional_info) or {}
            di = info.get('distr_info')
            if di and di.get('rank') == 0 and di.get('master_port'):
                c['ports'].add(di['master_port'])
        self.computers = [dict(v, name=k) for k, v in comps.items()]
        self.auxiliary['computers'] = [
            {k: (sorted(v) if isinstance(v, set) else v) for k, v in c.items() if k not in ('usage', 'meta')}
            for c in self.computers]

    # ------------------------------------------------------------------ placement
    @staticmethod
    def free_gpus(c: dict) -> List[int]:
        return [i for i, g in enumerate(c['gpu']) if not g]

    def _valid_computer(self, task: Task, c: dict, single_node: bool, docker: str) -> Optional[str]:
        if not c.get('can_process_tasks', True):
            return 'this computer can not process tasks'
        if task.computer and task.computer != c['name']:
            return f'task is pinned to computer {task.computer}'
        if (task.cpu or 0) > c['cpu']:
            return f'task cpu = {task.cpu} > computer free cpu = {c["cpu"]}'
        if (task.memory or 0) * 1024 > c['memory']:
            return f'task memory = {task.memory} GB > computer free memory = {c["memory"] / 1024:.1f} GB'
        if queue_name(c['name'], docker) not in self.queues:
            return f'queue {queue_name(c["name"], docker)} is not alive'
        free = len(self.free_gpus(c))
        if task.gpu > 0 and free == 0:
            return 'task requires gpu, but there is not any free'
        if single_node and task.gpu > free:
            return f'task requires {task.gpu} gpus but there are only {free} free'
        return None

    @staticmethod
    def pick_gpus(free: List[int], n: int, total: int) -> List[int]:
        """n GPU indices from ``free``, inside one half (socket) of the node if possible."""
        half = max(1, total // 2)
        groups = [[g for g in free if g // half == h] for h in range((total + half - 1) // half)]
        fitting = [g for g in groups if len(g) >= n]
        if fitting:
            return sorted(min(fitting, key=len)[:n])  # best-fit half
        return sorted(free[:n])

    def process_task(self, task: Task, aux: dict):
        dag = self.dag_provider.by_id(task.dag)
        cfg = yaml_load(dag.config) or {}
        executor = cfg.get('executors', {}).get(task.executor, {})
        docker = dag.docker_img or 'default'
        single_node = executor.get('single_node', True)
        distr = executor.get('distr', True)
        candidates, errors = [], []
        for c in self.computers:
            err = self._valid_computer(task, c, single_node, docker)
            errors.append({'name': c['name'], 'error': err})
            if err is None:
                candidates.append(c)
        aux['computers'] = errors
        if not candidates:
            return
        want = task.gpu_max or task.gpu or 0
        if task.gpu > 0:
            # best-fit: the computer with the fewest free GPUs that still satisfies the task
            candidates.sort(key=lambda c: (len(self.free_gpus(c)), c['name']))
            if single_node:
                candidates = [c for c in candidates if len(self.free_gpus(c)) >= task.gpu][:1]
            total_free = sum(len(self.free_gpus(c)) for c in candidates)
            if task.gpu > total_free:
                aux['not_valid'] = f'task needs {task.gpu} gpus, {total_free} free'
                return
        if want > 1 and distr:
            ranks = []
            for c in candidates:
                free = self.free_gpus(c)
                take = min(len(free), want - len(ranks))
                for g in self.pick_gpus(free, take, len(c['gpu'])):
                    ranks.append((c, g))
                if len(ranks) >= want:
                    break
            self._dispatch_distributed(task, ranks, docker)
        elif want > 0:
            c = candidates[0]
            gpus = self.pick_gpus(self.free_gpus(c), min(want, len(self.free_gpus(c))), len(c['gpu']))
            task.gpu_assigned = ','.join(map(str, gpus))
            self._send(task, c, docker)
        else:
            self._send(task, candidates[0], docker)

    def _find_port(self, c: dict, docker: str) -> int:
        d = self.docker_provider.get(c['name'], docker)
        lo, hi = map(int, (d.ports if d else '29500-29510').split('-'))
        for p in range(lo, hi + 1):
            if p not in c['ports']:
                return p
        raise RuntimeError(f'all master ports of {c["name"]} are taken')

    def _dispatch_distributed(self, task: Task, ranks, docker: str):
        if not ranks:
            return
        master = ranks[0][0]
        port = self._find_port(master, docker)
        master['ports'].add(port)
        names = {c['name'] for c, _ in ranks}
        if len(names) == 1:
            task.computer_assigned = master['name']
        info = yaml_load(task.additional_info) or {}
        # every rank on a computer sees ALL of the job's GPUs there (HIP_VISIBLE_DEVICES) and
        # picks its own by local_rank: RCCL then finds its peers and connects them over
        # xGMI P2P (with one visible GPU per process it cannot, and falls back to host SHM)
        node_gpus: Dict[str, List[int]] = {}
        for c, gpu in ranks:
            node_gpus.setdefault(c['name'], []).append(gpu)
        for rank, (c, gpu) in enumerate(ranks):
            addr = '127.0.0.1' if c['name'] == master['name'] else (master.get('ip') or master['name'])
            child_info = dict(info)
            mine = node_gpus[c['name']]
            child_info['distr_info'] = {'master_addr': addr, 'rank': rank, 'local_rank': mine.index(gpu),
                                        'gpu': gpu, 'visible_gpus': ','.join(map(str, mine)),
                                        'master_port': port, 'world_size': len(ranks),
                                        'master_computer': master['name']}
            child = Task(name=task.name, computer=task.computer, executor=task.executor,
                         status=TaskStatus.NotRan.value, type=TaskType.Service.value,
                         gpu_assigned=str(gpu), gpu=1, gpu_max=1, cpu=task.cpu, memory=task.memory,
                         parent=task.id, report=task.report, dag=task.dag, debug=False,
                         continued=False, steps=task.steps, additional_info=yaml_dump(child_info))
            self.provider.add(child)
            self._send(child, c, docker)
        task.status = TaskStatus.Queued.value
        self.provider.commit()

    def _send(self, task: Task, c: dict, docker: str):
        q = queue_name(c['name'], docker)
        mid = self.broker.send_task(q, 'execute', task.id)
        task.status = TaskStatus.Queued.value
        task.computer_assigned = c['name']
        task.docker_assigned = docker
        task.celery_id = mid
        if task.gpu_assigned:
            for g in str(task.gpu_assigned).split(','):
                c['gpu'][int(g)] = task.id
        c['cpu'] -= task.cpu or 0
        c['memory'] -= (task.memory or 0) * 1024
        self.sent_tasks += 1
        self.provider.commit()
        self.logger.info(f'sent task {task.id} to {q} (gpus={task.gpu_assigned})', ComponentType.Supervisor)

    def process_tasks(self):
        self.auxiliary['process_tasks'] = []
        for task in self.not_ran_tasks:
            aux = {'id': task.id, 'name': task.name}
            self.auxiliary['process_tasks'].append(aux)
            deps = self.dep_status.get(task.id, set())
            if deps & {TaskStatus.Stopped.value, TaskStatus.Failed.value, TaskStatus.Skipped.value}:
                aux['not_valid'] = 'a dependency failed, stopped or was skipped'
                self.provider.change_status(task, TaskStatus.Skipped)
                continue
            if deps and deps != {TaskStatus.Success.value}:
                aux['not_valid'] = 'not all dependencies are finished'
                continue
            self.process_task(task, aux)
        self.auxiliary['process_tasks'] = self.auxiliary['process_tasks'][:5]

    def write_auxiliary(self):
        self.auxiliary['duration'] = (now() - self.auxiliary['time']).total_seconds()
        self.auxiliary['time'] = str(self.auxiliary['time'])
        data = yaml_dump(self.auxiliary)
        if len(data) <= 16000:
            self.auxiliary_provider.set('supervisor', data)

    def build(self):
        try:
            self.auxiliary = {'time': now()}
            self.create_base()
            self.process_commands()
            self.process_parent_tasks()
            self.load_tasks()
            self.process_orphans()
            self.load_tasks()
            self.load_computers()
            self.process_tasks()
            self.write_auxiliary()
        except Exception as e:
            if Session.sqlalchemy_error(e):
                Session.cleanup(self.session_key)
                self.session = Session.create_session(key=self.session_key)
                self.logger = create_logger(self.session, 'SupervisorBuilder', console=False)
                self._providers()
            self.logger.error(traceback.format_exc(), ComponentType.Supervisor)


class SchedulerThread(threading.Thread):
    """Runs ``builder.build`` every ``interval`` seconds; never two ticks at once."""

    def __init__(self, builder: SupervisorBuilder, interval: float = 1.0):
        super().__init__(daemon=True, name='mlcomp-scheduler')
        self.builder = builder
        self.interval = interval
        self._stop_ev = threading.Event()

    def run(self):
        while not self._stop_ev.is_set():
            t0 = time.time()
            self.builder.build()
            self._stop_ev.wait(max(0.0, self.interval - (time.time() - t0)))

    def stop(self):
        self._stop_ev.set()


_SUPERVISOR: Optional[SupervisorBuilder] = None


def register_supervisor(interval: float = 1.0) -> SupervisorBuilder:
    global _SUPERVISOR
    _SUPERVISOR = SupervisorBuilder()
    SchedulerThread(_SUPERVISOR, interval).start()
    return _SUPERVISOR


def get_supervisor() -> Optional[SupervisorBuilder]:
    return _SUPERVISOR


__all__ = ['SupervisorBuilder', 'SchedulerThread', 'register_supervisor', 'get_supervisor']
