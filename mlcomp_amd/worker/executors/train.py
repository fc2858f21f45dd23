"""``type: train`` (alias ``catalyst`` so the reference's YAMLs run unchanged) - the
config-driven training executor (`mlcomp/worker/executors/catalyst_/catalyst_.py`).

* reads ``args.config`` (Catalyst-style YAML) from the task folder, merges the grid
  cell and ``params`` overrides (smart suffix merge);
* DDP: ``distr_info`` from the scheduler -> MASTER_ADDR/PORT, WORLD_SIZE, RANK,
  one visible GPU per rank (LOCAL_RANK 0), ``init_process_group('nccl')`` (RCCL);
  each rank process runs only the first remaining stage and returns
  ``{stage, stages}`` so the worker re-queues it for the next stage;
* resume: picks ``last_full.pth`` / ``best_full.pth`` of the master task (local
  folder or copied from the master computer), drops finished stages, shortens
  ``num_epochs`` and restores the weights;
* ``Memory`` table: sets ``batch_size`` to the largest recorded one that fits the
  device memory (`catalyst_.py:247-265`);
* DB callback: stage/epoch steps, batch progress + loss into the task row at most
  every 10 s, per-epoch ``report_series`` rows (part = loader) and the best score of
  the layout's metric on the (parent) task;
* ``trace``: TorchScript export of the trained model.
"""
from __future__ import annotations

import os
import socket
from copy import deepcopy
from os.path import join

import torch

from mlcomp_amd import config
from mlcomp_amd.db.models import ReportSeries, now
from mlcomp_amd.db.providers import ComputerProvider, MemoryProvider, ReportSeriesProvider
from mlcomp_amd.db.report_info import ReportLayoutInfo
from mlcomp_amd.train.callbacks import Callback, CheckpointCallback
from mlcomp_amd.train.experiment import import_experiment
from mlcomp_amd.train.runner import Runner
from mlcomp_amd.utils.misc import merge_dicts_smart, set_global_seed, yaml_dump, yaml_load
from .base import Executor


def weights_digest(model) -> str:
    """sha1 (16 hex digits) of a model's parameters in registration order, as fp32."""
    import hashlib
    h = hashlib.sha1()
    for p in model.parameters():
        h.update(p.detach().float().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:16]


class DbCallback(Callback):
    order = 200
    master_only = True

    def __init__(self, ex: 'Train'):
        self.ex = ex
        self.last = None
        self.loader_start = None

    def on_epoch_start(self, state):
        stages = self.ex.all_stages
        idx = stages.index(state.stage) if state.stage in stages else 0
        self.ex.step.start(1, name=state.stage, index=idx)
        self.ex.step.start(2, name=f'epoch {state.epoch}', index=state.epoch)

    def on_loader_start(self, state):
        self.loader_start = now()

    def on_batch_start(self, state):
        if self.last is not None and state.loader_step != state.loader_len and \
                (now() - self.last).total_seconds() < 10:
            return
        t = self.ex.parent_task()
        t.batch_index = state.loader_step
        t.batch_total = state.loader_len
        t.loader_name = state.loader_name
        dur = int((now() - self.loader_start).total_seconds())
        t.epoch_duration = dur
        if state.loader_step:
            t.epoch_time_remaining = int(dur * state.loader_len / state.loader_step) - dur
        self.ex.task_provider.commit()
        self.last = now()

    def on_epoch_end(self, state):
        self.ex.step.end(2)
        t = self.ex.parent_task()
        sp = ReportSeriesProvider(self.ex.session)
        metric = self.ex.report.metric if self.ex.report else None
        for k, v in state.epoch_metrics.items():
            part, name = '', k
            for loader in state.loaders:
                if k.startswith(loader + '_'):
                    part, name = loader, k[len(loader) + 1:]
                    break
            sp.add(ReportSeries(part=part, name=name, epoch=state.epoch, task=t.id, value=float(v),
                                time=now(), stage=state.stage), commit=False)
            if name == 'loss':
                t.loss = float(v)
        sp.commit()
        if metric is not None:
            v = state.valid_metrics.get(metric.name)
            if v is not None and metric.better(float(v), t.score):
                t.score = float(v)
        self.ex.task_provider.commit()

    def on_stage_end(self, state):
        self.ex.step.end(1)


@Executor.register
class Train(Executor):
    def __init__(self, args: dict = None, report_config=None, distr_info=None, resume=None,
                 grid_config=None, params=None, trace=None, **kwargs):
        super().__init__(**kwargs)
        self.args = dict(args or {})
        self.report = ReportLayoutInfo(report_config) if report_config else None
        self.distr_info = distr_info or {}
        self.resume = resume
        self.grid_config = grid_config or {}
        self.params = params or {}
        self.trace = trace
        self.master = True
        self._parent = None

    @classmethod
    def _from_config(cls, executor, config_, additional_info):
        ex = deepcopy(executor)
        args = ex.pop('args', {}) or {}
        params = dict(ex.get('params', {}) or {})
        params.update(additional_info.get('params', {}) or {})
        grid = {k: v for k, v in ex.items() if k not in
                ('type', 'depends', 'gpu', 'cpu', 'memory', 'distr', 'single_node', 'grid', 'env',
                 'task_type', 'computer', 'steps', 'params', 'trace', 'name')}
        return cls(args=args, report_config=additional_info.get('report_config'),
                   distr_info=additional_info.get('distr_info'), resume=additional_info.get('resume'),
                   grid_config=grid, params=params, trace=ex.get('trace'))

    def parent_task(self):
        if self.task.parent:
            if self._parent is None:
                self._parent = self.task_provider.by_id(self.task.parent)
            return self._parent
        return self.task

    # ------------------------------------------------------------------ setup
    def load_config(self) -> dict:
        path = self.args.get('config', 'catalyst.yml')
        cfg = yaml_load(file=path) if os.path.exists(path) else {}
        cfg.setdefault('args', {})
        for k, v in self.args.items():
            if k != 'config':
                cfg['args'][k] = v
        if self.grid_config:
            cfg = merge_dicts_smart(cfg, self.grid_config)
        if self.params:
            cfg = merge_dicts_smart(cfg, self.params)
        return cfg

    def set_dist_env(self):
        info = self.distr_info
        os.environ['MASTER_ADDR'] = str(info['master_addr'])
        os.environ['MASTER_PORT'] = str(info['master_port'])
        os.environ['WORLD_SIZE'] = str(info['world_size'])
        os.environ['RANK'] = str(info['rank'])
        # with distr_info.visible_gpus the rank sees its job's GPUs on this computer and
        # local_rank indexes them (`catalyst_.py:214-236` saw one GPU and used LOCAL_RANK=0)
        local = int(info.get('local_rank', 0)) if info.get('visible_gpus') is not None else 0
        os.environ['LOCAL_RANK'] = str(local)
        cuda = torch.cuda.is_available()
        if cuda:
            torch.cuda.set_device(local)
            from mlcomp_amd.parallel.comm import enable_transport_log
            enable_transport_log(os.getcwd())
        import torch.distributed as dist
        dist.init_process_group('nccl' if cuda else 'gloo', init_method='env://',
                                world_size=int(info['world_size']), rank=int(info['rank']))
        self.master = info['rank'] == 0

    def _log_transports(self, runner):
        """Which RCCL transport this rank's connections use (P2P = xGMI; SHM / NET inside
        one computer means the peers were not reachable directly)."""
        from mlcomp_amd.parallel import comm as C
        ns = runner.native_step
        cm = getattr(ns, 'comm', None) if ns is not None else None
        tr = cm.transports_now() if isinstance(cm, C.RcclComm) else C._read_transport_log()
        if not tr:
            return
        msg = 'RCCL transports of rank {}: {}'.format(self.distr_info.get('rank'),
                                                     ', '.join(f'{k} x{v}' for k, v in sorted(tr.items())))
        single = len({self.distr_info.get('master_computer')}) == 1 and self.distr_info.get('master_addr') in (
            '127.0.0.1', 'localhost')
        if single and any(not k.startswith('P2P') for k in tr):
            self.warning(msg + ' - intra-node traffic is not on xGMI P2P', db=True)
        else:
            self.info(msg, db=True)

    def fix_memory(self, experiment):
        if not torch.cuda.is_available():
            return
        total_gb = torch.cuda.get_device_properties(0).total_memory / 2 ** 30
        mp = MemoryProvider(self.session)
        model_params = experiment._config.get('model_params', {}) or {}
        for stage, v in experiment.stages_config.items():
            dp = v.setdefault('data_params', {})
            q = {'model': model_params.get('model'), 'variant': model_params.get('variant'),
                 'num_classes': model_params.get('num_classes'), 'img_size': dp.get('image_size')}
            rows = [r for r in mp.find(q) if r.memory < total_gb]
            if rows:
                dp['batch_size'] = max(rows, key=lambda r: r.memory).batch_size

    def fix_resume(self, experiment) -> int:
        """Apply the resume pointer; returns the epoch to start the first stage at."""
        r = self.resume
        if not r or not experiment.logdir:
            return 0
        fname = 'last_full.pth' if r.get('load_last') else 'best_full.pth'
        ckdir = join(experiment.logdir, 'checkpoints')
        path = join(ckdir, fname)
        s = config.get()
        if r.get('master_computer') and r['master_computer'] != (os.environ.get('MLCOMP_COMPUTER')
                                                                 or socket.gethostname()):
            from mlcomp_amd.worker.sync import copy_remote
            src = ComputerProvider(self.session).by_name(r['master_computer'])
            if src is not None:
                os.makedirs(ckdir, exist_ok=True)
                remote = join(src.root_folder or s.ROOT_FOLDER, 'tasks', str(r['master_task_id']),
                              experiment.logdir, 'checkpoints', fname)
                try:
                    copy_remote(self.session, r['master_computer'], remote, path)
                except Exception as e:
                    self.error(f'checkpoint copy failed: {e}')
        elif r.get('master_task_id') and r['master_task_id'] != self.task.id:
            path = join(s.TASK_FOLDER, str(r['master_task_id']), experiment.logdir, 'checkpoints', fname)
        other = join(os.path.dirname(path), 'best_full.pth' if fname == 'last_full.pth' else 'last_full.pth')
        from mlcomp_amd.train.callbacks import load_checkpoint
        got, ckpt = load_checkpoint(path, other)
        if ckpt is None:
            self.info(f'no readable checkpoint at {path} (or {other}): starting fresh')
            return 0
        if got != path:
            self.error(f'checkpoint {path} unreadable: resuming from {got}')
        path = got
        start = 0
        for k in list(experiment.stages_config):
            if k == ckpt['stage']:
                ep = ckpt['checkpoint_data']['epoch'] + 1
                n = int(experiment.stages_config[k].get('state_params', {}).get('num_epochs', 1))
                if ep >= n or r.get('load_best'):
                    del experiment.stages_config[k]
                else:
                    start = ep
                break
            del experiment.stages_config[k]
        self.resume_path = path
        self.info(f'resuming from {path} (stage {ckpt["stage"]}, epoch {ckpt["checkpoint_data"]["epoch"]})')
        return start

    def _engine_chosen(self, e: dict):
        """Record which engine trains a stage (and why not the native one) in the task's
        DB log and ``additional_info['engine'][stage]`` - a fallback is never silent."""
        msg = f"stage {e['stage']}: {e['engine']} engine" + (f" ({e['kind']})" if e['kind'] else '') + \
            f", {e['precision']}" + (f" - {e['reason']}" if e['reason'] else '')
        if e['reason'] and e['engine'] == 'torch' and 'requested' not in e['reason']:
            self.warning(msg, db=True)
        else:
            self.info(msg, db=True)
        info = yaml_load(self.task.additional_info) or {}
        info.setdefault('engine', {})[e['stage']] = {k: e[k] for k in ('engine', 'kind', 'precision', 'reason')}
        self.task.additional_info = yaml_dump(info)
        self.task_provider.commit()

    # ------------------------------------------------------------------ run
    def work(self):
        cfg = self.load_config()
        if self.distr_info:
            self.set_dist_env()
        set_global_seed(int(cfg['args'].get('seed', 42)))
        Experiment = import_experiment(cfg['args'].get('expdir', '.'))
        experiment = Experiment(cfg)
        self.all_stages = experiment.stages[:]
        if self.master:
            self.parent_task().steps = len(self.all_stages)
            self.task_provider.commit()
        self.resume_path = None
        start_epoch = self.fix_resume(experiment)
        self.fix_memory(experiment)
        stages = experiment.stages[:]
        if not stages:
            return {}
        if self.distr_info:
            stages = stages[:1]
            info = yaml_load(self.task.additional_info) or {}
            info['resume'] = {'master_computer': self.distr_info['master_computer'],
                              'master_task_id': self.task.id - self.distr_info['rank'],
                              'load_last': True}
            self.task.additional_info = yaml_dump(info)
            self.task_provider.commit()
        extra = {'mlcomp_db': DbCallback(self)} if self.master else {}
        rank = int(self.distr_info.get('rank', 0))
        world = int(self.distr_info.get('world_size', 1))
        device = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device('cpu')
        runner = Runner(experiment, device=device, extra_callbacks=extra, rank=rank, world_size=world)
        runner.engine_hook = self._engine_chosen
        if self.resume_path:
            # full state (weights, optimizer, LR schedule, best score), applied when the
            # first remaining stage starts
            runner.resume(self.resume_path)
        runner.run_experiment(stages, start_epoch=start_epoch)
        if self.distr_info:
            # data parallelism keeps every rank's weights identical: one digest line per rank
            # makes that checkable from the task logs
            self.info(f'rank {rank} of {world}: stage {stages[-1]} weights digest '
                      f'{weights_digest(runner.model)}', db=True)
            if torch.cuda.is_available():
                self._log_transports(runner)
        if self.master and self.trace:
            model = runner.model.eval().cpu().float()
            # one real input of the last stage (channels / size as the data has them)
            traced = torch.jit.trace(model, experiment.get_native_batch(stages[-1]).cpu().float())
            torch.jit.save(traced, self.trace)
        if self.distr_info:
            import torch.distributed as dist
            dist.destroy_process_group()
        return {'stage': stages[-1], 'stages': self.all_stages}


# YAML compatibility with the reference: ``type: catalyst``
Executor._child['Catalyst'] = Train
Executor._child['catalyst'] = Train


__all__ = ['Train', 'DbCallback', 'weights_digest']
