"""Stage / epoch / loader / batch training loop with callbacks (replacement for the
Catalyst runner the reference executes, `catalyst_.py:365-430`).

Two engines behind one loop:

* ``torch`` - any ``nn.Module``: forward under autocast(bf16) (``args.precision: bf16``,
  default) or in plain fp32 (``precision: fp32``, the reference's Catalyst default),
  criterion, backward, ``torch.optim`` step; DDP through
  ``torch.nn.parallel.DistributedDataParallel`` (backend "nccl" == RCCL on ROCm) when
  ``world_size > 1``.
* ``native`` - any model the fx lowering accepts (:mod:`mlcomp_amd.models.native_generic`:
  the reference's example nets, the classification zoo incl. grouped / depthwise convs,
  segmentation models) on the generic engine, and the hand-lowered engines for
  ResNet-family classifiers (``groups == 1``), BERT and ResNet-encoder
  U-Nets (:class:`~mlcomp_amd.train.native_seg_step.NativeSegmentationStep`) on a GPU: the whole step
  runs through :class:`~mlcomp_amd.train.native_step.NativeClassifierStep` (hand-written
  HIP kernels, flat arenas, fused optimizer, RCCL bucketer, HIP-graph replay).  Loss and
  accuracy are accumulated on the device and read once per loader, so the graph replays
  back to back without host syncs.

``engine: auto`` (default) picks native when the model/device qualify.
"""
from __future__ import annotations

import logging
import time
from collections import OrderedDict, defaultdict
from typing import Dict, List, Optional

import torch
import torch.nn as nn

from mlcomp_amd.utils import faults

from .callbacks import Callback
from .data import DeviceSyntheticLoader, make_loader
from .experiment import ConfigExperiment

_log = logging.getLogger(__name__)


class State:
    def __init__(self):
        self.stage = None
        self.epoch = 0
        self.num_epochs = 1
        self.loader_name = None
        self.is_train = True
        self.input = None
        self.output = None
        self.loss = None
        self.batch_size = 0
        self.batch_metrics: Dict[str, float] = {}
        self.loader_metrics: Dict[str, float] = {}
        self.epoch_metrics: Dict[str, float] = {}
        self.valid_metrics: Dict[str, float] = {}
        self.loaders = OrderedDict()
        self.loader_step = 0
        self.loader_len = 0
        self.main_metric = 'loss'
        self.minimize_metric = True
        self.need_early_stop = False
        self.step_count = 0
        self.native = False
        self.native_correct = None
        self.world_size = 1
        self.rank = 0
        self.logdir = None
        self.checkpoint_data = {}
        self.runner = None

    # delegated to the runner
    @property
    def model(self):
        return self.runner.model

    @property
    def optimizer(self):
        return self.runner.optimizer

    @property
    def scheduler(self):
        return self.runner.scheduler

    @property
    def criterion(self):
        return self.runner.criterion

    def make_checkpoint(self) -> dict:
        return self.runner.make_checkpoint()

    def load_checkpoint(self, ckpt: dict):
        self.runner.load_checkpoint(ckpt)

    def sync_lr(self):
        self.runner.sync_lr()

    def current_lr(self) -> float:
        return self.runner.current_lr()


def _native_kind(model: nn.Module, device: torch.device) -> Optional[str]:
    """'resnet' / 'bert' / 'unet' (U-Net, LinkNet, FPN, PSPNet, DeepLab segmentation) when the model runs on a
    native engine on this device."""
    if device.type != 'cuda':
        return None
    from mlcomp_amd.models.bert import BertForSequenceClassification
    from mlcomp_amd.models.resnet import ResNet
    if isinstance(model, ResNet) and model.groups == 1 and model.include_top:
        return 'resnet'
    if isinstance(model, BertForSequenceClassification):
        from mlcomp_amd.models.native_bert import native_bert_unsupported
        if native_bert_unsupported(model.config) is None:
            return 'bert'
        return None
    from mlcomp_amd.contrib.segmentation.deeplab import DeepLab, ResNetBackbone
    from mlcomp_amd.contrib.segmentation.models import FPN, Linknet, PSPNet, Unet
    if isinstance(model, DeepLab):     # dilated-ResNet backbone, sigmoid heads of <= 4 classes
        if isinstance(model.backbone, ResNetBackbone) and model.backbone.body.groups == 1 \
                and not model._freeze and model.decoder.body[4].out_channels <= 4:
            return 'unet'
    if isinstance(model, PSPNet):      # sigmoid heads of <= 4 classes (BCE + Dice)
        from mlcomp_amd.contrib.segmentation.encoders import ResNetEncoder
        dec = model.decoder
        if isinstance(model.encoder, ResNetEncoder) and model.encoder.body.groups == 1 \
                and dec.final_conv.out_channels <= 4 and dec.aux is None \
                and isinstance(dec.conv[1], nn.BatchNorm2d):
            return 'unet'
    if isinstance(model, FPN):         # the segmentation engine kind ('unet': BCE+Dice head)
        from mlcomp_amd.contrib.segmentation.encoders import ResNetEncoder
        if isinstance(model.encoder, ResNetEncoder) and model.encoder.body.groups == 1 \
                and model.decoder.final_conv.out_channels <= 4:
            return 'unet'
    if isinstance(model, Linknet):
        from mlcomp_amd.contrib.segmentation.encoders import ResNetEncoder
        dec = model.decoder
        if isinstance(model.encoder, ResNetEncoder) and model.encoder.body.groups == 1 \
                and dec.final_conv.out_channels <= 4 \
                and all(len(b.body) == 5 and isinstance(b.body[2], nn.BatchNorm2d) for b in dec.blocks):
            return 'unet'
    if isinstance(model, Unet):
        from mlcomp_amd.contrib.segmentation.encoders import ResNetEncoder
        dec = model.decoder
        if isinstance(model.encoder, ResNetEncoder) and model.encoder.body.groups == 1 \
                and isinstance(dec.center, nn.Identity) and dec.final_conv.out_channels <= 4 \
                and all(isinstance(b.att_in, nn.Identity) and isinstance(b.convs[0][1], nn.BatchNorm2d)
                        for b in dec.blocks):
            return 'unet'
    # everything else the fx lowering accepts runs on the generic native engine
    from mlcomp_amd.models.native_generic import lower_or_none
    return 'generic' if lower_or_none(model) is None else None


def _generic_reason(model: nn.Module) -> Optional[str]:
    from mlcomp_amd.models.bert import BertForSequenceClassification
    if isinstance(model, BertForSequenceClassification):
        from mlcomp_amd.models.native_bert import native_bert_unsupported
        return native_bert_unsupported(model.config)
    from mlcomp_amd.models.native_generic import lower_or_none
    return lower_or_none(model)


def _native_capable(model: nn.Module, device: torch.device) -> bool:
    return _native_kind(model, device) is not None


class Runner:
    def __init__(self, experiment: ConfigExperiment, device=None, extra_callbacks=None,
                 rank: int = 0, world_size: int = 1, engine: Optional[str] = None):
        self.experiment = experiment
        self.device = torch.device(device or ('cuda' if torch.cuda.is_available() else 'cpu'))
        self.extra_callbacks = extra_callbacks or OrderedDict()
        self.rank, self.world_size = rank, world_size
        self.engine = engine or experiment.args.get('engine', 'auto')
        if self.engine not in ('auto', 'native', 'torch'):
            raise ValueError(f'args.engine: auto / native / torch, not {self.engine!r}')
        # torch engine compute precision: bf16 (autocast, the default) or fp32 (the
        # reference's Catalyst default: no autocast at all); the native engines are bf16
        self.precision = str(experiment.args.get('precision', 'bf16')).lower()
        if self.precision not in ('bf16', 'fp32'):
            raise ValueError(f'args.precision: bf16 / fp32, not {self.precision!r}')
        # one entry per built stage: which engine ran it and why (see _select_engine)
        self.engine_log: List[dict] = []
        self.engine_hook = None     # callable(entry), set by the train executor
        self.model: Optional[nn.Module] = None
        self.ddp_model = None
        self.native_step = None
        self.optimizer = self.scheduler = self.criterion = None
        self.state = State()
        self.state.runner = self
        self.state.rank, self.state.world_size = rank, world_size
        self.state.logdir = experiment.logdir
        self.exception = None
        self._resume_ckpt: Optional[dict] = None   # applied at the start of the first stage
        self._native_opt_state: Optional[dict] = None  # applied when the native step is built

    # ------------------------------------------------------------------ setup
    def _select_engine(self, stage) -> dict:
        """Which engine trains ``stage`` and why: ``{'engine': 'native'|'torch', 'kind',
        'precision', 'reason'}``.  ``engine: native`` raises when the stage cannot run
        natively; ``engine: auto`` falls back to the torch engine and the reason is kept
        (``engine_log``, reported to the task by the train executor)."""
        forced = self.engine == 'native'
        kind = _native_kind(self.model, self.device)
        reason = None
        if self.engine == 'torch':
            reason = 'engine: torch requested'
        elif self.precision != 'bf16':
            reason = f'precision {self.precision}: the native engines compute in bf16 (fp32 master weights)'
        elif kind is None:
            reason = ('no HIP device: the native engines run on MI355X GPUs' if self.device.type != 'cuda' else
                      f'{type(self.model).__name__} has no native lowering: {_generic_reason(self.model)}')
        if reason is None:
            from .native_spec import NativeUnsupported, native_plan
            try:
                self._native_plan = native_plan(self.experiment, stage, kind)
            except NativeUnsupported as e:
                reason = str(e)
        if reason is None and self.device.type != 'cuda':
            reason = 'no HIP device: the native engines run on MI355X GPUs'
        if reason is not None and forced:
            raise RuntimeError(f'engine: native cannot run stage {stage!r}: {reason}')
        if reason is not None:
            return {'stage': stage, 'engine': 'torch', 'kind': None, 'precision': self.precision,
                    'reason': reason}
        return {'stage': stage, 'engine': 'native', 'kind': kind, 'precision': 'bf16', 'reason': None}

    def _build_model(self, stage):
        if self.model is None:
            self.model = self.experiment.get_model(stage)
        self._native_plan = None
        choice = self._select_engine(stage)
        use_native = choice['engine'] == 'native'
        self.native_kind = choice['kind']
        self.engine_log.append(choice)
        if choice['reason'] and self.engine == 'auto' and self.device.type == 'cuda':
            _log.warning('stage %s: %s - training on the PyTorch engine', stage, choice['reason'])
        if self.engine_hook is not None:
            self.engine_hook(choice)
        self.state.native = use_native
        if not use_native:
            self.model.to(self.device)
            if self.device.type == 'cuda':
                self.model = self.model.to(memory_format=torch.channels_last)
            if self.world_size > 1:
                from torch.nn.parallel import DistributedDataParallel as DDP
                ids = [self.device.index] if self.device.type == 'cuda' else None
                self.ddp_model = DDP(self.model, device_ids=ids)
            else:
                self.ddp_model = self.model

    def _build_native(self, stage, batch):
        plan = dict(self._native_plan or {})
        use_graph = self.experiment.args.get('graph', True)
        if self.native_kind == 'generic':
            from .native_generic_step import NativeGenericStep
            self.native_step = NativeGenericStep(
                torch_model=self.model, x=batch['features'], y=batch['targets'], device=self.device,
                world_size=self.world_size, use_graph=use_graph, criterion=self.criterion, **plan)
            self._apply_native_opt_state()
            return
        if self.native_kind == 'bert':
            from .native_bert_step import NativeBertStep
            ids = batch['input_ids']
            self.model.to(self.device)
            self.native_step = NativeBertStep(
                torch_model=self.model, batch=ids.shape[0], seq_len=ids.shape[1], device=self.device,
                world_size=self.world_size, num_labels=self.model.config.num_labels, use_graph=use_graph, **plan)
            self._apply_native_opt_state()
            return
        if self.native_kind == 'unet':
            from .native_seg_step import NativeSegmentationStep
            x = batch['features']
            size = x.shape[1] if x.dtype == torch.bfloat16 and x.shape[-1] == 8 else x.shape[-1]
            self.native_step = NativeSegmentationStep(
                torch_model=self.model, batch=x.shape[0], image_size=size, device=self.device,
                world_size=self.world_size, use_graph=use_graph, **plan)
            self._apply_native_opt_state()
            return
        from .native_step import NativeClassifierStep
        x = batch['features']
        if x.dtype == torch.bfloat16 and x.shape[-1] == 16:     # stem space-to-depth image (pad 3)
            size = 2 * x.shape[1] - 6
        elif x.dtype == torch.bfloat16 and x.shape[-1] == 8:    # NHWC, channels padded to 8
            size = x.shape[1]
        else:
            size = x.shape[-1]
        self.native_step = NativeClassifierStep(
            torch_model=self.model, batch=x.shape[0], image_size=size, device=self.device,
            world_size=self.world_size, num_classes=self.model.fc.out_features, use_graph=use_graph, **plan)
        self._apply_native_opt_state()

    def _native_sched(self, stage):
        """Native engines: a torch optimizer over one dummy tensor carries the LR and drives
        the torch LR schedulers (built with the stage, before the first batch, so a resumed
        scheduler/LR state can be loaded into it)."""
        lr = self.experiment.optimizer_spec(stage).get('lr', 0.1)
        dummy = torch.zeros(1, requires_grad=True)
        self.optimizer = torch.optim.SGD([dummy], lr=lr)
        self.scheduler = self.experiment.get_scheduler(stage, self.optimizer)

    def _apply_native_opt_state(self):
        if self._native_opt_state is not None and self.native_step is not None:
            self.native_step.opt.load_state_dict(self._native_opt_state)
            self._native_opt_state = None

    def sync_lr(self):
        if self.native_step is not None:
            self.native_step.set_lr(self.optimizer.param_groups[0]['lr'])

    def current_lr(self) -> float:
        return float(self.optimizer.param_groups[0]['lr']) if self.optimizer else 0.0

    def _loaders(self, stage) -> 'OrderedDict[str, object]':
        dp = self.experiment.stage_params(stage, 'data_params')
        bs = int(dp.get('batch_size', 32))
        if dp.get('dataset') == 'synthetic_classification' and dp.get('on_device') and self.device.type == 'cuda':
            from mlcomp_amd.models.native_resnet import STEM_CIN
            kw = {k: v for k, v in dp.items() if k not in ('dataset', 'batch_size', 'on_device', 'steps', 'seed')}
            steps = int(dp.get('steps', max(1, int(dp.get('num_samples', bs)) // (bs * self.world_size))))
            out = OrderedDict(train=DeviceSyntheticLoader(bs, steps, device=self.device,
                                                          nhwc_pad=STEM_CIN if self.native_kind == 'resnet' else None,
                                                          seed=self.rank, **kw))
            return out
        if dp.get('dataset') == 'records':
            return self._record_loaders(dp, bs)
        datasets = self.experiment.get_datasets(stage, **dp)
        out = OrderedDict()
        for name, ds in datasets.items():
            if isinstance(ds, dict):  # {'dataset': ds, 'sampler': ...}
                ds, sampler = ds['dataset'], ds.get('sampler')
            else:
                sampler = None
            out[name] = make_loader(ds, bs, shuffle=name.startswith('train'), sampler=sampler,
                                    num_workers=int(dp.get('num_workers', 0)), world_size=self.world_size,
                                    rank=self.rank, drop_last=self.state.native and name.startswith('train'))
        return out

    def _record_loaders(self, dp, bs) -> 'OrderedDict[str, object]':
        """``dataset: records``: the native input pipeline over ``path`` (train) and
        ``valid_path`` record files (:mod:`mlcomp_amd.train.records`); the native engine
        gets the stem's space-to-depth image straight from the augment kernel."""
        from .records import RecordLoader
        layout = 's2d' if self.state.native and self.native_kind == 'resnet' else 'nchw'
        common = dict(out_size=int(dp.get('image_size', 224)), rank=self.rank, world_size=self.world_size,
                      threads=int(dp.get('num_workers', 8) or 8), layout=layout, device=self.device,
                      seed=int(dp.get('seed', 0)))
        out = OrderedDict()
        out['train'] = RecordLoader(dp['path'], bs, train=True, scale=tuple(dp.get('scale', (0.08, 1.0))),
                                    **common)
        if dp.get('valid_path'):
            out['valid'] = RecordLoader(dp['valid_path'], bs, train=False, **common)
        return out

    def _callbacks(self, stage) -> List[Callback]:
        cbs = OrderedDict(self.experiment.get_callbacks(stage))
        cbs.update(self.extra_callbacks)
        out = [c for c in cbs.values() if not (c.master_only and self.rank != 0)]
        return sorted(out, key=lambda c: c.order)

    def _fire(self, event: str):
        for c in self.callbacks:
            getattr(c, event)(self.state)

    # ------------------------------------------------------------------ checkpoints
    def make_checkpoint(self) -> dict:
        if self.native_step is not None:
            self.native_step.net.export_to_torch()
        return {'stage': self.state.stage, 'epoch': self.state.epoch,
                'model_state_dict': {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                'optimizer_state_dict': self.optimizer.state_dict() if self.optimizer else None,
                'scheduler_state_dict': self.scheduler.state_dict() if self.scheduler else None,
                'native_optimizer': self.native_step.opt.state_dict() if self.native_step is not None else None,
                'checkpoint_data': dict(self.state.checkpoint_data, epoch=self.state.epoch),
                'epoch_metrics': dict(self.state.epoch_metrics),
                'valid_metrics': dict(self.state.valid_metrics)}

    def resume(self, ckpt_or_path):
        """Resume mid-stage (`catalyst_.py:341-345` hands the checkpoint to Catalyst's
        CheckpointCallback): weights, optimizer moments (torch or native arenas), LR
        scheduler position and the best score are restored when the first stage starts,
        on every rank."""
        if isinstance(ckpt_or_path, str):
            from .callbacks import load_checkpoint
            _, ckpt_or_path = load_checkpoint(ckpt_or_path)
        self._resume_ckpt = ckpt_or_path

    def load_checkpoint(self, ckpt: dict):
        """Full state restore into the built stage (model, optimizer, scheduler)."""
        self.model.load_state_dict(ckpt['model_state_dict'])
        if self.state.native:
            # the native step is (re)built from the loaded weights on the next batch; its
            # arena optimizer state is applied right after it is built
            self.native_step = None
            self._native_opt_state = ckpt.get('native_optimizer')
        if ckpt.get('optimizer_state_dict') and self.optimizer is not None:
            try:
                self.optimizer.load_state_dict(ckpt['optimizer_state_dict'])
            except (ValueError, KeyError):
                pass
        if ckpt.get('scheduler_state_dict') and self.scheduler is not None:
            self.scheduler.load_state_dict(ckpt['scheduler_state_dict'])
        from .callbacks import CheckpointCallback
        for c in getattr(self, 'callbacks', []):
            if isinstance(c, CheckpointCallback):
                c.best_score = ckpt.get('best_score')

    # ------------------------------------------------------------------ loops
    def _run_batch_torch(self, batch):
        st = self.state
        if 'input_ids' in batch:   # text classification (BERT family)
            dev = lambda k: batch[k].to(self.device, non_blocking=True) if batch.get(k) is not None else None  # noqa
            ids, y = dev('input_ids'), dev('targets')
            st.input = {'input_ids': ids, 'targets': y}
            with torch.set_grad_enabled(st.is_train), self._autocast():
                out = (self.ddp_model if st.is_train else self.model)(ids, dev('token_type_ids'),
                                                                     dev('attention_mask'))
            st.output = {'logits': out.float()}
            st.batch_size = ids.shape[0]
            return
        x = batch['features'].to(self.device, non_blocking=True)
        y = batch['targets'].to(self.device, non_blocking=True)
        if self.device.type == 'cuda' and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        st.input = {'features': x, 'targets': y}
        with torch.set_grad_enabled(st.is_train), self._autocast():
            out = (self.ddp_model if st.is_train else self.model)(x)
        st.output = {'logits': out.float() if isinstance(out, torch.Tensor) else out}
        st.batch_size = x.shape[0]

    def _autocast(self):
        """bf16 autocast on a GPU for ``precision: bf16``; a no-op context for fp32."""
        return torch.autocast(self.device.type, dtype=torch.bfloat16,
                              enabled=self.device.type == 'cuda' and self.precision == 'bf16')

    def _run_loader(self, name, loader):
        st = self.state
        st.loader_name = name
        st.is_train = name.startswith('train')
        st.loader_len = len(loader)
        if hasattr(getattr(loader, 'sampler', None), 'set_epoch'):
            loader.sampler.set_epoch(st.epoch)
        st.loader_metrics = {}
        sums, count = defaultdict(float), 0
        dev_loss = dev_correct = None
        n_samples = 0
        if self.model is not None and not st.native:
            self.model.train(st.is_train)
        self._fire('on_loader_start')
        for i, batch in enumerate(loader):
            st.loader_step = i + 1
            if st.is_train:
                self._train_batches = getattr(self, '_train_batches', 0) + 1
                faults.maybe_kill_rank(self.rank, self._train_batches)
            st.batch_metrics = {}
            st.loss = None
            st.output = None
            st.native_correct = None
            self._fire('on_batch_start')
            if st.native and st.is_train:
                if self.native_step is None:
                    self._build_native(st.stage, batch)
                    self.sync_lr()
                ns = self.native_step
                if self.native_kind == 'generic':
                    # any model / criterion: the stage's metric callbacks read the step's output
                    ns.load_batch(batch['features'], batch['targets'])
                    ns()
                    st.batch_size = ns.batch
                    st.input = {'features': ns.x, 'targets': ns.y}
                    st.output = {'logits': ns.out}
                    st.loss = ns._loss
                    self._fire('on_batch_end')
                    for k, v in st.batch_metrics.items():
                        sums[k] += v * st.batch_size
                    count += st.batch_size
                    continue
                if self.native_kind == 'unet':
                    ns.load_batch(batch['features'], batch['targets'])
                    ns()
                    st.batch_size = ns.batch
                    if dev_loss is None:
                        dev_loss = torch.zeros(2, device=self.device)
                    s4 = ns.net.head.sums()
                    dev_loss[0] += ns._loss * ns.batch
                    dev_loss[1] += (2 * s4[1] + 1e-7) / (s4[2] + s4[3] + 1e-7) * ns.batch
                    n_samples += ns.batch
                    self._fire('on_batch_end')
                    count += st.batch_size
                    continue
                if self.native_kind == 'bert':
                    ns.load_batch(batch['input_ids'], batch['targets'], batch.get('token_type_ids'),
                                  batch.get('attention_mask'))
                    head = ns.net
                else:
                    ns.load_batch(batch['features'], batch['targets'])
                    head = ns.net.head
                ns()
                st.batch_size = ns.batch
                if dev_loss is None:
                    dev_loss = torch.zeros(2, device=self.device)
                dev_loss[0] += head.loss_sum()[0]
                dev_loss[1] += head.correct()[0]
                n_samples += ns.batch
            elif st.native:
                self._run_native_eval(batch)
            else:
                self._run_batch_torch(batch)
            self._fire('on_batch_end')
            for k, v in st.batch_metrics.items():
                sums[k] += v * st.batch_size
            count += st.batch_size
        if dev_loss is not None:
            v = dev_loss.tolist()
            sums['loss'] += v[0]
            sums['dice' if self.native_kind == 'unet' else 'accuracy01'] += v[1]
            count = max(count, n_samples)
        for k, v in sums.items():
            st.loader_metrics[k] = v / max(1, count)
        self._fire('on_loader_end')
        for k, v in st.loader_metrics.items():
            st.epoch_metrics[f'{name}_{k}'] = v

    def _run_native_eval(self, batch):
        """Validation / inference batches on the native kernels too (the reference runs
        train and valid loaders through one runner, `catalyst_.py:423`): inference-mode
        BatchNorm / no dropout, no autograd, nothing routed to MIOpen or hipBLASLt."""
        st = self.state
        if self.native_step is None:       # a valid-only stage: build the engine from this batch
            self._build_native(st.stage, batch)
            self.sync_lr()
        ns = self.native_step
        y = batch['targets'].to(self.device)
        if self.native_kind == 'generic':
            x = batch['features'].to(self.device)
            out = ns.predict(x)
            st.input = {'features': x, 'targets': y}
            st.output = {'logits': out.float()}
            st.batch_size = x.shape[0]
            st.loss = self._eval_loss(st.output['logits'], y)
            return
        if self.native_kind == 'bert':
            logits = ns.predict(batch['input_ids'], batch.get('token_type_ids'), batch.get('attention_mask'))
            st.input = {'input_ids': batch['input_ids'], 'targets': y}
            st.output = {'logits': logits}
            st.batch_size = logits.shape[0]
            st.loss = self._eval_loss(logits, y)
            return
        x = batch['features'].to(self.device)
        if x.dtype != torch.bfloat16:
            from mlcomp_amd.ops import functional as Fn
            from mlcomp_amd.models.native_resnet import STEM_CIN
            x = Fn.nchw_to_nhwc(x.float(), pad_to=STEM_CIN)
        if self.native_kind == 'unet':
            logits, loss = ns.net.predict(x, y)
            st.input = {'features': x, 'targets': y}
            st.output = {'logits': logits}
            st.batch_size = x.shape[0]
            st.loss = loss
            return
        net = ns.net
        net.eval()
        with torch.no_grad():
            logits = net.logits(x).float()
        net.train()
        st.input = {'features': x, 'targets': y}
        st.output = {'logits': logits}
        st.batch_size = x.shape[0]
        st.loss = self._eval_loss(logits, y)

    def _eval_loss(self, logits, y):
        """The stage criterion on the native logits (label smoothing included)."""
        if self.criterion is not None:
            return self.criterion(logits, y)
        return torch.nn.functional.cross_entropy(logits, y)

    def run_stage(self, stage: str, start_epoch: int = 0):
        st = self.state
        st.stage = stage
        sp = self.experiment.get_state_params(stage)
        st.num_epochs = int(sp.get('num_epochs', 1))
        st.main_metric = sp.get('main_metric', 'loss')
        st.minimize_metric = bool(sp.get('minimize_metric', True))
        st.checkpoint_data = sp.get('checkpoint_data', {}) or {}
        self._build_model(stage)
        self.criterion = self.experiment.get_criterion(stage)
        if not st.native:
            self.optimizer = self.experiment.get_optimizer(stage, self.model)
            self.scheduler = self.experiment.get_scheduler(stage, self.optimizer)
        else:
            self.native_step = None
            self._native_sched(stage)
        self.loaders = self._loaders(stage)
        st.loaders = self.loaders
        self.callbacks = self._callbacks(stage)
        if self._resume_ckpt is not None:
            ck, self._resume_ckpt = self._resume_ckpt, None
            if ck.get('stage') in (None, stage):
                self.load_checkpoint(ck)
            else:   # the checkpointed stage had finished: carry the weights only
                self.model.load_state_dict(ck['model_state_dict'])
        self._fire('on_stage_start')
        for epoch in range(start_epoch, st.num_epochs):
            st.epoch = epoch
            st.epoch_metrics = {}
            self._fire('on_epoch_start')
            for name, loader in self.loaders.items():
                self._run_loader(name, loader)
                ns = self.native_step
                if ns is not None and name.startswith('train') and ns.bn_broadcast == 'eval':
                    ns.broadcast_buffers()     # every rank validates / checkpoints rank 0's BN stats
            valid = 'valid' if 'valid' in self.loaders else next(iter(self.loaders))
            st.valid_metrics = {k[len(valid) + 1:]: v for k, v in st.epoch_metrics.items()
                                if k.startswith(valid + '_')}
            self._fire('on_epoch_end')
            if st.need_early_stop:
                st.need_early_stop = False
                break
        if self.native_step is not None:
            self.native_step.net.export_to_torch()
        self._fire('on_stage_end')

    def save_config(self):
        """``logdir/configs/_config.json`` - what model tracing / model_add rebuild from."""
        if self.rank != 0 or not self.experiment.logdir:
            return
        import json
        import os
        d = os.path.join(self.experiment.logdir, 'configs')
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, '_config.json'), 'w') as f:
            json.dump(self.experiment._config, f, indent=2, default=str)

    def run_experiment(self, stages: Optional[List[str]] = None, start_epoch: int = 0):
        from mlcomp_amd.train.graphed import work_stream
        self.save_config()
        with work_stream(self.device):       # no native kernel on the NULL stream (graphed.py)
            for i, s in enumerate(stages or self.experiment.stages):
                self.run_stage(s, start_epoch if i == 0 else 0)
        return self.state


__all__ = ['Runner', 'State']
