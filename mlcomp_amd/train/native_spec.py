"""What the native engines implement of a Catalyst-style stage config, and the step
keyword arguments that express it.

The reference trains whatever ``criterion_params`` / ``optimizer_params`` /
``callbacks_params`` name through Catalyst (`mlcomp/worker/executors/catalyst_/catalyst_.py:365-430`,
e.g. `examples/digit-recognizer/catalyst.yml:23-40`).  A native engine fuses the loss and
the optimizer into its own kernels, so it can only run a stage whose loss, optimizer and
optimizer-callback options it implements exactly.  :func:`native_plan` either returns the
native step's keyword arguments for the stage or raises :class:`NativeUnsupported` naming
the option it cannot honour; the runner then raises (``engine: native``) or trains that
stage on the PyTorch path (``engine: auto``) - never a silently different objective.
"""
from __future__ import annotations

from typing import Dict


class NativeUnsupported(ValueError):
    """The stage asks for something the native engine does not implement."""


# torch.optim defaults (the reference builds torch.optim.<name>(**optimizer_params))
_SGD_DEFAULTS = dict(momentum=0.0, weight_decay=0.0, nesterov=False, dampening=0.0)
_ADAM_DEFAULTS = {'Adam': dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0),
                  'AdamW': dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01)}
_OPT_KEYS = {'SGD': {'lr', 'momentum', 'weight_decay', 'nesterov', 'dampening', 'maximize', 'foreach',
                     'differentiable', 'fused'},
             'Adam': {'lr', 'betas', 'eps', 'weight_decay', 'amsgrad', 'maximize', 'foreach', 'capturable',
                      'differentiable', 'fused'},
             'AdamW': {'lr', 'betas', 'eps', 'weight_decay', 'amsgrad', 'maximize', 'foreach', 'capturable',
                       'differentiable', 'fused'}}
# the optimizers each native engine has fused kernels for
_ENGINE_OPTS = {'resnet': ('SGD', 'Adam', 'AdamW'), 'unet': ('SGD', 'Adam', 'AdamW'),
                'bert': ('SGD', 'Adam', 'AdamW'), 'generic': ('SGD', 'Adam', 'AdamW')}
# a criterion's own flags that only select an implementation, never the objective
_NEUTRAL = {'reduction': 'mean'}


def _optimizer(spec: dict, kind: str, default_lr: float) -> Dict:
    p = dict(spec)
    name = p.pop('optimizer', 'Adam')
    lw = p.pop('layerwise_params', None)
    if lw:
        raise NativeUnsupported(f'optimizer_params.layerwise_params ({sorted(lw)}): per-layer optimizer '
                                'settings are not implemented by the native engines')
    if name not in _ENGINE_OPTS[kind]:
        raise NativeUnsupported(f'optimizer {name!r}: the native {kind} engine fuses only '
                                f'{"/".join(_ENGINE_OPTS[kind])}')
    unknown = set(p) - _OPT_KEYS[name]
    if unknown:
        raise NativeUnsupported(f'optimizer_params {sorted(unknown)} of {name} are not implemented natively')
    for flag in ('maximize', 'amsgrad', 'differentiable'):
        if p.get(flag):
            raise NativeUnsupported(f'{name}({flag}=True) is not implemented natively')
    out = {'optimizer': name, 'lr': float(p.get('lr', default_lr))}
    if name == 'SGD':
        d = dict(_SGD_DEFAULTS, **{k: p[k] for k in _SGD_DEFAULTS if k in p})
        out.update(momentum=float(d['momentum']), weight_decay=float(d['weight_decay']),
                   nesterov=bool(d['nesterov']), dampening=float(d['dampening']))
    else:
        d = dict(_ADAM_DEFAULTS[name], **{k: p[k] for k in _ADAM_DEFAULTS[name] if k in p})
        out.update(betas=tuple(float(b) for b in d['betas']), eps=float(d['eps']),
                   weight_decay=float(d['weight_decay']))
    return out


def _criterion(spec: dict, kind: str) -> Dict:
    if kind == 'generic':
        return {}      # the generic engine runs the stage's own criterion (torch ops on fp32 logits)
    p = dict(spec)
    name = p.pop('criterion', 'CrossEntropyLoss')
    for k, v in _NEUTRAL.items():
        if k in p and p.pop(k) != v:
            raise NativeUnsupported(f'{name}(reduction={spec[k]!r}): the native loss is a batch mean')
    if kind in ('resnet', 'bert'):
        if name == 'CrossEntropyLoss':
            smoothing = float(p.pop('label_smoothing', 0.0))
        elif name == 'LabelSmoothingCrossEntropy':
            smoothing = float(p.pop('eps', 0.1))
        else:
            raise NativeUnsupported(f'criterion {name!r}: the native {kind} engine computes softmax '
                                    'cross-entropy (CrossEntropyLoss / LabelSmoothingCrossEntropy)')
        if p.get('weight') is not None or p.get('ignore_index', -100) != -100:
            raise NativeUnsupported(f'{name} class weights / ignore_index are not implemented natively')
        p.pop('weight', None)
        p.pop('ignore_index', None)
        if p:
            raise NativeUnsupported(f'criterion_params {sorted(p)} of {name} are not implemented natively')
        if kind == 'bert' and smoothing:
            raise NativeUnsupported('label smoothing is not implemented by the native BERT head')
        return {'smoothing': smoothing} if kind == 'resnet' else {}
    # unet: the fused 1x1 head computes  bce_w * BCE + dice_w * (1 - dice)
    if name == 'BCEDiceLoss':
        out = {'bce_w': float(p.pop('bce_weight', 1.0)), 'dice_w': float(p.pop('dice_weight', 1.0)),
               'loss_eps': float(p.pop('eps', 1e-7))}
    elif name == 'BCEWithLogitsLoss':
        if p.get('weight') is not None or p.get('pos_weight') is not None:
            raise NativeUnsupported('BCEWithLogitsLoss weight / pos_weight are not implemented natively')
        p.pop('weight', None)
        p.pop('pos_weight', None)
        out = {'bce_w': 1.0, 'dice_w': 0.0, 'loss_eps': 1e-7}
    elif name == 'DiceLoss':
        if p.pop('activation', 'sigmoid') != 'sigmoid':
            raise NativeUnsupported('DiceLoss: the native head uses sigmoid probabilities')
        out = {'bce_w': 0.0, 'dice_w': 1.0, 'loss_eps': float(p.pop('eps', 1e-7))}
    else:
        raise NativeUnsupported(f'criterion {name!r}: the native U-Net head computes BCEDiceLoss / '
                                'BCEWithLogitsLoss / DiceLoss')
    if p:
        raise NativeUnsupported(f'criterion_params {sorted(p)} of {name} are not implemented natively')
    return out


def _callbacks(spec: dict) -> None:
    for key, c in (spec or {}).items():
        if not isinstance(c, dict) or c.get('callback') != 'OptimizerCallback':
            continue
        if c.get('grad_clip_params'):
            raise NativeUnsupported(f'callbacks_params.{key}.grad_clip_params: gradient clipping is not '
                                    'implemented by the native engines')
        if int(c.get('accumulation_steps', 1)) != 1:
            raise NativeUnsupported(f'callbacks_params.{key}.accumulation_steps: gradient accumulation is '
                                    'not implemented by the native engines')


_DEFAULT_LR = {'resnet': 0.1, 'unet': 3e-4, 'bert': 2e-5, 'generic': 1e-3}


def native_plan(experiment, stage: str, kind: str) -> Dict:
    """Keyword arguments of the native ``kind`` step for ``stage`` (optimizer name and
    hyper-parameters with torch.optim's defaults, loss options), or NativeUnsupported."""
    out = _optimizer(experiment.stage_params(stage, 'optimizer_params'), kind, _DEFAULT_LR[kind])
    out.update(_criterion(experiment.stage_params(stage, 'criterion_params'), kind))
    _callbacks(experiment.stage_params(stage, 'callbacks_params'))
    return out


__all__ = ['NativeUnsupported', 'native_plan']
