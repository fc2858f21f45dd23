"""Native-engine fidelity (`mlcomp_amd/train/native_spec.py`): the native steps get the
optimizer / loss the stage config names (torch.optim defaults included), and a stage
asking for something they do not implement raises under ``engine: native`` and trains on
the PyTorch path under ``engine: auto`` - never a silently different objective."""
import pytest
import torch

from mlcomp_amd.train import runner as runner_mod
from mlcomp_amd.train.experiment import ConfigExperiment
from mlcomp_amd.train.native_spec import NativeUnsupported, native_plan
from mlcomp_amd.train.runner import Runner


def _exp(opt=None, crit=None, cbs=None, engine='auto', logdir='.'):
    st = {'data_params': {'dataset': 'synthetic_classification', 'batch_size': 8, 'num_samples': 16,
                          'image_size': 16, 'num_classes': 4},
          'state_params': {'num_epochs': 1},
          'criterion_params': crit if crit is not None else {'criterion': 'CrossEntropyLoss'},
          'optimizer_params': opt if opt is not None else {'optimizer': 'SGD', 'lr': 0.1, 'momentum': 0.9},
          'callbacks_params': cbs if cbs is not None else {'loss': {'callback': 'CriterionCallback'},
                                                           'optimizer': {'callback': 'OptimizerCallback'}},
          'stage1': {}}
    return ConfigExperiment({'model_params': {'model': 'SimpleCNN', 'num_classes': 4, 'width': 8},
                             'args': {'expdir': '.', 'logdir': str(logdir), 'engine': engine}, 'stages': st})


def test_plan_uses_torch_optimizer_defaults():
    p = native_plan(_exp(opt={'optimizer': 'SGD', 'lr': 0.2}), 'stage1', 'resnet')
    assert p == {'optimizer': 'SGD', 'lr': 0.2, 'momentum': 0.0, 'weight_decay': 0.0, 'nesterov': False,
                 'dampening': 0.0, 'smoothing': 0.0}
    p = native_plan(_exp(opt={'optimizer': 'AdamW', 'lr': 1e-3}), 'stage1', 'bert')
    assert p == {'optimizer': 'AdamW', 'lr': 1e-3, 'betas': (0.9, 0.999), 'eps': 1e-8, 'weight_decay': 0.01}
    p = native_plan(_exp(opt={'optimizer': 'Adam', 'betas': [0.8, 0.9], 'eps': 1e-6},
                         crit={'criterion': 'BCEDiceLoss'}), 'stage1', 'unet')
    assert p['betas'] == (0.8, 0.9) and p['eps'] == 1e-6 and p['weight_decay'] == 0.0
    assert p['bce_w'] == 1.0 and p['dice_w'] == 1.0


def test_plan_maps_losses():
    e = _exp(crit={'criterion': 'CrossEntropyLoss', 'label_smoothing': 0.1})
    assert native_plan(e, 'stage1', 'resnet')['smoothing'] == 0.1
    e = _exp(crit={'criterion': 'LabelSmoothingCrossEntropy', 'eps': 0.2})
    assert native_plan(e, 'stage1', 'resnet')['smoothing'] == 0.2
    e = _exp(crit={'criterion': 'BCEDiceLoss', 'bce_weight': 0.5, 'dice_weight': 2.0})
    p = native_plan(e, 'stage1', 'unet')
    assert (p['bce_w'], p['dice_w'], p['loss_eps']) == (0.5, 2.0, 1e-7)
    p = native_plan(_exp(crit={'criterion': 'BCEWithLogitsLoss'}), 'stage1', 'unet')
    assert (p['bce_w'], p['dice_w']) == (1.0, 0.0)
    p = native_plan(_exp(crit={'criterion': 'DiceLoss'}), 'stage1', 'unet')
    assert (p['bce_w'], p['dice_w']) == (0.0, 1.0)


@pytest.mark.parametrize('kw, kind, needle', [
    ({'opt': {'optimizer': 'RMSprop', 'lr': 0.01}}, 'resnet', 'RMSprop'),
    ({'opt': {'optimizer': 'Adam', 'amsgrad': True}}, 'resnet', 'amsgrad'),
    ({'opt': {'optimizer': 'SGD', 'foo': 1}}, 'unet', 'foo'),
    ({'opt': {'optimizer': 'SGD', 'layerwise_params': {'fc': {'lr': 1}}}}, 'resnet', 'layerwise'),
    ({'crit': {'criterion': 'FocalLoss'}}, 'resnet', 'FocalLoss'),
    ({'crit': {'criterion': 'CrossEntropyLoss', 'weight': [1, 2]}}, 'resnet', 'weights'),
    ({'crit': {'criterion': 'CrossEntropyLoss', 'reduction': 'sum'}}, 'resnet', 'reduction'),
    ({'crit': {'criterion': 'CrossEntropyLoss', 'label_smoothing': 0.1}}, 'bert', 'smoothing'),
    ({'crit': {'criterion': 'CrossEntropyLoss'}}, 'unet', 'CrossEntropyLoss'),
    ({'cbs': {'o': {'callback': 'OptimizerCallback', 'grad_clip_params': {'max_norm': 1.0}}}}, 'resnet',
     'clipping'),
    ({'cbs': {'o': {'callback': 'OptimizerCallback', 'accumulation_steps': 4}}}, 'bert', 'accumulation'),
])
def test_plan_rejects_what_native_cannot_do(kw, kind, needle):
    if kind == 'unet' and 'crit' not in kw:
        kw = dict(kw, crit={'criterion': 'BCEDiceLoss'})
    with pytest.raises(NativeUnsupported, match=needle):
        native_plan(_exp(**kw), 'stage1', kind)


def test_runner_native_raises_auto_falls_back(tmp_path, monkeypatch):
    """With a model the native engine would take: RMSprop under engine: native raises;
    under engine: auto the stage trains (on the torch path) with RMSprop."""
    monkeypatch.setattr(runner_mod, '_native_kind', lambda model, device: 'resnet')
    opt = {'optimizer': 'RMSprop', 'lr': 0.01}
    r = Runner(_exp(opt=opt, engine='native', logdir=tmp_path), device='cpu')
    with pytest.raises(RuntimeError, match='RMSprop'):
        r.run_experiment()
    r = Runner(_exp(opt=opt, engine='auto', logdir=tmp_path), device='cpu')
    st = r.run_experiment()
    assert not st.native and isinstance(r.optimizer, torch.optim.RMSprop)
    assert 'train_loss' in st.epoch_metrics
