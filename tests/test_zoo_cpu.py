"""The classification zoo behind the reference's per-model presets
(`mlcomp/contrib/catalyst/configs/classify/*.yml`): every preset names a registered model,
the architectures defined from their papers (models/cadene.py, models/nas.py) have the
published parameter counts, and each one trains a step."""
import os

import pytest
import torch

from mlcomp_amd.models import MODELS, build_model, _populate
from mlcomp_amd.contrib.presets import load_preset, preset_names

REF_PRESETS = '/root/reference/mlcomp/contrib/catalyst/configs/classify'

# published parameter counts (torch, running statistics excluded), in millions
PARAMS = {'xception': 22.855952, 'inceptionv3': 23.834568, 'inceptionv4': 42.679816, 'bninception': 11.295240,
          'fbresnet152': 60.268520, 'cafferesnet101': 44.549160, 'nasnetamobile': 5.289978,
          'pnasnet5large': 86.057668, 'dpn68b': 12.611602}


def _count(m):
    return sum(p.numel() for p in m.parameters()) / 1e6


def test_every_preset_names_a_registered_model():
    _populate()
    import mlcomp_amd.models.zoo as zoo
    zoo._register_encoder_classifiers()
    names = preset_names()
    if os.path.isdir(REF_PRESETS):   # the reference's preset list, when it is mounted
        ref = {f[:-4] for f in os.listdir(REF_PRESETS) if f.endswith('.yml')}
        assert ref <= set(names), sorted(ref - set(names))
    for n in names:
        assert load_preset(n)['model_params']['variant'] in MODELS, n


@pytest.mark.parametrize('name', sorted(PARAMS))
def test_parameter_counts(name):
    assert _count(build_model(name, num_classes=1000)) == pytest.approx(PARAMS[name], abs=2e-6)


def test_inceptionv3_aux_head_and_polynet_count():
    assert _count(build_model('inceptionv3', num_classes=1000, aux_logits=True)) == pytest.approx(27.161264, abs=2e-6)
    # NASNet-A Large and PolyNet are not pinned to a published torch count (see models/nas.py)
    assert 88 < _count(build_model('nasnetalarge', num_classes=1000)) < 90


@pytest.mark.parametrize('name,size', [('xception', 96), ('inceptionv3', 96), ('inceptionv4', 96),
                                       ('bninception', 64), ('fbresnet152', 64), ('cafferesnet101', 64),
                                       ('nasnetamobile', 64), ('nasnetalarge', 64), ('pnasnet5large', 64),
                                       ('polynet', 96), ('dpn68b', 64)])
def test_train_step(name, size):
    torch.manual_seed(0)
    m = build_model('Pretrained', variant=name, num_classes=3)
    opt = torch.optim.SGD(m.parameters(), lr=0.01)
    x, y = torch.randn(2, 3, size, size), torch.tensor([0, 2])
    loss = torch.nn.functional.cross_entropy(m(x), y)
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
    head = [mod for mod in m.modules() if isinstance(mod, torch.nn.Linear)][-1]
    assert head.out_features == 3 and head.weight.grad.abs().sum() > 0
