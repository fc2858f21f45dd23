"""Per-model data presets for classification configs (the reference's
`contrib/catalyst/configs/classify/*.yml`): ``model_params.variant`` plus
``data_params`` (batch size, input size, normalisation).  Batch sizes are per GPU and
sized for a 288 GB MI355X instead of the reference's 11-16 GB cards; merge one into a
config with ``merge_dicts_smart`` or ``load_preset(name)``."""
from __future__ import annotations

import os

import yaml

FOLDER = os.path.join(os.path.dirname(__file__), 'classify')


def preset_names():
    return sorted(f[:-4] for f in os.listdir(FOLDER) if f.endswith('.yml'))


def load_preset(name: str) -> dict:
    path = os.path.join(FOLDER, f'{name}.yml')
    if not os.path.exists(path):
        raise KeyError(f'no preset {name}; available: {preset_names()}')
    with open(path) as f:
        return yaml.safe_load(f)


__all__ = ['load_preset', 'preset_names']
