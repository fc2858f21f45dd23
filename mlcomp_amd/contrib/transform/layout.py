"""Array layout helpers for image pipelines (`contrib/transform/albumentations.py`):
``ChannelTranspose`` HWC -> CHW (or back), ``Ensure4d`` adds a channel axis to HxW masks."""
from __future__ import annotations

import numpy as np


class ChannelTranspose:
    def __init__(self, axes=(2, 0, 1)):
        self.axes = axes

    def __call__(self, image=None, mask=None, **kw):
        out = dict(kw)
        if image is not None:
            out['image'] = np.transpose(image, self.axes)
        if mask is not None:
            out['mask'] = np.transpose(mask, self.axes) if mask.ndim == 3 else mask
        return out


class Ensure4d:
    def __call__(self, image=None, mask=None, **kw):
        out = dict(kw)
        if image is not None:
            out['image'] = image[..., None] if image.ndim == 2 else image
        if mask is not None:
            out['mask'] = mask[..., None] if mask.ndim == 2 else mask
        return out


__all__ = ['ChannelTranspose', 'Ensure4d']
