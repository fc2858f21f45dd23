"""Test-time augmentation: ``TtaWrap`` wraps a dataset and applies a flip / transpose to
``features``; ``inverse`` undoes it on the (image-shaped) predictions, so segmentation
masks from every TTA pass line up before averaging (`contrib/transform/tta.py:9-31`)."""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


def _apply(x, hflip, vflip, transpose):
    # x: [..., H, W]
    if hflip:
        x = x.flip(-1)
    if vflip:
        x = x.flip(-2)
    if transpose:
        x = x.transpose(-1, -2)
    return x


class TtaWrap(Dataset):
    def __init__(self, dataset: Dataset, tfms=None, hflip=False, vflip=False, transpose=False):
        self.dataset = dataset
        self.tfms = tfms
        self.hflip, self.vflip, self.transpose = hflip, vflip, transpose

    def __len__(self):
        return len(self.dataset)

    def __getitem__(self, i):
        item = dict(self.dataset[i])
        x = torch.as_tensor(item['features'])
        item['features'] = _apply(x, self.hflip, self.vflip, self.transpose)
        return item

    def inverse(self, a):
        """Undo the augmentation on predictions shaped [..., H, W] (inverse order)."""
        if not torch.is_tensor(a) or a.dim() < 3:
            return a
        if self.transpose:
            a = a.transpose(-1, -2)
        if self.vflip:
            a = a.flip(-2)
        if self.hflip:
            a = a.flip(-1)
        return a


__all__ = ['TtaWrap']
