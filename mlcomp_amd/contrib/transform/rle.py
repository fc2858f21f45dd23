"""Run-length encoding of binary masks in the Kaggle convention: column-major
(Fortran) pixel order, 1-based ``start length`` pairs (`contrib/transform/rle.py`)."""
from __future__ import annotations

import numpy as np


def mask2rle(img: np.ndarray) -> str:
    pixels = np.asarray(img).T.flatten()
    pixels = np.concatenate([[0], pixels, [0]])
    runs = np.where(pixels[1:] != pixels[:-1])[0] + 1
    runs[1::2] -= runs[::2]
    return ' '.join(str(x) for x in runs)


def rle2mask(rle: str, shape) -> np.ndarray:
    """``shape`` = (width, height) of the transposed image, as the convention stores it;
    returns an HxW uint8 mask."""
    w, h = shape[0], shape[1]
    mask = np.zeros(w * h, dtype=np.uint8)
    if isinstance(rle, str) and rle.strip():
        s = np.asarray(rle.split(), dtype=np.int64)
        starts, lengths = s[0::2] - 1, s[1::2]
        for a, n in zip(starts, lengths):
            mask[a:a + n] = 1
    return mask.reshape(w, h).T


__all__ = ['mask2rle', 'rle2mask']
