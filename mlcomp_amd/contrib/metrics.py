"""Segmentation metrics (`mlcomp/contrib/metrics/dice.py`)."""
from __future__ import annotations

import numpy as np
import torch


def dice(outputs: torch.Tensor, targets: torch.Tensor, eps: float = 1e-7, threshold: float = None,
         activation: str = 'sigmoid') -> torch.Tensor:
    """Soft (or thresholded) Dice over the whole batch."""
    if activation == 'sigmoid':
        outputs = torch.sigmoid(outputs.float())
    elif activation == 'softmax':
        outputs = torch.softmax(outputs.float(), dim=1)
    if threshold is not None:
        outputs = (outputs > threshold).float()
    targets = targets.float()
    inter = (outputs * targets).sum()
    union = outputs.sum() + targets.sum()
    return (2 * inter + eps) / (union + eps)


def dice_numpy(pred: np.ndarray, target: np.ndarray, empty_one: bool = True, eps: float = 1e-7) -> float:
    """Per-image Dice on binary masks; two empty masks score ``1`` when ``empty_one``."""
    p = pred.astype(bool)
    t = target.astype(bool)
    s = p.sum() + t.sum()
    if s == 0:
        return 1.0 if empty_one else 0.0
    return float(2 * (p & t).sum() / (s + eps))


__all__ = ['dice', 'dice_numpy']
