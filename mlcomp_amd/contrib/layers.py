"""Small torch helpers (`mlcomp/contrib/torch/{layers,tensors}.py`)."""
from __future__ import annotations

import torch
import torch.nn as nn


class LambdaLayer(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x):
        return self.fn(x)


def flip(x: torch.Tensor, dim: int) -> torch.Tensor:
    """Reverse ``x`` along ``dim``."""
    return torch.flip(x, (dim,))


__all__ = ['LambdaLayer', 'flip']
