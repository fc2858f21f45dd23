"""Loss functions referenced by name from ``criterion_params.criterion``
(`mlcomp/contrib/criterion/{ring,ce,triplet}.py`).

All are plain autograd modules: losses are a negligible share of step time next to
the backbone, so they stay in PyTorch (the native classifier path has its own fused
softmax-CE kernel with label smoothing, ``mlc_softmax_ce``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

_EPS = 1e-8


class LabelSmoothingCrossEntropy(nn.Module):
    """``(1-eps) * NLL + eps * mean_c(-log p_c)``."""

    def __init__(self, eps: float = 0.1, reduction: str = 'mean'):
        super().__init__()
        self.eps, self.reduction = eps, reduction

    def forward(self, logits, target):
        logp = F.log_softmax(logits.float(), dim=-1)
        smooth = -logp.mean(dim=-1)
        nll = F.nll_loss(logp, target, reduction='none')
        loss = (1 - self.eps) * nll + self.eps * smooth
        if self.reduction == 'mean':
            return loss.mean()
        if self.reduction == 'sum':
            return loss.sum()
        return loss


class RingLoss(nn.Module):
    """Cross-entropy plus a ring penalty pulling feature norms to a learned radius.

    ``type``: ``'l1'`` (symmetric smooth-L1 against the radius), ``'l2'`` (squared
    distance) or ``'auto'`` (squared distance normalised by the batch mean norm).
    The radius is initialised lazily to the first batch's mean norm.
    """

    def __init__(self, type: str = 'auto', loss_weight: float = 1.0, softmax_loss_weight: float = 1.0):
        super().__init__()
        self.radius = nn.Parameter(torch.full((1,), -1.0))
        self.kind, self.w, self.ce_w = type, loss_weight, softmax_loss_weight

    def forward(self, x, y):
        ce = F.cross_entropy(x.float(), y) * self.ce_w
        norm = x.float().norm(dim=1)
        if float(self.radius.detach()) < 0:
            with torch.no_grad():
                self.radius.fill_(float(norm.mean()))
        r = self.radius.expand_as(norm)
        if self.kind == 'l1':
            ring = (F.smooth_l1_loss(norm, r) + F.smooth_l1_loss(r, norm)) * self.w
        elif self.kind == 'auto':
            ring = ((norm - r) / norm.mean().detach().clamp(min=0.5)).pow(2).mean() * self.w
        else:
            ring = (norm - r).pow(2).mean() * self.w
        return ce + ring


def cosine_distance(emb: torch.Tensor) -> torch.Tensor:
    e = F.normalize(emb.float(), dim=1)
    return 1.0 - e @ e.t()


def triplet_mask(labels: torch.Tensor) -> torch.Tensor:
    """``mask[a, p, n]`` = 1 for distinct a, p, n with label(a)==label(p)!=label(n)."""
    same = labels[:, None] == labels[None, :]
    eye = torch.eye(len(labels), dtype=torch.bool, device=labels.device)
    pos = same & ~eye
    neg = ~same
    return (pos[:, :, None] & neg[:, None, :]).float()


def triplet_loss(embeddings, labels, margin: float = 0.3, reduction: str = 'mean'):
    """Batch-all triplet loss over cosine distances; ``mean`` averages over the
    triplets that still violate the margin."""
    d = cosine_distance(embeddings)
    loss = F.relu(d[:, :, None] - d[:, None, :] + margin) * triplet_mask(labels)
    if reduction == 'mean':
        return loss.sum() / ((loss > _EPS).sum().float() + _EPS)
    if reduction == 'none':
        return loss.sum(dim=(1, 2))
    raise ValueError(f'unknown reduction {reduction}')


class TripletLoss(nn.Module):
    def __init__(self, margin: float = 0.3, reduction: str = 'mean'):
        super().__init__()
        self.margin, self.reduction = margin, reduction

    def forward(self, embeddings, labels):
        return triplet_loss(embeddings, labels, self.margin, self.reduction)


class DiceLoss(nn.Module):
    """``1 - dice`` on sigmoid probabilities (segmentation configs)."""

    def __init__(self, eps: float = 1e-7, activation: str = 'sigmoid'):
        super().__init__()
        self.eps, self.activation = eps, activation

    def forward(self, logits, target):
        from .metrics import dice
        return 1.0 - dice(logits, target, eps=self.eps, activation=self.activation)


class BCEDiceLoss(nn.Module):
    def __init__(self, eps: float = 1e-7, bce_weight: float = 1.0, dice_weight: float = 1.0):
        super().__init__()
        self.dice = DiceLoss(eps)
        self.bw, self.dw = bce_weight, dice_weight

    def forward(self, logits, target):
        bce = F.binary_cross_entropy_with_logits(logits.float(), target.float())
        return self.bw * bce + self.dw * self.dice(logits, target)


__all__ = ['LabelSmoothingCrossEntropy', 'RingLoss', 'TripletLoss', 'triplet_loss', 'cosine_distance',
           'triplet_mask', 'DiceLoss', 'BCEDiceLoss']
