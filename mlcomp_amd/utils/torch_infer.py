"""Inference helpers (`mlcomp/utils/torch.py:11-71`): run a traced model file over a
dataset (optionally batch-by-batch), apply an activation, undo TTA.

On the GPU the model runs under bf16 autocast with channels-last inputs (MIOpen/
hipBLASLt pick their NHWC kernels); logits come back as fp32 numpy.
"""
from __future__ import annotations

from typing import Iterator, Optional

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset


def apply_activation(x: torch.Tensor, activation: Optional[str]):
    if not activation:
        return x
    if activation == 'sigmoid':
        return torch.sigmoid(x)
    if activation == 'softmax':
        return torch.softmax(x, 1)
    raise ValueError(f'unknown activation = {activation}')


def _device():
    return torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu')


def load_model(file: str, device=None):
    dev = device or _device()
    try:
        m = torch.jit.load(file, map_location=dev)
    except RuntimeError:
        raise RuntimeError(f'{file} is not a TorchScript model (export it with trace / model_add)')
    return m.eval()


def _collate(batch):
    from mlcomp_amd.train.data import collate_dict
    return collate_dict(batch)


def _batches(model, loader, activation, dev) -> Iterator[dict]:
    from mlcomp_amd.contrib.transform.tta import TtaWrap
    use_amp = dev.type == 'cuda'
    with torch.no_grad():
        for batch in loader:
            x = batch['features'].to(dev, non_blocking=True).float()
            if x.dim() == 4 and use_amp:
                x = x.contiguous(memory_format=torch.channels_last)
            with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=use_amp):
                logits = model(x)
            p = apply_activation(logits.float(), activation)
            if isinstance(loader.dataset, TtaWrap):
                p = loader.dataset.inverse(p)
            p = p.cpu().numpy()
            yield {'prob': p, 'count': p.shape[0], **batch}


def infer(x: Dataset, file: str, batch_size: int = 1, batch_mode: bool = False, activation=None,
          num_workers: int = 0, model=None):
    dev = _device()
    loader = DataLoader(x, batch_size=batch_size, shuffle=False, num_workers=num_workers,
                        pin_memory=dev.type == 'cuda', collate_fn=_collate)
    model = model if model is not None else load_model(file, dev)
    it = _batches(model, loader, activation, dev)
    if batch_mode:
        return it
    out = [b['prob'] for b in it]
    return np.concatenate(out, axis=0) if out else np.zeros((0,))


__all__ = ['infer', 'apply_activation', 'load_model']
