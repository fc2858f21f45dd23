"""Datasets / loaders used by config-driven training.

* ``synthetic_classification`` - ImageNet/CIFAR/MNIST-shaped random images with
  random labels; with ``on_device: true`` batches are produced directly in GPU memory
  (NHWC bf16, channel-padded for the native stem) so data loading never limits the
  step rate - the configuration of the headline ResNet-50 DAG benchmark.
* ``csv_classification`` - ``fold.csv``-style frame + image folder (contrib dataset).
* ``DistributedSamplerIndices`` - wraps any sampler for DDP: epoch-seeded shuffle,
  pad to a multiple of world size, stride by rank
  (`mlcomp/contrib/sampler/distributed.py:6-31`).
"""
from __future__ import annotations

import math
from typing import Dict, Iterator, Optional

import torch
from torch.utils.data import DataLoader, Dataset, Sampler

DATASETS: Dict[str, type] = {}


def register_dataset(name):
    def deco(cls):
        DATASETS[name] = cls
        return cls
    return deco


@register_dataset('synthetic_classification')
class SyntheticClassification(Dataset):
    def __init__(self, num_samples=1024, image_size=224, channels=3, num_classes=1000, seed=0, **_):
        self.n, self.size, self.c, self.k, self.seed = num_samples, image_size, channels, num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        x = torch.randn(self.c, self.size, self.size, generator=g)
        y = int(torch.randint(0, self.k, (1,), generator=g))
        return {'features': x, 'targets': y}


@register_dataset('synthetic_text_classification')
class SyntheticTextClassification(Dataset):
    """Random token ids (two segments) with labels; ``learnable`` makes the label a
    function of the first token so fine-tuning has signal."""

    def __init__(self, num_samples=256, seq_len=128, vocab_size=30522, num_classes=2, seed=0, learnable=True,
                 pad_fraction=0.0, **_):
        g = torch.Generator().manual_seed(seed)
        self.ids = torch.randint(1, vocab_size, (num_samples, seq_len), generator=g)
        self.y = (self.ids[:, 1] % num_classes) if learnable else torch.randint(0, num_classes, (num_samples,),
                                                                                 generator=g)
        self.tt = torch.zeros(num_samples, seq_len, dtype=torch.long)
        self.tt[:, seq_len // 2:] = 1
        self.mask = torch.ones(num_samples, seq_len, dtype=torch.long)
        if pad_fraction > 0:
            lens = torch.randint(int(seq_len * (1 - pad_fraction)), seq_len + 1, (num_samples,), generator=g)
            self.mask = (torch.arange(seq_len)[None] < lens[:, None]).long()

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        return {'input_ids': self.ids[i], 'token_type_ids': self.tt[i], 'attention_mask': self.mask[i],
                'targets': int(self.y[i])}


@register_dataset('synthetic_segmentation')
class SyntheticSegmentation(Dataset):
    """Images with 1-3 random filled discs per class; targets are the one-hot masks
    (learnable: the disc colour encodes its class)."""

    def __init__(self, num_samples=64, image_size=128, num_classes=1, seed=0, **_):
        self.n, self.size, self.k, self.seed = num_samples, image_size, num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1000003 + i)
        s = self.size
        yy, xx = torch.meshgrid(torch.arange(s), torch.arange(s), indexing='ij')
        img = torch.randn(3, s, s, generator=g) * 0.3
        mask = torch.zeros(self.k, s, s)
        for c in range(self.k):
            for _ in range(int(torch.randint(1, 4, (1,), generator=g))):
                cy, cx = torch.randint(0, s, (2,), generator=g).tolist()
                r = int(torch.randint(s // 16 + 1, s // 5 + 2, (1,), generator=g))
                disc = ((yy - cy) ** 2 + (xx - cx) ** 2) <= r * r
                mask[c][disc] = 1.0
                img[c % 3][disc] += 1.0 + 0.5 * (c // 3)
        return {'features': img, 'targets': mask}


class DeviceSyntheticLoader:
    """Fixed random batches resident on the device (NHWC bf16 when ``nhwc_pad`` is set
    for the native engine, NCHW fp32 otherwise); ``steps`` batches per epoch."""

    def __init__(self, batch_size, steps, image_size=224, channels=3, num_classes=1000,
                 device='cuda', nhwc_pad: Optional[int] = None, seed=0, **_):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        if nhwc_pad:
            img = torch.randn(batch_size, image_size, image_size, channels, device=device, generator=g)
            self.x = torch.nn.functional.pad(img, (0, nhwc_pad - channels)).to(torch.bfloat16).contiguous()
        else:
            self.x = torch.randn(batch_size, channels, image_size, image_size, device=device, generator=g)
        self.y = torch.randint(0, num_classes, (batch_size,), device=device, generator=g)
        self.steps = steps
        self.batch_size = batch_size
        self.dataset = range(batch_size * steps)

    def __len__(self):
        return self.steps

    def __iter__(self):
        for _ in range(self.steps):
            yield {'features': self.x, 'targets': self.y}


class DistributedSamplerIndices(Sampler):
    def __init__(self, sampler, num_replicas: int, rank: int, shuffle: bool = True, seed: int = 0):
        self.sampler = sampler
        self.num_replicas, self.rank, self.shuffle, self.seed = num_replicas, rank, shuffle, seed
        self.epoch = 0
        self.num_samples = int(math.ceil(len(sampler) / num_replicas))
        self.total_size = self.num_samples * num_replicas

    def __iter__(self) -> Iterator[int]:
        idx = list(self.sampler)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = [idx[i] for i in torch.randperm(len(idx), generator=g).tolist()]
        idx += idx[:self.total_size - len(idx)]
        return iter(idx[self.rank:self.total_size:self.num_replicas])

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch: int):
        self.epoch = epoch


def collate_dict(batch):
    if isinstance(batch[0], (tuple, list)):   # torchvision-style (x, y) samples
        batch = [{'features': b[0], 'targets': b[1]} for b in batch]
    out = {}
    for k in batch[0]:
        v = [b[k] for b in batch]
        if isinstance(v[0], torch.Tensor):
            out[k] = torch.stack(v)
        elif isinstance(v[0], (int, float)):
            out[k] = torch.tensor(v)
        else:
            try:
                import numpy as np
                out[k] = torch.as_tensor(np.stack(v))
            except Exception:
                out[k] = v
    return out


def make_loader(dataset, batch_size, shuffle, num_workers=0, world_size=1, rank=0, drop_last=False,
                sampler=None, pin_memory=True):
    if world_size > 1:
        base = sampler or range(len(dataset))
        sampler = DistributedSamplerIndices(base, world_size, rank, shuffle=shuffle)
        shuffle = False
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle if sampler is None else False,
                      sampler=sampler, num_workers=num_workers, collate_fn=collate_dict,
                      drop_last=drop_last, pin_memory=pin_memory and torch.cuda.is_available(),
                      persistent_workers=num_workers > 0)


__all__ = ['DATASETS', 'register_dataset', 'SyntheticClassification', 'SyntheticTextClassification',
           'SyntheticSegmentation', 'DeviceSyntheticLoader',
           'DistributedSamplerIndices', 'make_loader', 'collate_dict']
