"""Samplers (`mlcomp/contrib/sampler/{balanced,distributed,hard_negative}.py`).

* ``BalanceClassSampler`` - per-class down/up-sampling to a common count
  (``'downsampling'`` = smallest class, ``'upsampling'`` = largest, or an int, or an
  explicit ``count_per_class``), reshuffled every epoch.
* ``DistributedSamplerIndices`` - DDP wrapper around any sampler (``train.data``).
* ``HardNegativeSampler`` (+ Pair / Triple / Four) - yields ``count`` indices per epoch in
  batches; after every batch of its loader it records the per-sample loss and the next
  batch re-draws the samples whose loss lies in the ``hard_interval`` percentile band,
  filling the rest at random.  It is also a training callback (add it to the runner's
  callbacks) so it sees each batch's loss.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, Iterator, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import Sampler

from mlcomp_amd.train.callbacks import Callback
from mlcomp_amd.train.data import DistributedSamplerIndices  # noqa: F401  (re-export)


class BalanceClassSampler(Sampler):
    def __init__(self, labels: List[int], mode: Union[str, int] = 'downsampling', max_count: int = None,
                 count_per_class: Dict[int, int] = None, seed: int = 0):
        labels = np.asarray(labels)
        self.lbl2idx = {int(l): np.where(labels == l)[0] for l in sorted(set(labels.tolist()))}
        sizes = {l: len(i) for l, i in self.lbl2idx.items()}
        if isinstance(mode, int):
            n = mode
        elif mode == 'upsampling':
            n = max(sizes.values())
        else:
            n = min(sizes.values())
        if max_count is not None:
            n = min(n, max_count)
        self.count_per_class = count_per_class or {l: n for l in self.lbl2idx}
        self.length = sum(self.count_per_class.values())
        self.rng = np.random.RandomState(seed)

    def __iter__(self) -> Iterator[int]:
        out = []
        for l, n in self.count_per_class.items():
            idx = self.lbl2idx[l]
            out.append(self.rng.choice(idx, n, replace=n > len(idx)))
        out = np.concatenate(out) if out else np.zeros(0, np.int64)
        self.rng.shuffle(out)
        return iter(out.tolist())

    def __len__(self) -> int:
        return self.length


class HardNegativeSampler(Sampler, Callback):
    order = 25   # after the criterion, before the optimizer's zero_grad of the next batch

    def __init__(self, data_source, name: str, count: int, batch_size: int = None,
                 hard_interval: Tuple[float, float] = (50, 100), index_count: int = 1,
                 criterion_data: dict = None, seed: int = 0):
        self.data_source = data_source
        self.name = name
        self.count = count
        self.batch_size = batch_size or count
        self.hard_interval = hard_interval
        self.index_count = index_count
        self.criterion_data = criterion_data
        self.max_index = len(data_source)
        self.loss = np.zeros(0)
        self.indices: List[np.ndarray] = []
        self.sampled = 0
        self.rng = np.random.RandomState(seed)

    def __len__(self):
        return self.count

    def random(self, count: int = None) -> List[np.ndarray]:
        count = self.batch_size if count is None else count
        return [self.rng.choice(self.max_index, count, replace=count > self.max_index)
                for _ in range(self.index_count)]

    def sample_batch(self):
        if len(self.loss):
            lo, hi = np.percentile(self.loss, self.hard_interval[0]), np.percentile(self.loss, self.hard_interval[1])
            hard = np.where((self.loss >= lo) & (self.loss <= hi))[0]
            picked = [np.asarray(idx)[hard] for idx in self.indices]
        else:
            picked = [np.zeros(0, np.int64) for _ in range(self.index_count)]
        rand = self.random(self.batch_size - len(picked[0]))
        perm = self.rng.permutation(self.batch_size)
        out = [np.concatenate([p, r])[perm].astype(np.int64) for p, r in zip(picked, rand)]
        return out[0] if len(out) == 1 else list(zip(*out))

    def __iter__(self):
        while self.sampled < self.count:
            batch = self.sample_batch()
            self.sampled += self.batch_size
            yield from (b.item() if hasattr(b, 'item') else b for b in batch)
        self.sampled = 0

    # ------------------------------------------------------------------ callback side
    def per_sample_loss(self, state, criterion=None, meta: dict = None) -> np.ndarray:
        criterion = criterion if criterion is not None else state.criterion
        if isinstance(criterion, dict):
            total = 0
            for k, c in criterion.items():
                total = total + self.per_sample_loss(state, c, self.criterion_data[k])
            return total
        out_key = 'logits' if meta is None else meta['output_key']
        in_key = 'targets' if meta is None else meta['input_key']
        logits, target = state.output[out_key], state.input[in_key]
        if isinstance(criterion, torch.nn.CrossEntropyLoss):
            loss = F.cross_entropy(logits.float(), target, reduction='none').detach().cpu().numpy()
        else:
            loss = np.array([float(criterion(logits[i:i + 1], target[i:i + 1])) for i in range(len(target))])
        return loss * (1 if meta is None else meta.get('weight', 1))

    def on_batch_end(self, state):
        if state.loader_name != self.name or state.output is None:
            return
        self.loss = self.per_sample_loss(state)
        self.indices = [state.input[k].detach().cpu().numpy() for k in sorted(state.input) if 'index_' in k]
        if not self.indices and 'index' in state.input:
            self.indices = [state.input['index'].detach().cpu().numpy()]


class HardNegativePairSampler(HardNegativeSampler):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, index_count=2, **kwargs)


class HardNegativeTripleSampler(HardNegativeSampler):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, index_count=3, **kwargs)


class HardNegativeFourSampler(HardNegativeSampler):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, index_count=4, **kwargs)


__all__ = ['BalanceClassSampler', 'DistributedSamplerIndices', 'HardNegativeSampler', 'HardNegativePairSampler',
           'HardNegativeTripleSampler', 'HardNegativeFourSampler']
