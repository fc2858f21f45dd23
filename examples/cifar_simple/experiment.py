"""Experiment for the cifar_simple example: CIFAR-10-shaped data (3x32x32, 10 classes).

There is no network access here, so the images are synthetic: each class has its own
mean colour pattern plus noise, which gives the model something to learn.  Point
``get_datasets`` at ``mlcomp_amd.contrib.dataset.ImageDataset`` to train on real files."""
from collections import OrderedDict

import torch
from torch.utils.data import Dataset

import model  # noqa: F401  (registers CifarNet)
from mlcomp_amd.train.experiment import ConfigExperiment


class SyntheticCifar(Dataset):
    def __init__(self, n: int, seed: int):
        g = torch.Generator().manual_seed(seed)
        self.y = torch.randint(0, 10, (n,), generator=g)
        protos = torch.randn(10, 3, 32, 32, generator=torch.Generator().manual_seed(1234))
        self.x = protos[self.y] + 0.8 * torch.randn(n, 3, 32, 32, generator=g)

    def __len__(self):
        return len(self.y)

    def __getitem__(self, i):
        return {'features': self.x[i], 'targets': int(self.y[i])}


class Experiment(ConfigExperiment):
    def get_datasets(self, stage: str, **data_params):
        n = int(data_params.get('num_samples', 2048))
        return OrderedDict(train=SyntheticCifar(n, 0), valid=SyntheticCifar(n // 4, 1))
