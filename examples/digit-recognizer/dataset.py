"""Kaggle digit-recognizer CSVs as a dataset of {'features': [1, 28, 28] float, 'targets'}."""
import numpy as np
import torch
from torch.utils.data import Dataset


class MnistDataset(Dataset):
    def __init__(self, file: str, fold_csv: str = None, fold: int = 0, train: bool = True, max_count: int = None):
        import pandas as pd
        df = pd.read_csv(file)
        if fold_csv is not None:
            folds = pd.read_csv(fold_csv)['fold'].values
            df = df[(folds != fold) if train else (folds == fold)]
        if max_count:
            df = df.iloc[:max_count]
        self.labels = df['label'].values.astype(np.int64) if 'label' in df else np.zeros(len(df), np.int64)
        pix = df[[c for c in df.columns if c.startswith('pixel')]].values
        self.images = pix.reshape(-1, 1, 28, 28).astype(np.float32) / 255.0

    def __len__(self):
        return len(self.labels)

    def subset(self, a: int, b: int):
        s = MnistDataset.__new__(MnistDataset)
        s.labels, s.images = self.labels[a:b], self.images[a:b]
        return s

    def __getitem__(self, i):
        return {'features': torch.from_numpy(self.images[i]), 'targets': int(self.labels[i])}
