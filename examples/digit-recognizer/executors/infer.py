"""``type: infer_mnist``: class probabilities for the test (or validation) rows, saved to
``data/pred/<model>_<suffix>.npy``; with ``prepare_submit`` also the Kaggle submission
``data/submissions/<model>_<suffix>.csv`` (``ImageId, Label``)."""
import os

import numpy as np

from mlcomp_amd.worker.executors.infer import Infer
from mlcomp_amd.worker.executors import Executor

from dataset import MnistDataset


@Executor.register
class InferMnist(Infer):
    def __init__(self, fold: int = 0, **kwargs):
        super().__init__(**kwargs)
        self.fold = int(fold)
        self.preds = []

    def create_base(self):
        if self.test:
            self.data = MnistDataset('data/test.csv')
        else:
            self.data = MnistDataset('data/train.csv', fold_csv='data/fold.csv', fold=self.fold, train=False)

    def count(self):
        return len(self.data)

    def adjust_part(self, part):
        self.x = self.data.subset(*part)

    def save(self, preds, folder):
        self.preds.append(np.asarray(preds))

    def save_final(self, folder):
        np.save(os.path.join(folder, f'{self.model_name}_{self.suffix}.npy'), np.concatenate(self.preds))

    def submit_final(self, folder):
        import pandas as pd
        labels = np.concatenate(self.preds).argmax(1)
        pd.DataFrame({'ImageId': np.arange(1, len(labels) + 1), 'Label': labels}).to_csv(
            os.path.join(folder, f'{self.model_name}_{self.suffix}.csv'), index=False)
