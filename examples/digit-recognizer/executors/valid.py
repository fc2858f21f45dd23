"""``type: valid_mnist``: accuracy of the traced model on the validation fold."""
import numpy as np

from mlcomp_amd.worker.executors.valid import Valid
from mlcomp_amd.worker.executors import Executor

from dataset import MnistDataset


@Executor.register
class ValidMnist(Valid):
    def __init__(self, fold: int = 0, **kwargs):
        super().__init__(**kwargs)
        self.fold = int(fold)
        self.correct = []

    def create_base(self):
        self.data = MnistDataset('data/train.csv', fold_csv='data/fold.csv', fold=self.fold, train=False)

    def count(self):
        return len(self.data)

    def adjust_part(self, part):
        self.x = self.data.subset(*part)

    def score(self, preds):
        ok = (np.asarray(preds).argmax(1) == self.x.labels).astype(np.float64)
        self.correct.extend(ok)
        return ok

    def score_final(self):
        return float(np.mean(self.correct)) if self.correct else 0.0
