"""``type: mnist_prepare``: writes ``data/train.csv`` / ``data/test.csv`` in the Kaggle
digit-recognizer format (``label, pixel0 .. pixel783`` / ``pixel0 .. pixel783``).

The reference downloads them with the Kaggle client (``type: download``); there is no
network here, so the digits are synthetic: one 28x28 prototype per class plus noise."""
import os

import numpy as np

from mlcomp_amd.worker.executors import Executor


@Executor.register
class MnistPrepare(Executor):
    def __init__(self, train_rows: int = 2000, test_rows: int = 300, **kwargs):
        super().__init__(**kwargs)
        self.train_rows, self.test_rows = int(train_rows), int(test_rows)

    def work(self):
        import pandas as pd
        rng = np.random.default_rng(0)
        protos = rng.integers(0, 256, (10, 784))
        cols = [f'pixel{i}' for i in range(784)]

        def rows(n):
            y = rng.integers(0, 10, n)
            x = np.clip(protos[y] * 0.7 + rng.normal(0, 40, (n, 784)), 0, 255).astype(np.uint8)
            return y, pd.DataFrame(x, columns=cols)
        os.makedirs('data', exist_ok=True)
        y, df = rows(self.train_rows)
        df.insert(0, 'label', y)
        df.to_csv('data/train.csv', index=False)
        _, dt = rows(self.test_rows)
        dt.to_csv('data/test.csv', index=False)
        self.info(f'wrote {self.train_rows} train / {self.test_rows} test rows')
        return {'train': self.train_rows, 'test': self.test_rows}
