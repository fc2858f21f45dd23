"""``type: split`` - stratified k-fold of a CSV into ``data/<project>/fold.csv``
(`mlcomp/worker/executors/split.py:11-44`)."""
from __future__ import annotations

import os

from mlcomp_amd import config
from .base import Executor


@Executor.register
class Split(Executor):
    def __init__(self, variant: str = 'frame', out: str = None, n_splits: int = 5, file: str = None,
                 label: str = None, group: str = None, **kwargs):
        super().__init__(**kwargs)
        self.variant, self.out, self.n_splits = variant, out, n_splits
        self.file, self.label, self.group = file, label, group

    @classmethod
    def _from_config(cls, executor, config_, additional_info):
        project = config_['info']['project']
        data = os.path.join(config.get().DATA_FOLDER, project)
        return cls(variant=executor.get('variant', 'frame'),
                   out=os.path.join(data, executor.get('out', 'fold.csv')),
                   n_splits=executor.get('n_splits', 5),
                   file=os.path.join(data, executor['file']) if executor.get('file') else None,
                   label=executor.get('label'), group=executor.get('group'))

    def work(self):
        import pandas as pd
        from mlcomp_amd.contrib.split import stratified_group_k_fold, stratified_k_fold
        df = pd.read_csv(self.file)
        if self.group:
            fold = stratified_group_k_fold(df[self.label].values, df[self.group].values, self.n_splits)
        else:
            fold = stratified_k_fold(df[self.label].values if self.label else None, self.n_splits,
                                     n=len(df))
        pd.DataFrame({'fold': fold}).to_csv(self.out, index=False)
        self.info(f'split {len(df)} rows into {self.n_splits} folds -> {self.out}')
        return {'out': self.out}


__all__ = ['Split']
