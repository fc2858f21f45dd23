"""K-fold split helpers (`mlcomp/contrib/split/frame.py:10-68`,
`mlcomp/contrib/scripts/split.py:8-60`): stratified, stratified-by-group (every sample
of a group lands in one fold, groups stratified by one of their labels) and file
group k-fold that writes a ``fold.csv``-style frame."""
from __future__ import annotations

from collections import defaultdict
from os.path import basename, splitext
from typing import Optional, Sequence

import numpy as np


def stratified_k_fold(labels: Optional[Sequence] = None, n_splits: int = 5, seed: int = 0,
                      n: Optional[int] = None) -> np.ndarray:
    """Fold index per row; stratified on ``labels`` (plain shuffled k-fold if None)."""
    from sklearn.model_selection import KFold, StratifiedKFold
    rs = np.random.RandomState(seed)
    if labels is None:
        idx = np.arange(n)
        splitter = KFold(n_splits=n_splits, shuffle=True, random_state=rs).split(idx)
    else:
        labels = np.asarray(labels)
        idx = np.arange(len(labels))
        splitter = StratifiedKFold(n_splits=n_splits, shuffle=True, random_state=rs).split(idx, labels)
    res = np.zeros(len(idx), dtype=np.int64)
    for i, (_, val) in enumerate(splitter):
        res[val] = i
    return res


def stratified_group_k_fold(labels: Sequence, groups: Sequence, n_splits: int = 5,
                            seed: int = 0) -> np.ndarray:
    from sklearn.model_selection import StratifiedKFold
    rs = np.random.RandomState(seed)
    group_labels = defaultdict(set)
    for g, l in zip(groups, labels):
        group_labels[g].add(l)
    keys = list(group_labels)
    y = [rs.choice(sorted(group_labels[k], key=str)) for k in keys]
    gfold = {}
    for i, (_, val) in enumerate(StratifiedKFold(n_splits=n_splits, shuffle=True,
                                                 random_state=rs).split(np.arange(len(keys)), y)):
        for j in val:
            gfold[keys[j]] = i
    return np.array([gfold[g] for g in groups], dtype=np.int64)


def file_group_kfold(n_splits: int, output: str = None, get_group=None, sort: bool = False,
                     must_equal=(), seed: int = 0, **files):
    import pandas as pd
    from sklearn.model_selection import GroupKFold
    assert files, 'at least one list of files is required'
    keys = sorted(files)

    def name(f):
        return splitext(basename(f))[0]

    if sort:
        files = {k: sorted(v, key=name) for k, v in files.items()}
    first = files[keys[0]]
    assert len(first) > n_splits, f'at least {n_splits} files are required, got {len(first)}'
    for k, v in files.items():
        assert len(v) == len(first), f'count of files in {k} differs from {keys[0]}'
        if k in must_equal:
            for a, b in zip(v, first):
                assert name(a) == name(b), f'file name mismatch in {k}: {basename(a)}'
    df = pd.DataFrame({k: files[k] for k in keys})
    df['fold'] = 0
    groups = [i if get_group is None else get_group(f) for i, f in enumerate(first)]
    for i, (_, test) in enumerate(GroupKFold(n_splits).split(groups, groups=groups)):
        df.loc[test, 'fold'] = i
    df = df.sample(frac=1, random_state=seed)
    if output:
        df.to_csv(output, index=False)
    return df


__all__ = ['stratified_k_fold', 'stratified_group_k_fold', 'file_group_kfold']
