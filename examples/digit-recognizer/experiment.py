"""Train on every fold of data/fold.csv except fold 0, validate on fold 0."""
from collections import OrderedDict

from mlcomp_amd.train.experiment import ConfigExperiment

from dataset import MnistDataset


class Experiment(ConfigExperiment):
    def get_datasets(self, stage: str, **data_params):
        fold = int(data_params.get('fold', 0))
        n = data_params.get('max_count')
        return OrderedDict(
            train=MnistDataset('data/train.csv', fold_csv='data/fold.csv', fold=fold, train=True, max_count=n),
            valid=MnistDataset('data/train.csv', fold_csv='data/fold.csv', fold=fold, train=False, max_count=n))
