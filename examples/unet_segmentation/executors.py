"""Validation node of the U-Net DAG: runs the traced model (equation ``y``) over a
held-out synthetic set part by part, scores Dice per image and writes overlays."""
import numpy as np

from mlcomp_amd.contrib.metrics import dice_numpy
from mlcomp_amd.train.data import SyntheticSegmentation
from mlcomp_amd.worker.executors import Executor
from mlcomp_amd.worker.executors.valid import Valid
from mlcomp_amd.worker.reports import SegmentationReportBuilder


class _Part:
    def __init__(self, ds, a, b):
        self.ds, self.a, self.b = ds, a, b

    def __len__(self):
        return self.b - self.a

    def __getitem__(self, i):
        return self.ds[self.a + i]


@Executor.register
class ValidSegmentation(Valid):
    def __init__(self, **kwargs):
        super().__init__(layout='img-segment', **kwargs)
        self.src = SyntheticSegmentation(num_samples=256, image_size=256, num_classes=1, seed=99)
        self.scores = []

    def create_base(self):
        self.builder = SegmentationReportBuilder(self.session, self.task, self.layout, plot_count=self.plot_count)
        self.builder.create_base()

    def count(self):
        return len(self.src)

    def adjust_part(self, part):
        self.x = _Part(self.src, *part)

    def score(self, preds):
        res = [dice_numpy(p[0] > 0.5, self.x[i]['targets'][0].numpy() > 0.5) for i, p in enumerate(preds)]
        self.scores.extend(res)
        return np.array(res)

    def score_final(self):
        return float(np.mean(self.scores))

    def plot(self, preds, scores):
        imgs = [((self.x[i]['features'].numpy().transpose(1, 2, 0) * 60) + 100).clip(0, 255).astype(np.uint8)
                for i in range(len(preds))]
        tg = [self.x[i]['targets'].numpy() for i in range(len(preds))]
        self.builder.process_pred(imgs, preds, tg, scores={'dice': scores})
