"""Classification report: per-image ``ReportImg`` rows (JPEG, y, y_pred, score, attrs)
for ``img_classify`` layout items, the confusion matrix (JSON bytes, group
``<item>_confusion``) and ``series`` scores (`reports/classification.py:22-152`)."""
from __future__ import annotations

import json

import numpy as np

from mlcomp_amd.db.models import ReportImg
from ._common import ReportBuilderBase, encode_jpeg, resize_saving_ratio


def confusion_matrix(y: np.ndarray, y_pred: np.ndarray, num_classes: int) -> np.ndarray:
    m = np.zeros((num_classes, num_classes), dtype=np.int64)
    np.add.at(m, (np.asarray(y, dtype=np.int64), np.asarray(y_pred, dtype=np.int64)), 1)
    return m


class ClassificationReportBuilder(ReportBuilderBase):
    def __init__(self, session, task, layout: str, part: str = 'valid', name: str = 'img_classify',
                 max_img_size=None, main_metric: str = 'accuracy', plot_count: int = 0):
        super().__init__(session, task, layout, part, name or 'img_classify', max_img_size, main_metric,
                         plot_count)

    def process_pred(self, imgs, preds: np.ndarray, targets=None, attrs=None, scores=None):
        preds = np.asarray(preds)
        for key, item in self.items('img_classify'):
            rows = []
            dag = self.dag_provider.by_id(self.task.dag)
            for i in range(len(imgs)):
                if self.plot_count <= 0:
                    break
                img = resize_saving_ratio(np.asarray(imgs[i]), self.max_img_size)
                data = encode_jpeg(img)
                attr = {k: float(v) for k, v in (attrs[i] if attrs else {}).items()}
                y = int(targets[i]) if targets is not None else None
                score = float(scores[self.main_metric][i]) if (targets is not None and scores) else None
                rows.append(ReportImg(group=key, epoch=0, task=self.task.id, img=data, dag=self.task.dag,
                                      part=self.part, project=self.project, y_pred=int(preds[i].argmax()),
                                      y=y, score=score, size=len(data), **attr))
                dag.img_size = (dag.img_size or 0) + len(data)
            if rows:
                self.session.add_all(rows, commit=False)
            if targets is not None and item.get('confusion_matrix'):
                m = confusion_matrix(targets, preds.argmax(axis=1), preds.shape[1])
                blob = json.dumps({'data': m.tolist()}).encode()
                self.session.add(ReportImg(group=f'{key}_confusion', epoch=0, task=self.task.id, img=blob,
                                           project=self.project, dag=self.task.dag, part=self.part,
                                           size=len(blob)), commit=False)
            self.session.commit()
            self.plot_count -= 1
        if targets is not None:
            self._plot_items(np.asarray(targets), preds)

    def _plot_items(self, targets, preds):
        """``f1`` (per-class precision/recall/F1 heatmap) and ``precision_recall`` items."""
        from mlcomp_amd.utils.plot import plot_classification_report, plot_precision_recall
        for kind, fn in (('f1', lambda: plot_classification_report(targets, preds.argmax(1), preds.shape[1])),
                         ('precision_recall', lambda: plot_precision_recall(targets, preds))):
            for key, item in self.items(kind):
                data = fn()
                self.session.add(ReportImg(group=key, epoch=0, task=self.task.id, img=data, dag=self.task.dag,
                                           part=self.part, project=self.project, size=len(data)), commit=False)
        self.session.commit()


__all__ = ['ClassificationReportBuilder', 'confusion_matrix']
