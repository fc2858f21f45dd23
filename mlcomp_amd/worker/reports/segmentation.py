"""Segmentation report: per-image overlay of the ground-truth contours and the predicted
masks (one colour per class) stacked above the image, stored as ``ReportImg`` rows with
the per-image score (`reports/segmenation.py:16-325`)."""
from __future__ import annotations

import numpy as np

from mlcomp_amd.db.models import ReportImg
from ._common import ReportBuilderBase, encode_jpeg, resize_saving_ratio

PALETTE = np.array([[230, 25, 75], [60, 180, 75], [255, 225, 25], [0, 130, 200], [245, 130, 48],
                    [145, 30, 180], [70, 240, 240], [240, 50, 230], [210, 245, 60], [250, 190, 212]],
                   dtype=np.float32)


def _contour(mask: np.ndarray) -> np.ndarray:
    m = mask.astype(bool)
    inner = m.copy()
    inner[1:, :] &= m[:-1, :]
    inner[:-1, :] &= m[1:, :]
    inner[:, 1:] &= m[:, :-1]
    inner[:, :-1] &= m[:, 1:]
    return m & ~inner


def overlay(img: np.ndarray, pred: np.ndarray, target: np.ndarray = None, alpha: float = 0.45) -> np.ndarray:
    """img HxWx3 uint8, pred/target CxHxW in {0,1}; returns (2H)xWx3: the image with the
    target contours on top, the predicted masks blended below."""
    img = np.asarray(img)
    if img.ndim == 2:
        img = np.repeat(img[..., None], 3, axis=2)
    top = img.astype(np.float32).copy()
    bottom = img.astype(np.float32).copy()
    for c in range(pred.shape[0]):
        col = PALETTE[c % len(PALETTE)]
        pm = pred[c].astype(bool)
        bottom[pm] = (1 - alpha) * bottom[pm] + alpha * col
        if target is not None:
            top[_contour(target[c])] = col
    return np.concatenate([top, bottom], axis=0).clip(0, 255).astype(np.uint8)


class SegmentationReportBuilder(ReportBuilderBase):
    def __init__(self, session, task, layout: str = 'segment', part: str = 'valid', name: str = 'img_segment',
                 max_img_size=None, main_metric: str = 'dice', plot_count: int = 0):
        super().__init__(session, task, layout, part, name or 'img_segment', max_img_size, main_metric,
                         plot_count)

    def process_pred(self, imgs, preds, targets=None, attrs=None, scores=None, threshold: float = 0.5):
        for key, item in self.items('img_segment'):
            rows = []
            dag = self.dag_provider.by_id(self.task.dag)
            for i in range(len(imgs)):
                if self.plot_count <= 0:
                    break
                p = (np.asarray(preds[i]) > threshold).astype(np.uint8)
                t = np.asarray(targets[i]).astype(np.uint8) if targets is not None else None
                vis = resize_saving_ratio(overlay(imgs[i], p, t), self.max_img_size)
                data = encode_jpeg(vis)
                attr = {k: float(v) for k, v in (attrs[i] if attrs else {}).items()}
                score = float(scores[self.main_metric][i]) if scores else None
                rows.append(ReportImg(group=key, epoch=0, task=self.task.id, img=data, dag=self.task.dag,
                                      part=self.part, project=self.project, score=score, size=len(data), **attr))
                dag.img_size = (dag.img_size or 0) + len(data)
            if rows:
                self.session.add_all(rows, commit=False)
            self.session.commit()
            self.plot_count -= 1


__all__ = ['SegmentationReportBuilder', 'overlay']
