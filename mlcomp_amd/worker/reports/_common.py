"""Shared helpers: image encoding (PIL - OpenCV is not part of this stack), resizing
that keeps the aspect ratio, and the report/layout bootstrap."""
from __future__ import annotations

import io
from typing import Optional, Tuple

import numpy as np

from mlcomp_amd.db.models import Report, ReportTasks, now
from mlcomp_amd.db.providers import (DagProvider, ReportLayoutProvider, ReportProvider, ReportSeriesProvider,
                                     TaskProvider)
from mlcomp_amd.utils.misc import yaml_dump


def resize_saving_ratio(img: np.ndarray, max_size: Optional[Tuple[int, int]]) -> np.ndarray:
    """Shrink so that height <= max_size[0] and width <= max_size[1] (never upscales)."""
    if not max_size:
        return img
    from PIL import Image
    h, w = img.shape[:2]
    k = min(max_size[0] / h, max_size[1] / w, 1.0)
    if k >= 1.0:
        return img
    im = Image.fromarray(img)
    return np.asarray(im.resize((max(1, int(w * k)), max(1, int(h * k))), Image.BILINEAR))


def encode_jpeg(img: np.ndarray, quality: int = 90) -> bytes:
    from PIL import Image
    a = np.asarray(img)
    if a.dtype != np.uint8:
        a = np.clip(a, 0, 255).astype(np.uint8)
    if a.ndim == 3 and a.shape[2] == 1:
        a = a[..., 0]
    buf = io.BytesIO()
    Image.fromarray(a).save(buf, format='JPEG', quality=quality)
    return buf.getvalue()


def encode_png(img: np.ndarray) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(np.asarray(img).astype(np.uint8)).save(buf, format='PNG')
    return buf.getvalue()


class ReportBuilderBase:
    def __init__(self, session, task, layout: str, part: str = 'valid', name: str = None,
                 max_img_size=None, main_metric: str = 'accuracy', plot_count: int = 0):
        self.session = session
        self.task = task
        self.part = part
        self.name = name
        self.max_img_size = max_img_size
        self.main_metric = main_metric
        self.plot_count = plot_count
        self.dag_provider = DagProvider(session)
        self.report_provider = ReportProvider(session)
        self.task_provider = TaskProvider(session)
        self.series_provider = ReportSeriesProvider(session)
        self.project = self.task_provider.project(task.id).id
        layouts = ReportLayoutProvider(session).all()
        if layout not in layouts:   # the reference's examples say img_classify for img-classify
            layout = layout.replace('_', '-') if layout.replace('_', '-') in layouts else layout
        if layout not in layouts:
            raise KeyError(f'unknown layout {layout}')
        self.layout_name = layout
        self.layout_dict = layouts[layout]

    def items(self, type_: str):
        for key, item in (self.layout_dict.get('items') or {}).items():
            if item.get('type') == type_:
                yield key, item

    def create_base(self):
        r = Report(config=yaml_dump(self.layout_dict), time=now(), layout=self.layout_name,
                   project=self.project, name=self.name)
        self.report_provider.add(r)
        self.session.add(ReportTasks(report=r.id, task=self.task.id))
        self.task.report = r.id
        self.task_provider.commit()
        return r

    def process_scores(self, scores: dict, epoch: int = 0, stage: str = 'stage1'):
        from mlcomp_amd.db.models import ReportSeries
        for key, item in self.items('series'):
            k = item.get('key', key)
            if k in scores:
                self.series_provider.add(ReportSeries(name=key, value=float(scores[k]), epoch=epoch, time=now(),
                                                      task=self.task.id, part=self.part, stage=stage))
