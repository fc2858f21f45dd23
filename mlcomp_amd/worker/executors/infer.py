"""``Infer``: evaluates equation ``y`` part by part; ``save`` / ``save_final`` write the
predictions (``data/<project>/pred``), ``submit`` / ``submit_final`` a submission file
(``data/submissions``) when ``prepare_submit`` is set."""
from __future__ import annotations

import os

from mlcomp_amd import config
from .base import Executor
from .equation import Equation


class Infer(Equation):
    def save(self, preds, folder: str):
        pass

    def save_final(self, folder: str):
        pass

    def submit(self, preds):
        pass

    def submit_final(self, folder: str):
        pass

    def plot(self, preds):
        pass

    def folders(self):
        s = config.get()
        project = 'default'
        try:
            project = self.task_provider.project(self.task.id).name
        except Exception:
            pass
        pred = os.path.join(s.DATA_FOLDER, project, 'pred')
        sub = os.path.join(s.DATA_FOLDER, project, 'submissions')
        os.makedirs(pred, exist_ok=True)
        os.makedirs(sub, exist_ok=True)
        if not os.path.exists('data/submissions'):
            try:
                os.makedirs('data', exist_ok=True)
                os.symlink(sub, 'data/submissions')
            except OSError:
                pass
        return pred, sub

    def work(self):
        self.create_base()
        pred_folder, submit_folder = self.folders()
        for part in self.tqdm(self.parts(), desc='infer', interval=5):
            self.begin_part(part)
            preds = self.solve('y', part)
            self.save(preds, pred_folder)
            if self.prepare_submit:
                self.submit(preds)
            if self.layout and self.plot_count:
                self.plot(preds)
        self.save_final(pred_folder)
        if self.prepare_submit:
            self.submit_final(submit_folder)
        return {}


Executor.register(Infer)
__all__ = ['Infer']
