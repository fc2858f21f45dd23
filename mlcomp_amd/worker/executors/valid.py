"""``Valid``: scores equation ``y`` against the data part by part, plots the first
``plot_count`` parts into the report, and stores the final score on the task."""
from __future__ import annotations

from .base import Executor
from .equation import Equation


class Valid(Equation):
    def score(self, preds):
        raise NotImplementedError

    def score_final(self) -> float:
        raise NotImplementedError

    def plot(self, preds, scores):
        pass

    def plot_final(self, score):
        pass

    def work(self):
        self.create_base()
        parts = self.parts()
        for i, part in enumerate(self.tqdm(parts, desc='valid', interval=5)):
            self.begin_part(part)
            preds = self.solve('y', part)
            scores = self.score(preds)
            if self.layout and self.plot_count:
                self.plot(preds, scores)
        score = float(self.score_final())
        self.plot_final(score)
        self.task.score = score
        self.task_provider.commit()
        return {'score': score}


Executor.register(Valid)
__all__ = ['Valid']
