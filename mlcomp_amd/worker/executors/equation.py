"""Equation executors: inference / validation pipelines described by expressions.

The reference's examples subclass ``Valid`` / ``Infer`` (their base classes are missing
from its snapshot, `SURVEY.md` 2.6), configured like::

    infer:
      type: infer_mnist
      y: torch(x, file='net.pth', batch_size=128)
      suffix: test
      model_name: net

Every executor kwarg whose value is a string expression is an *equation*.  ``solve(name)``
evaluates it in a namespace holding ``x`` (the current part of the dataset, set by
``adjust_part``), the other equations (solved lazily; names in ``cache_names`` are kept
across parts) and the functions ``torch(x, file, batch_size, activation, tta)`` (run a
traced model from the project's model folder), ``np`` and ``mean``.  Work is processed in
parts of ``part_size`` items so arbitrarily large test sets stream through memory.
"""
from __future__ import annotations

import ast
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

from mlcomp_amd import config
from mlcomp_amd.db.providers import ModelProvider, ProjectProvider, TaskProvider
from mlcomp_amd.utils.misc import yaml_load
from .base import Executor

RESERVED = {'type', 'depends', 'gpu', 'cpu', 'memory', 'distr', 'single_node', 'grid', 'env', 'task_type',
            'computer', 'steps', 'slot', 'name', 'layout', 'plot_count', 'max_count', 'part_size', 'suffix',
            'model_id', 'model_name', 'test', 'prepare_submit', 'cache_names', 'activation', 'batch_size'}


BUILTIN_NAMES = {'x', 'torch', 'np', 'mean', 'part'}


def _names(v: str):
    try:
        tree = ast.parse(v, mode='eval')
    except SyntaxError:
        return None
    if isinstance(tree.body, ast.Constant):
        return None
    return {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)}


def find_equations(kwargs: dict) -> Dict[str, str]:
    """String kwargs that are expressions over the equation namespace: every name they
    use is a builtin (x, torch, np, mean, part) or another equation (fixpoint)."""
    cand = {}
    for k, v in kwargs.items():
        if k in RESERVED or not isinstance(v, str) or not v.strip():
            continue
        names = _names(v)
        if names is not None:
            cand[k] = names
    changed = True
    while changed:
        changed = False
        for k in list(cand):
            if not cand[k] <= BUILTIN_NAMES | set(cand):
                del cand[k]
                changed = True
    return {k: kwargs[k] for k in cand}


class Equation(Executor):
    def __init__(self, model_id: int = None, model_name: str = None, suffix: str = '', max_count: int = None,
                 part_size: int = None, cache_names=(), name: str = None, layout: str = None,
                 plot_count: int = 0, test: bool = False, prepare_submit: bool = False, **kwargs):
        self.equations: Dict[str, str] = find_equations(kwargs)
        other = {k: v for k, v in kwargs.items() if k not in self.equations}
        super().__init__(**other)
        self.model_id = model_id
        self.model_name = model_name
        self.suffix = suffix
        self.max_count = max_count
        self.part_size = part_size
        self.cache_names = list(cache_names or [])
        self.name = name or type(self).__name__.lower()
        self.layout = layout
        self.plot_count = plot_count
        self.test = test
        self.prepare_submit = prepare_submit
        self.cache: Dict[str, object] = {}
        self.part: Optional[Tuple[int, int]] = None
        self.x = None
        self._models = {}

    @classmethod
    def _from_config(cls, executor: dict, config_: dict, additional_info: dict):
        kw = {k: v for k, v in executor.items() if k not in ('type', 'depends', 'gpu', 'cpu', 'memory', 'distr',
                                                            'single_node', 'grid', 'env', 'task_type',
                                                            'computer', 'steps', 'slot')}
        return cls(**kw)

    # ------------------------------------------------------------------ hooks
    def create_base(self):
        pass

    def count(self) -> int:
        return len(self.x) if self.x is not None else 0

    def adjust_part(self, part: Tuple[int, int]):
        pass

    # ------------------------------------------------------------------ parts
    def parts(self) -> List[Tuple[int, int]]:
        n = self.count()
        if self.max_count:
            n = min(n, int(self.max_count))
        size = int(self.part_size or n or 1)
        return [(a, min(n, a + size)) for a in range(0, n, size)] or [(0, 0)]

    # ------------------------------------------------------------------ solving
    def model_folder(self) -> str:
        s = config.get()
        project = None
        if self.task is not None:
            try:
                project = TaskProvider(self.session).project(self.task.id).name
            except Exception:
                project = None
        return os.path.join(s.MODEL_FOLDER, project) if project else s.MODEL_FOLDER

    def resolve_model_file(self, file: str) -> str:
        for cand in (file, os.path.join(self.model_folder(), file), os.path.join('models', file)):
            if os.path.exists(cand):
                return cand
        raise FileNotFoundError(f'model file {file} not found (looked in {self.model_folder()})')

    def torch(self, x, file: str = None, batch_size: int = 32, activation: str = None, num_workers: int = 0,
              tta=None):
        from mlcomp_amd.utils.torch_infer import infer, load_model
        file = file or f'{self.model_name}.pth'
        path = self.resolve_model_file(file)
        if path not in self._models:
            self._models[path] = load_model(path)
        model = self._models[path]
        preds = infer(x, path, batch_size=batch_size, activation=activation, num_workers=num_workers, model=model)
        if tta:
            from mlcomp_amd.contrib.transform.tta import TtaWrap
            import torch as _t
            outs = [preds]
            for t in tta:
                w = TtaWrap(x, **t)
                p = infer(w, path, batch_size=batch_size, activation=activation, num_workers=num_workers,
                          model=model)
                outs.append(w.inverse(_t.as_tensor(p)).numpy())
            preds = np.mean(outs, axis=0)
        return preds

    def _namespace(self):
        ns = {'np': np, 'mean': lambda *a: np.mean(a, axis=0), 'x': self.x, 'torch': self.torch,
              'part': self.part}
        for k in self.equations:
            if k in self.cache:
                ns[k] = self.cache[k]
        return ns

    def solve(self, name: str, part=None):
        if name in self.cache and (name in self.cache_names or self.part == part):
            return self.cache[name]
        expr = self.equations[name]
        tree = ast.parse(expr, mode='eval')
        deps = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)} & set(self.equations)
        for d in deps - {name}:
            self.cache[d] = self.solve(d, part)
        res = eval(compile(tree, f'<equation {name}>', 'eval'), {'__builtins__': {}}, self._namespace())
        self.cache[name] = res
        return res

    def begin_part(self, part):
        self.part = part
        for k in list(self.cache):
            if k not in self.cache_names:
                del self.cache[k]
        self.adjust_part(part)


__all__ = ['Equation']
