"""``type: click`` - run a click command from the task folder
(`mlcomp/worker/executors/click.py:10-50`): imports ``<module>.py``, injects the
executor's DB-backed ``tqdm`` into the module, overrides option defaults with the
executor kwargs and redirects stdout into the task log."""
from __future__ import annotations

import importlib.util
import os
import sys

from .base import Executor


@Executor.register
class Click(Executor):
    def __init__(self, module: str, command: str = None, **kwargs):
        super().__init__(**kwargs)
        self.module = module
        self.command = command

    def work(self):
        path = os.path.join(os.getcwd(), self.module + '.py')
        spec = importlib.util.spec_from_file_location(self.module, path)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        m.tqdm = self.tqdm
        command = getattr(m, self.command)
        for p in command.params:
            if p.name in self.kwargs:
                p.default = self.kwargs[p.name]
        argv, stdout = sys.argv, sys.stdout
        sys.argv = sys.argv[:1]
        sys.stdout = self
        try:
            command(standalone_mode=False)
        finally:
            sys.stdout, sys.argv = stdout, argv
        return {}


__all__ = ['Click']
