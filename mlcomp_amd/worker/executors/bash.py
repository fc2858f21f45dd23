"""``type: bash`` - run a shell command (`mlcomp/worker/executors/bash.py:7-47`).

``$key`` placeholders are substituted from the executor's kwargs (grid cells included),
``&&``-separated sub-commands run in order, stdout lines stream into the task log, and a
non-zero exit raises with the captured stderr.  stderr is drained on a thread so a
chatty process can never deadlock on a full pipe."""
from __future__ import annotations

import subprocess
import threading

from .base import Executor


@Executor.register
class Bash(Executor):
    def __init__(self, command: str, **kwargs):
        super().__init__(**kwargs)
        for k, v in sorted(kwargs.items(), key=lambda kv: -len(kv[0])):
            command = command.replace(f'${k}', str(v))
        self.command = command

    def work(self):
        for sub in [c.strip() for c in self.command.split('&&') if c.strip()]:
            self.info('executing ' + sub)
            p = subprocess.Popen('exec ' + sub, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                 shell=True)
            err = []
            t = threading.Thread(target=lambda: err.extend(l.decode(errors='replace').rstrip()
                                                           for l in p.stderr), daemon=True)
            t.start()
            try:
                self.add_child_process(p.pid)
                for line in p.stdout:
                    self.info(line.decode(errors='replace').rstrip())
                p.wait()
                t.join()
                if p.returncode != 0:
                    raise RuntimeError('\n'.join(err) or f'exit code {p.returncode}')
                for line in err:
                    self.warning(line)
            finally:
                if p.poll() is None:
                    p.kill()
        return {}


__all__ = ['Bash']
