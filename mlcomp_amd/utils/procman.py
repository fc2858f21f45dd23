"""Minimal process supervisor replacing supervisord for ``mlcomp-server start`` /
``mlcomp-worker start``: runs a set of named programs, restarts any that exits
(exponential back-off capped at 30 s, reset after 60 s of healthy uptime), writes a
pid file + live status JSON into CONFIG_FOLDER, and on SIGTERM/SIGINT terminates every
program's process group (SIGTERM, then SIGKILL after a grace period).

Programs are started with ``start_new_session=True`` so each one - and every task
process it spawns - can be signalled as a group by exact pgid, never by name pattern.
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional


class Program:
    def __init__(self, name: str, argv: List[str], env: Optional[Dict[str, str]] = None,
                 autorestart: bool = True, log: Optional[str] = None):
        self.name, self.argv, self.env, self.autorestart, self.log = name, argv, env, autorestart, log
        self.proc: Optional[subprocess.Popen] = None
        self.started = 0.0
        self.restarts = 0
        self.backoff = 1.0
        self.next_start = 0.0

    def start(self):
        out = open(self.log, 'ab') if self.log else subprocess.DEVNULL
        self.proc = subprocess.Popen(self.argv, env=dict(os.environ, **(self.env or {})),
                                     stdout=out, stderr=subprocess.STDOUT, start_new_session=True)
        self.started = time.time()

    def alive(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    def signal(self, sig):
        if self.alive():
            try:
                os.killpg(self.proc.pid, sig)
            except ProcessLookupError:
                pass

    def to_dict(self):
        return {'name': self.name, 'argv': self.argv, 'pid': self.proc.pid if self.proc else None,
                'alive': self.alive(), 'restarts': self.restarts, 'started': self.started}


class ProcessManager:
    def __init__(self, programs: List[Program], state_dir: str, name: str = 'mlcomp'):
        self.programs = programs
        self.pid_file = os.path.join(state_dir, f'{name}-procman.pid')
        self.status_file = os.path.join(state_dir, f'{name}-procman.json')
        self._stop = False

    def _write_status(self):
        tmp = self.status_file + '.tmp'
        with open(tmp, 'w') as f:
            json.dump({'pid': os.getpid(), 'programs': [p.to_dict() for p in self.programs]}, f)
        os.replace(tmp, self.status_file)

    def _on_signal(self, *_):
        self._stop = True

    def run(self, poll: float = 0.5, grace: float = 10.0):
        with open(self.pid_file, 'w') as f:
            f.write(str(os.getpid()))
        signal.signal(signal.SIGTERM, self._on_signal)
        signal.signal(signal.SIGINT, self._on_signal)
        for p in self.programs:
            p.start()
        try:
            while not self._stop:
                now = time.time()
                for p in self.programs:
                    if p.alive():
                        if now - p.started > 60:
                            p.backoff = 1.0
                        continue
                    if not p.autorestart and p.proc is not None:
                        continue
                    if p.next_start == 0.0:
                        p.next_start = now + p.backoff
                        p.backoff = min(30.0, p.backoff * 2)
                    elif now >= p.next_start:
                        p.restarts += 1
                        p.next_start = 0.0
                        p.start()
                self._write_status()
                time.sleep(poll)
        finally:
            self.shutdown(grace)

    def shutdown(self, grace: float = 10.0):
        for p in self.programs:
            p.signal(signal.SIGTERM)
        deadline = time.time() + grace
        while time.time() < deadline and any(p.alive() for p in self.programs):
            time.sleep(0.1)
        for p in self.programs:
            p.signal(signal.SIGKILL)
        for f in (self.pid_file,):
            try:
                os.remove(f)
            except OSError:
                pass
        self._write_status()


def read_status(state_dir: str, name: str = 'mlcomp') -> Optional[dict]:
    path = os.path.join(state_dir, f'{name}-procman.json')
    pid_file = os.path.join(state_dir, f'{name}-procman.pid')
    if not os.path.exists(pid_file):
        return None
    try:
        pid = int(open(pid_file).read().strip())
        os.kill(pid, 0)
    except (OSError, ValueError):
        return None
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return {'pid': pid, 'programs': []}


def stop_manager(state_dir: str, name: str = 'mlcomp', timeout: float = 20.0) -> bool:
    st = read_status(state_dir, name)
    if not st:
        return False
    os.kill(st['pid'], signal.SIGTERM)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            os.kill(st['pid'], 0)
        except OSError:
            return True
        time.sleep(0.2)
    return False


def python_module(module: str, *args) -> List[str]:
    return [sys.executable, '-m', module, *map(str, args)]


__all__ = ['Program', 'ProcessManager', 'read_status', 'stop_manager', 'python_module']
