"""``mlcomp-worker`` (`mlcomp/worker/__main__.py:164-283`).

    mlcomp-worker worker N|A-B       worker slot(s) N (or A..B) in this process
    mlcomp-worker worker-supervisor  heartbeat / usage / liveness / control queue / sync
    mlcomp-worker start [--workers]  supervisor + workers under the process manager
    mlcomp-worker stop
"""
from __future__ import annotations

import signal
import threading

import click

from mlcomp_amd import config


def _indices(spec: str):
    if '-' in spec:
        a, b = spec.split('-')
        return list(range(int(a), int(b) + 1))
    return [int(spec)]


def _wait_forever(stop_fn):
    ev = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: ev.set())
    signal.signal(signal.SIGINT, lambda *_: ev.set())
    ev.wait()
    stop_fn()


@click.group()
def main():
    pass


@main.command()
@click.argument('number')
def worker(number):
    """Run worker slot(s): pop this computer's queues and run each task in a child process."""
    from mlcomp_amd.worker.daemon import WorkerPool
    pool = WorkerPool(_indices(number)).start()
    _wait_forever(pool.stop)


@main.command('worker-supervisor')
@click.option('--workers', type=int, default=None)
def worker_supervisor(workers):
    """Per-computer daemon: registration, usage, liveness, kill/remove queue, file sync."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    from mlcomp_amd.db.enums import ComponentType
    from mlcomp_amd.worker.daemon import WorkerSupervisor
    ws = WorkerSupervisor()
    ws.logger.info('worker_supervisor start', ComponentType.WorkerSupervisor)
    ws.start()
    _wait_forever(ws.stop)


@main.command()
@click.option('--daemon', type=bool, default=False)
@click.option('--workers', type=int, default=None)
def start(daemon, workers):
    """Start the worker supervisor and workers (for a computer joining a remote server)."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    from mlcomp_amd.server.__main__ import _launch, _programs
    if workers is None:
        from mlcomp_amd.worker.daemon import GpuInfo
        workers = GpuInfo().count() + 2
    _launch('worker', _programs(workers, with_site=False, with_broker=False), daemon,
            ['mlcomp_amd.worker', 'start', '--workers', str(workers)])


@main.command()
def stop():
    from mlcomp_amd.utils.procman import stop_manager
    click.echo('stopped' if stop_manager(config.get().CONFIG_FOLDER, 'worker') else 'not running')


if __name__ == '__main__':
    main()
