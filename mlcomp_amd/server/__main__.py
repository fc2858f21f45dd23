"""``mlcomp-server`` (`mlcomp/server/__main__.py:16-145`).

    mlcomp-server start-site          REST API + UI + scheduler thread (foreground)
    mlcomp-server stop-site           ask the running site to shut down
    mlcomp-server start [--workers N] [--daemon]
                                      broker + site + worker-supervisor + worker pool
                                      under the built-in process manager
    mlcomp-server stop                stop everything ``start`` launched
    mlcomp-server status              what is running
"""
from __future__ import annotations

import os
import subprocess
import sys
import time

import click

from mlcomp_amd import config


@click.group()
def main():
    pass


@main.command('start-site')
@click.option('--host', default=None)
@click.option('--port', type=int, default=None)
def start_site(host, port):
    """Start only the site (API + UI + scheduler)."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    from mlcomp_amd.server.api import start_server
    start_server(host, port)


@main.command('stop-site')
def stop_site():
    from mlcomp_amd.server.api import stop_server
    stop_server()


def _programs(workers: int, with_site: bool = True, with_broker: bool = True):
    from mlcomp_amd.build import build_broker
    from mlcomp_amd.utils.procman import Program, python_module
    s = config.get()
    log = lambda n: os.path.join(s.LOG_FOLDER, f'{n}.out')  # noqa: E731
    progs = []
    if with_broker:
        # the journal keeps dispatched-but-unfinished task messages across broker restarts
        os.makedirs(s.DB_FOLDER, exist_ok=True)
        progs.append(Program('broker', [build_broker(), '--port', str(s.BROKER_PORT), '--journal',
                                        os.path.join(s.DB_FOLDER, 'broker.journal')], log=log('broker')))
    if with_site:
        progs.append(Program('site', python_module('mlcomp_amd.server', 'start-site'), log=log('site')))
    progs.append(Program('supervisor', python_module('mlcomp_amd.worker', 'worker-supervisor', '--workers', workers),
                         log=log('worker-supervisor')))
    if workers > 0:
        progs.append(Program('workers', python_module('mlcomp_amd.worker', 'worker', f'0-{workers - 1}'),
                             log=log('workers')))
    return progs


def _launch(name: str, progs, daemon: bool, relaunch_args):
    """Run the process manager here, or (``daemon``) re-launch this command detached.
    The CLI process never initialises a GPU, so spawning a child is safe."""
    from mlcomp_amd.utils.procman import ProcessManager, read_status
    s = config.get()
    if read_status(s.CONFIG_FOLDER, name):
        raise click.ClickException(f'{name} is already running (mlcomp-server status)')
    if daemon:
        subprocess.Popen([sys.executable, '-m', *relaunch_args], start_new_session=True,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for _ in range(100):
            if read_status(s.CONFIG_FOLDER, name):
                click.echo(f'{name} started in the background')
                return
            time.sleep(0.2)
        raise click.ClickException('background start did not come up')
    ProcessManager(progs, s.CONFIG_FOLDER, name).run()


@main.command()
@click.option('--daemon', type=bool, default=False, help='detach and return')
@click.option('--workers', type=int, default=None, help='worker slots (default: GPUs + 2)')
def start(daemon, workers):
    """Start broker, site, worker supervisor and workers on this machine."""
    from mlcomp_amd.db.migrate import migrate
    migrate()
    if workers is None:
        from mlcomp_amd.worker.daemon import GpuInfo
        workers = GpuInfo().count() + 2
    _launch('server', _programs(workers), daemon,
            ['mlcomp_amd.server', 'start', '--workers', str(workers)])


@main.command()
def stop():
    """Stop everything ``start`` launched."""
    from mlcomp_amd.utils.procman import stop_manager
    ok = stop_manager(config.get().CONFIG_FOLDER, 'server')
    click.echo('stopped' if ok else 'not running')


@main.command()
def status():
    """Show whether the server stack is running."""
    from mlcomp_amd.utils.procman import read_status
    s = config.get()
    found = False
    for name in ('server', 'worker'):
        st = read_status(s.CONFIG_FOLDER, name)
        if not st:
            continue
        found = True
        click.echo(f'{name} manager pid {st["pid"]}')
        for p in st.get('programs', []):
            mark = 'ok ' if p['alive'] else 'DOWN'
            click.echo(f'  ({mark}) {p["name"]:11s} pid {p["pid"]} restarts {p["restarts"]}')
    if not found:
        click.echo('There are no mlcomp services started')


if __name__ == '__main__':
    main()
