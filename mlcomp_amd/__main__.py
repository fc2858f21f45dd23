"""``mlcomp`` command line (`mlcomp/__main__.py:107-256`).

    mlcomp migrate                      create / upgrade the DB schema
    mlcomp dag CONFIG [--params k:v]*   submit a DAG (one per grid cell)
    mlcomp execute CONFIG [--params]    run a DAG locally, in this process, on all GPUs
    mlcomp report                       zip diagnostics into REPORT_FOLDER
    mlcomp sync PROJECT [...]           rsync a project's folders with other computers
    mlcomp init                         detect the NIC for RCCL/NCCL_SOCKET_IFNAME
    mlcomp status                       print the health checks
    mlcomp build                        compile the native kernels / broker / runtime
"""
from __future__ import annotations

import os
import socket
import sys

import click


def _session(key='cli'):
    from mlcomp_amd.db.core import Session
    return Session.create_session(key=key)


def _dag(config_path: str, debug: bool = False, control_reqs: bool = True, params=()):
    from mlcomp_amd.dag import dag_from_config
    from mlcomp_amd.db.enums import ComponentType
    from mlcomp_amd.utils.logging import create_logger
    from mlcomp_amd.utils.misc import dict_from_list_str, yaml_load
    s = _session()
    logger = create_logger(s, name='_dag')
    text = open(config_path).read()
    cfg = yaml_load(text)
    logger.info('config parsed', ComponentType.Client)
    folder = os.path.dirname(os.path.abspath(config_path))
    cwd = os.getcwd()
    os.chdir(folder)   # code upload walks the config's folder
    try:
        return dag_from_config(s, cfg, config_path=config_path, config_text=text, debug=debug,
                               params=dict_from_list_str(list(params)), logger=logger,
                               component=ComponentType.Client, control_reqs=control_reqs)
    finally:
        os.chdir(cwd)


def _register_this_computer():
    from mlcomp_amd.worker.daemon import GpuInfo, register_computer
    return register_computer(_session(), GpuInfo())


@click.group()
def main():
    pass


@main.command()
def migrate():
    """Create or upgrade the database schema."""
    from mlcomp_amd.db.migrate import migrate as _migrate
    v = _migrate()
    click.echo(f'schema version {v}')


@main.command()
@click.argument('config')
@click.option('--control_reqs', type=bool, default=True)
@click.option('--params', multiple=True, help='key:value overrides (suffix match)')
def dag(config, control_reqs, params):
    """Submit a DAG to the scheduler."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    for d in _dag(config, control_reqs=control_reqs, params=params):
        click.echo(f'dag created: {d}')


@main.command()
@click.argument('config')
@click.option('--debug', type=bool, default=True)
@click.option('--params', multiple=True)
def execute(config, debug, params):
    """Run every task of the DAG here, in dependency order, on all local GPUs."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    from mlcomp_amd.db.enums import ComponentType, TaskStatus
    from mlcomp_amd.db.providers import StepProvider, TaskProvider
    from mlcomp_amd.utils.logging import create_logger
    from mlcomp_amd.worker.daemon import GpuInfo
    from mlcomp_amd.worker.tasks import execute_by_id
    s = _session()
    _register_this_computer()
    logger = create_logger(s, __name__)
    tp = TaskProvider(s)
    wi = int(os.environ.get('WORKER_INDEX', -1))
    for t in tp.by_status(TaskStatus.InProgress, worker_index=wi):
        logger.error(f'Task Id = {t.id} was in InProgress state when another task arrived to the same worker',
                     ComponentType.Worker, t.computer_assigned, t.id, StepProvider(s).last_for_task(t.id))
        tp.change_status(t, TaskStatus.Failed)
    n = GpuInfo().count()
    for d in _dag(config, debug=debug, params=params):
        for ids in d.values():
            for tid in ids:
                t = tp.by_id(tid)
                t.gpu_assigned = ','.join(map(str, range(n)))
                t.computer_assigned = os.environ.get('MLCOMP_COMPUTER') or socket.gethostname()
                tp.commit()
                execute_by_id(tid, exit_process=False)


@main.command()
def report():
    """Write the diagnostics bundle."""
    from mlcomp_amd.report import create_report
    create_report()


@main.command()
def status():
    """Print the health checks."""
    from mlcomp_amd.report import statuses
    for k, v in statuses().items():
        click.echo(f'{"ok " if v["ok"] else "ERR"} {k:9s} {v["message"]}')


@main.command()
@click.argument('project')
@click.option('--computer', help='sync this computer with all the others')
@click.option('--only_from', is_flag=True, help='only copy from the computer to the others')
@click.option('--only_to', is_flag=True, help='only copy from the others to the computer')
@click.option('--online', is_flag=True, help='only computers seen in the last 100 s')
def sync(project, computer, only_from, only_to, online):
    """Sync a project's ``sync_folders`` between computers (rsync over ssh)."""
    from mlcomp_amd.report import check_statuses
    check_statuses()
    from mlcomp_amd.db.models import now
    from mlcomp_amd.db.providers import ComputerProvider, ProjectProvider
    from mlcomp_amd.utils.misc import yaml_load
    from mlcomp_amd.worker.sync import correct_folders, sync_directed
    s = _session()
    name = _register_this_computer()
    cp = ComputerProvider(s)
    me = cp.by_name(computer or name)
    p = ProjectProvider(s).by_name(project)
    if p is None:
        raise click.ClickException(f'Project={project} is not found')
    sync_folders = correct_folders(yaml_load(p.sync_folders) or [], p.name)
    ignore = correct_folders(yaml_load(p.ignore_folders) or [], p.name)
    folders = [(f, ignore) for f in (sync_folders if isinstance(sync_folders, list) else [])]
    for c, last in cp.all_with_last_activity():
        if c.name == me.name:
            continue
        if online and (last is None or (now() - last).total_seconds() > 100):
            continue
        if not only_from:
            sync_directed(s, me, c, folders)
        if not only_to:
            sync_directed(s, c, me, folders)


@main.command()
def init():
    """Write the default network interface into configs/.env (NCCL_SOCKET_IFNAME)."""
    from mlcomp_amd import config
    from mlcomp_amd.utils.misc import default_network_interface
    s = config.get()
    path = os.path.join(s.CONFIG_FOLDER, '.env')
    lines = open(path).readlines() if os.path.exists(path) else []
    iface = default_network_interface()
    if iface:
        lines = [l for l in lines if not l.startswith('NCCL_SOCKET_IFNAME')]
        lines.append(f'NCCL_SOCKET_IFNAME={iface}\n')
        with open(path, 'w') as f:
            f.writelines(lines)
    click.echo(f'NCCL_SOCKET_IFNAME={iface}')


@main.command()
def build():
    """Compile the HIP kernel library, the broker and the runtime library."""
    from mlcomp_amd.build import build_all
    build_all(verbose=True)


@main.command()
def submit():
    """Kaggle kernel submission described by ./submit.yml."""
    from mlcomp_amd.utils.misc import yaml_load
    from mlcomp_amd.worker.executors.kaggle import Submit
    if not os.path.exists('submit.yml'):
        raise click.ClickException('no file submit.yml')
    d = yaml_load(file='submit.yml')
    Submit(competition=d['competition'], submit_type='kernel', max_size=d.get('max_size', 1),
           folders=d.get('folders', []), datasets=d.get('datasets', []), files=d.get('files', [])).work()


if __name__ == '__main__':
    main()
