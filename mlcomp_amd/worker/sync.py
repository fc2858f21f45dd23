"""Data/artefact sync between computers over rsync/ssh (`mlcomp/worker/sync.py:20-239`).

Code travels through the DB; data and model folders are rsync'ed: for every Success
task computed on another computer and not yet recorded in ``task_synced``, the
project's ``sync_folders`` (minus ``ignore_folders``) are pulled from that computer.
``copy_remote`` fetches a single file (checkpoint resume) with scp, or a local copy
when the source is this host (the reference forgot to assign that command).
On a single MI355X node nothing needs syncing; the module is used by multi-node setups.
"""
from __future__ import annotations

import os
import shlex
import shutil
import subprocess
from os.path import join
from typing import List, Tuple

from mlcomp_amd.db.enums import ComponentType
from mlcomp_amd.db.models import Computer, TaskSynced, now
from mlcomp_amd.db.providers import ComputerProvider, TaskSyncedProvider
from mlcomp_amd.utils.logging import create_logger
from .tasks import hostname


def rsync_command(source: Computer, target: Computer, folder: str, excluded: List[str],
                  current: str) -> str:
    end = '--perms --chmod=777 --size-only'
    for e in excluded:
        if e.startswith(folder) and e != folder:
            end += f' --exclude {shlex.quote(os.path.relpath(e, folder))}'
    src = join(source.root_folder, folder)
    dst = join(target.root_folder, folder)
    if current == source.name:
        return (f'rsync -vhru -e "ssh -p {target.port} -o StrictHostKeyChecking=no" {src}/ '
                f'{target.user}@{target.ip}:{dst}/ {end}')
    if current == target.name:
        return (f'rsync -vhru -e "ssh -p {source.port} -o StrictHostKeyChecking=no" '
                f'{source.user}@{source.ip}:{src}/ {dst}/ {end}')
    inner = (f'rsync -vhru -e \\"ssh -p {target.port} -o StrictHostKeyChecking=no\\" {src}/ '
             f'{target.user}@{target.ip}:{dst}/ {end}')
    return f'ssh -p {source.port} {source.user}@{source.ip} "{inner}"'


def sync_directed(session, source: Computer, target: Computer, folders: List[Tuple[str, List[str]]]):
    logger = create_logger(session, 'FileSync', console=False)
    for folder, excluded in folders:
        if folder in excluded:
            continue
        cmd = rsync_command(source, target, folder, excluded, hostname())
        logger.info(cmd, ComponentType.WorkerSupervisor, hostname())
        r = subprocess.run(cmd, shell=True, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(r.stdout + r.stderr)


def copy_remote(session, computer_from: str, path_from: str, path_to: str) -> bool:
    if computer_from == hostname():
        os.makedirs(os.path.dirname(path_to) or '.', exist_ok=True)
        shutil.copy(path_from, path_to)
    else:
        src = ComputerProvider(session).by_name(computer_from)
        subprocess.check_output(f'scp -P {src.port} {src.user}@{src.ip}:{path_from} {path_to}', shell=True)
    return os.path.exists(path_to)


def correct_folders(folders: List[str], project: str) -> List[str]:
    out = []
    for f in folders:
        parts = f.split('/')
        if parts[0] in ('data', 'models') and (len(parts) == 1 or parts[1] != project):
            parts[0] = join(parts[0], project)
        out.append('/'.join(parts))
    return out


class FileSync:
    def __init__(self, session):
        self.session = session
        self.logger = create_logger(session, 'FileSync', console=False)

    def sync(self):
        me = ComputerProvider(self.session).by_name(hostname())
        if me is None:
            return
        provider = TaskSyncedProvider(self.session)
        cp = ComputerProvider(self.session)
        for project, tasks in provider.for_computer(me.name):
            sync = correct_folders([f for f in (project.sync_folders or '').split() if f], project.name)
            ignore = correct_folders([f for f in (project.ignore_folders or '').split() if f], project.name)
            for src_name in {t.computer_assigned for t in tasks}:
                src = cp.by_name(src_name)
                if src is None or not src.sync_with_this_computer:
                    continue
                sync_directed(self.session, src, me, [(f, ignore) for f in sync])
            for t in tasks:
                provider.add(TaskSynced(computer=me.name, task=t.id), commit=False)
            me.last_synced = now()
            provider.commit()


__all__ = ['FileSync', 'sync_directed', 'copy_remote', 'correct_folders', 'rsync_command']
