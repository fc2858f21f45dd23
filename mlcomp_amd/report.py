"""Health checks and the diagnostics bundle (`mlcomp/report.py:21-185`).

``statuses()`` probes every dependency a command needs: the ROOT_FOLDER tree, the
database (connect + schema version == latest), the task broker (PING) and - new here -
the native kernel library and the visible MI355X devices (through amdsmi, without
creating a HIP context).  ``check_statuses()`` is the gate every CLI command calls: it
prints what is broken and exits non-zero.  ``create_report()`` zips the statuses, the
log files and the last 1000 error / service log rows into ``REPORT_FOLDER``.
"""
from __future__ import annotations

import json
import os
import sys
import zipfile
from collections import OrderedDict
from os.path import exists, join

from mlcomp_amd import config


def _check_folders(s):
    missing = [f for f in (s.ROOT_FOLDER, s.DATA_FOLDER, s.MODEL_FOLDER, s.TASK_FOLDER, s.LOG_FOLDER,
                           s.CONFIG_FOLDER, s.DB_FOLDER, s.REPORT_FOLDER, s.TMP_FOLDER) if not exists(f)]
    return (not missing, 'ok' if not missing else f'missing: {missing}')


def _check_db(s):
    try:
        from mlcomp_amd.db.core import Session
        from mlcomp_amd.db.migrate import LATEST, current_version
        sess = Session.create_session(key='report_status')
        v = current_version(sess.get_bind())
        if v != LATEST:
            return False, f'schema version {v} != {LATEST} (run `mlcomp migrate`)'
        return True, f'ok ({s.DB_TYPE}, schema v{v})'
    except Exception as e:
        return False, f'{type(e).__name__}: {e}'


def _check_broker(s):
    try:
        from mlcomp_amd.broker import new_connection
        b = new_connection()
        return (True, 'ok') if b.ping() else (False, 'no PING reply')
    except Exception as e:
        return False, f'{type(e).__name__}: {e} (start it with `mlcomp-server start`)'


def _check_kernels(s):
    from mlcomp_amd.build import KERNEL_LIB
    if not exists(KERNEL_LIB):
        return False, f'{KERNEL_LIB} not built (python -m mlcomp_amd.build)'
    return True, KERNEL_LIB


def _check_gpus(s):
    try:
        from mlcomp_amd.worker.daemon import GpuInfo
        g = GpuInfo()
        return True, f'{g.count()} device(s)'
    except Exception as e:
        return True, f'unknown ({e})'


CHECKS = OrderedDict(folders=_check_folders, database=_check_db, broker=_check_broker,
                     kernels=_check_kernels, gpus=_check_gpus)
REQUIRED = ('folders', 'database')


def statuses(names=None) -> 'OrderedDict[str, dict]':
    s = config.get()
    out = OrderedDict()
    for name, fn in CHECKS.items():
        if names and name not in names:
            continue
        ok, msg = fn(s)
        out[name] = {'ok': bool(ok), 'message': msg}
    return out


def check_statuses(required=REQUIRED, broker: bool = False):
    req = list(required) + (['broker'] if broker else [])
    st = statuses(req)
    bad = {k: v for k, v in st.items() if not v['ok']}
    if bad:
        for k, v in bad.items():
            print(f'[mlcomp] {k}: {v["message"]}', file=sys.stderr)
        sys.exit(1)
    return st


def create_report(path: str = None) -> str:
    s = config.get()
    os.makedirs(s.REPORT_FOLDER, exist_ok=True)
    path = path or join(s.REPORT_FOLDER, 'report.zip')
    st = statuses()
    with zipfile.ZipFile(path, 'w', zipfile.ZIP_DEFLATED) as z:
        z.writestr('statuses.json', json.dumps(st, indent=2))
        if exists(s.LOG_FOLDER):
            for f in sorted(os.listdir(s.LOG_FOLDER)):
                p = join(s.LOG_FOLDER, f)
                if os.path.isfile(p):
                    z.write(p, join('logs', f))
        if st.get('database', {}).get('ok'):
            from mlcomp_amd.db.core import Session
            from mlcomp_amd.db.enums import ComponentType, LogStatus
            from mlcomp_amd.db.models import Log
            sess = Session.create_session(key='report_status')
            for name, q in (('errors', Log.level >= LogStatus.Error.value),
                            ('service', Log.component != ComponentType.Worker.value)):
                rows = sess.query(Log).filter(q).order_by(Log.id.desc()).limit(1000).all()
                z.writestr(f'{name}.txt', '\n'.join(
                    f'{r.time} [{r.level}] c={r.component} task={r.task} {r.message}' for r in rows))
    print(f'report written to {path}')
    return path


__all__ = ['statuses', 'check_statuses', 'create_report', 'CHECKS']
