"""Process configuration.

Same knobs and file locations as the reference (`mlcomp/__init__.py:1-124`,
`mlcomp/docker/.env:1-26`): a ROOT_FOLDER tree (data, models, tasks, logs, configs,
db, report, tmp), ``configs/.env`` seeded from defaults on first use, an optional
``ENV=<name>`` overlay file, and ``os.environ`` taking precedence.  Differences:

* nothing happens at import time - :func:`get` builds an immutable :class:`Settings`
  lazily (tests call :func:`reset` after changing ``MLCOMP_ROOT``/``ROOT_FOLDER``);
* ``.env`` values never overwrite variables already present in the environment;
* no broker password / redis settings: the broker is the framework's own daemon
  (BROKER_HOST / BROKER_PORT).
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from os.path import join
from typing import Dict, List, Optional

DEFAULT_ENV = {
    'TOKEN': '5d2a7f73-75f8-4304-98d1-93bf7a65dc8f',
    'DB_TYPE': 'SQLITE',
    'POSTGRES_DB': 'mlcomp',
    'POSTGRES_USER': 'mlcomp',
    'POSTGRES_PASSWORD': '12345',
    'POSTGRES_HOST': 'localhost',
    'POSTGRES_PORT': '5432',
    'BROKER_HOST': '127.0.0.1',
    'BROKER_PORT': '6380',
    'WEB_HOST': '0.0.0.0',
    'WEB_PORT': '4201',
    'CONSOLE_LOG_LEVEL': 'INFO',
    'FILE_LOG_LEVEL': 'INFO',
    'DB_LOG_LEVEL': 'INFO',
    'IP': '127.0.0.1',
    'PORT': '22',
    'MASTER_PORT_RANGE': '29500-29510',
    'NCCL_SOCKET_IFNAME': 'lo',
    'FILE_SYNC_INTERVAL': '0',
    'WORKER_USAGE_INTERVAL': '10',
    'INSTALL_DEPENDENCIES': 'False',
    'SYNC_WITH_THIS_COMPUTER': 'True',
    'CAN_PROCESS_TASKS': 'True',
}


def _parse_env_file(path: str) -> Dict[str, str]:
    out = {}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith('#') or '=' not in line:
                continue
            k, v = line.split('=', 1)
            out[k.strip()] = v.strip()
    return out


@dataclass(frozen=True)
class Settings:
    ROOT_FOLDER: str
    env: Dict[str, str] = field(repr=False)

    # folders -----------------------------------------------------------------
    @property
    def DATA_FOLDER(self):
        return join(self.ROOT_FOLDER, 'data')

    @property
    def MODEL_FOLDER(self):
        return join(self.ROOT_FOLDER, 'models')

    @property
    def TASK_FOLDER(self):
        return join(self.ROOT_FOLDER, 'tasks')

    @property
    def LOG_FOLDER(self):
        return join(self.ROOT_FOLDER, 'logs')

    @property
    def CONFIG_FOLDER(self):
        return join(self.ROOT_FOLDER, 'configs')

    @property
    def DB_FOLDER(self):
        return join(self.ROOT_FOLDER, 'db')

    @property
    def REPORT_FOLDER(self):
        return join(self.ROOT_FOLDER, 'report')

    @property
    def TMP_FOLDER(self):
        return join(self.ROOT_FOLDER, 'tmp')

    # values ------------------------------------------------------------------
    def str(self, key: str, default: Optional[str] = None) -> Optional[str]:
        return self.env.get(key, default)

    def int(self, key: str, default: int = 0) -> int:
        v = self.env.get(key)
        return int(v) if v not in (None, '') else default

    def bool(self, key: str, default: bool = False) -> bool:
        v = self.env.get(key)
        return default if v is None else v.strip().lower() in ('1', 'true', 'yes')

    @property
    def TOKEN(self):
        return self.str('TOKEN')

    @property
    def DB_TYPE(self):
        return self.str('DB_TYPE', 'SQLITE').upper()

    @property
    def SA_CONNECTION_STRING(self):
        if self.env.get('SA_CONNECTION_STRING'):
            return self.env['SA_CONNECTION_STRING']
        if self.DB_TYPE == 'POSTGRESQL':
            e = self.env
            return (f"postgresql+psycopg2://{e['POSTGRES_USER']}:{e['POSTGRES_PASSWORD']}@"
                    f"{e['POSTGRES_HOST']}:{e['POSTGRES_PORT']}/{e['POSTGRES_DB']}")
        if self.DB_TYPE == 'SQLITE':
            return f'sqlite:///{self.DB_FOLDER}/sqlite3.sqlite'
        raise ValueError(f'Unknown DB_TYPE = {self.DB_TYPE}')

    @property
    def MASTER_PORT_RANGE(self) -> List[int]:
        a, b = self.str('MASTER_PORT_RANGE', '29500-29510').split('-')
        return [int(a), int(b)]

    @property
    def WEB_HOST(self):
        return self.str('WEB_HOST', '0.0.0.0')

    @property
    def WEB_PORT(self):
        return self.int('WEB_PORT', 4201)

    @property
    def BROKER_HOST(self):
        return self.str('BROKER_HOST', '127.0.0.1')

    @property
    def BROKER_PORT(self):
        return self.int('BROKER_PORT', 6380)

    @property
    def IP(self):
        return self.str('IP', '127.0.0.1')

    @property
    def PORT(self):
        return self.int('PORT', 22)

    @property
    def WORKER_INDEX(self):
        return self.int('WORKER_INDEX', -1)

    @property
    def FILE_SYNC_INTERVAL(self):
        return self.int('FILE_SYNC_INTERVAL', 0)

    @property
    def WORKER_USAGE_INTERVAL(self):
        return self.int('WORKER_USAGE_INTERVAL', 10)

    @property
    def INSTALL_DEPENDENCIES(self):
        return self.bool('INSTALL_DEPENDENCIES')

    @property
    def SYNC_WITH_THIS_COMPUTER(self):
        return self.bool('SYNC_WITH_THIS_COMPUTER', True)

    @property
    def CAN_PROCESS_TASKS(self):
        return self.bool('CAN_PROCESS_TASKS', True)

    @property
    def DOCKER_IMG(self):
        return self.str('DOCKER_IMG', 'default')

    @property
    def LOG_NAME(self):
        return self.str('LOG_NAME', 'log')

    @property
    def CONSOLE_LOG_LEVEL(self):
        return self.str('CONSOLE_LOG_LEVEL', 'INFO')

    @property
    def FILE_LOG_LEVEL(self):
        return self.str('FILE_LOG_LEVEL', 'INFO')

    @property
    def DB_LOG_LEVEL(self):
        return self.str('DB_LOG_LEVEL', 'INFO')


_LOCK = threading.Lock()
_SETTINGS: Optional[Settings] = None


def _root() -> str:
    r = os.getenv('MLCOMP_ROOT') or os.getenv('ROOT_FOLDER') or '~/mlcomp'
    root = os.path.abspath(os.path.expanduser(r))
    worker = os.getenv('PYTEST_XDIST_WORKER')
    if worker and not os.getenv('MLCOMP_ROOT'):
        root = join(root, 'tests', worker)
    return root


def get() -> Settings:
    global _SETTINGS
    if _SETTINGS is not None:
        return _SETTINGS
    with _LOCK:
        if _SETTINGS is not None:
            return _SETTINGS
        root = _root()
        for sub in ('', 'data', 'models', 'tasks', 'logs', 'configs', 'db', 'report', 'tmp'):
            os.makedirs(join(root, sub), exist_ok=True)
        env_file = join(root, 'configs', '.env')
        if not os.path.exists(env_file):
            with open(env_file, 'w') as f:
                for k, v in DEFAULT_ENV.items():
                    f.write(f'{k}={v}\n')
        env = dict(DEFAULT_ENV)
        env.update(_parse_env_file(env_file))
        extra = os.getenv('ENV')
        if extra:
            env.update(_parse_env_file(join(root, 'configs', extra + '.env')))
        for k in list(env) + ['SA_CONNECTION_STRING', 'DOCKER_IMG', 'WORKER_INDEX', 'LOG_NAME']:
            if k in os.environ:
                env[k] = os.environ[k]
        _SETTINGS = Settings(ROOT_FOLDER=root, env=env)
        return _SETTINGS


def reset():
    global _SETTINGS
    with _LOCK:
        _SETTINGS = None
