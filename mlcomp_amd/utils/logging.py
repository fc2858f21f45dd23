"""Console + rotating-file + DB logger (`mlcomp/utils/logging.py:16-159` semantics).

Call convention (same as the reference): positional args after the message are
``(component[, computer[, task[, step]]])`` and only records emitted from inside the
package are written to the ``log`` table; the message is not %-formatted with them.
"""
from __future__ import annotations

import logging
import os
import sys
from logging.handlers import RotatingFileHandler

from mlcomp_amd import config

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _from_pkg(record) -> bool:
    return record.pathname.startswith(PKG_ROOT)


class Formatter(logging.Formatter):
    def format(self, record):
        if _from_pkg(record) and record.args:
            record = logging.makeLogRecord(record.__dict__)
            record.args = ()
        return super().format(record)


class DbHandler(logging.Handler):
    def __init__(self, session):
        super().__init__()
        from mlcomp_amd.db.providers import LogProvider
        self.provider = LogProvider(session)

    def emit(self, record):
        if not _from_pkg(record) or not record.args:
            return
        try:
            from mlcomp_amd.db.models import Log, now
            args = list(record.args) + [None] * 4
            component, computer, task, step = args[:4]
            if hasattr(component, 'value'):
                component = component.value
            module = os.path.relpath(record.pathname, PKG_ROOT).replace(os.sep, '.')[:-3]
            if record.funcName and record.funcName != '<module>':
                module = f'{module}:{record.funcName}'
            msg = str(record.msg)
            if record.exc_info:
                msg += '\n' + logging.Formatter().formatException(record.exc_info)
            self.provider.add(Log(message=msg[-16000:], time=now(), level=record.levelno, step=step,
                                  component=component, line=record.lineno, module=module,
                                  task=task, computer=computer))
        except Exception:
            try:
                self.provider.rollback()
            except Exception:
                pass
            self.handleError(record)


def create_logger(session=None, name: str = 'mlcomp', db=True, file=True, console=True):
    s = config.get()
    logger = logging.Logger(name)
    fmt = '%(asctime)s.%(msecs)03d %(levelname)s %(module)s - %(funcName)s: %(message)s'
    datefmt = '%Y-%m-%d %H:%M:%S'
    if console:
        h = logging.StreamHandler(sys.stdout)
        h.setLevel(s.CONSOLE_LOG_LEVEL)
        h.setFormatter(Formatter(fmt, datefmt))
        logger.addHandler(h)
    if file:
        h = RotatingFileHandler(os.path.join(s.LOG_FOLDER, f'{s.LOG_NAME}.txt'), maxBytes=10 * 2 ** 20,
                                backupCount=1)
        h.setLevel(s.FILE_LOG_LEVEL)
        h.setFormatter(Formatter(fmt, datefmt))
        logger.addHandler(h)
    if db and session is not None:
        h = DbHandler(session)
        h.setLevel(s.DB_LOG_LEVEL)
        logger.addHandler(h)
    return logger


__all__ = ['create_logger', 'DbHandler']
