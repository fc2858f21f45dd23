"""Engine/session registry (`mlcomp/db/core/db.py:10-122` equivalent).

Sessions are keyed singletons: every component (API request threads, scheduler
thread, worker process, worker-supervisor jobs) asks for its own key so their
transactions never interleave.  SQLite runs with WAL, a 30 s busy timeout and
foreign keys ON (``ON DELETE CASCADE`` is relied upon by DAG/task removal).
"""
from __future__ import annotations

import threading
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import sqlalchemy as sa
from sqlalchemy import event
from sqlalchemy.orm import Session as _SASession
from sqlalchemy.orm import sessionmaker

from mlcomp_amd import config


class Session(_SASession):
    _registry: Dict[str, Tuple['Session', sa.engine.Engine]] = {}
    _lock = threading.Lock()

    @staticmethod
    def create_session(*, connection_string: Optional[str] = None, key: str = 'default') -> 'Session':
        with Session._lock:
            if key in Session._registry:
                return Session._registry[key][0]
            cs = connection_string or config.get().SA_CONNECTION_STRING
            connect_args = {}
            sqlite = cs.startswith('sqlite')
            if sqlite:
                connect_args = {'check_same_thread': False, 'timeout': 30}
            engine = sa.create_engine(cs, echo=False, connect_args=connect_args)
            if sqlite:
                @event.listens_for(engine, 'connect')
                def _pragmas(dbapi_con, _rec):
                    cur = dbapi_con.cursor()
                    cur.execute('pragma foreign_keys=ON')
                    cur.execute('pragma journal_mode=WAL')
                    cur.execute('pragma busy_timeout=30000')
                    cur.close()
            s = sessionmaker(bind=engine, class_=Session, expire_on_commit=False)()
            Session._registry[key] = (s, engine)
            return s

    @classmethod
    def cleanup(cls, key: Optional[str] = None):
        with cls._lock:
            keys = [key] if key else list(cls._registry)
            for k in keys:
                if k not in cls._registry:
                    continue
                s, engine = cls._registry.pop(k)
                try:
                    s.close()
                except Exception:
                    pass
                try:
                    engine.dispose()
                except Exception:
                    pass

    def add(self, obj, commit: bool = True, _warn: bool = True):  # noqa: D401
        super().add(obj, _warn=_warn)
        if commit:
            self.commit()
        return obj

    def add_all(self, objs, commit: bool = True):
        super().add_all(objs)
        if commit:
            self.commit()

    def commit(self):
        try:
            super().commit()
        except Exception:
            self.rollback()
            raise

    def update(self):
        self.commit()

    @staticmethod
    def sqlalchemy_error(e) -> bool:
        return 'sqlalchemy.' in str(type(e))


@dataclass
class PaginatorOptions:
    page_number: int = 0
    page_size: int = 0
    sort_column: str = ''
    sort_descending: bool = True


__all__ = ['Session', 'PaginatorOptions']
