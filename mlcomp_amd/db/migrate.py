"""Versioned schema migrations (replacement for the unmaintained sqlalchemy-migrate repo
at `mlcomp/migration/`).

Version numbers and effects match the reference (`mlcomp/migration/versions/001..010`):
1 base tables, 2 seed report layouts, 3 task.loss, 4 task.continued, 5 project
sync/ignore folders, 6 space, 7 space_relation, 8 space_tag, 9 dag_tag, 10 memory.
The current version is kept in the same ``migrate_version`` table sqlalchemy-migrate
uses, so ``mlcomp report``-style health checks read either framework's DB.
Every step is idempotent (inspects the live schema before altering it).
"""
from __future__ import annotations

import glob
import os
from typing import Callable, List

import sqlalchemy as sa

from .core import Session
from .models import Base, ReportLayout, now

REPO_ID = 'mlcomp'
LATEST = 10

_LATER_TABLES = {'space': 6, 'space_relation': 7, 'space_tag': 8, 'dag_tag': 9, 'memory': 10}


def _tables(engine):
    return set(sa.inspect(engine).get_table_names())


def _columns(engine, table):
    return {c['name'] for c in sa.inspect(engine).get_columns(table)}


def _create(engine, names):
    tables = [Base.metadata.tables[n] for n in names]
    Base.metadata.create_all(engine, tables=tables)


def _add_column(engine, table, col, ddl_type):
    if col not in _columns(engine, table):
        with engine.begin() as c:
            c.execute(sa.text(f'ALTER TABLE {table} ADD COLUMN {col} {ddl_type}'))


def v1(engine):
    base = [n for n in Base.metadata.tables if n not in _LATER_TABLES]
    _create(engine, base)


def v2(engine):
    seed_layouts(engine)


def v3(engine):
    _add_column(engine, 'task', 'loss', 'FLOAT')


def v4(engine):
    _add_column(engine, 'task', 'continued', 'BOOLEAN')


def v5(engine):
    _add_column(engine, 'project', 'sync_folders', "VARCHAR NOT NULL DEFAULT ''")
    _add_column(engine, 'project', 'ignore_folders', "VARCHAR NOT NULL DEFAULT ''")


def v6(engine):
    _create(engine, ['space'])


def v7(engine):
    _create(engine, ['space_relation'])


def v8(engine):
    _create(engine, ['space_tag'])


def v9(engine):
    _create(engine, ['dag_tag'])


def v10(engine):
    _create(engine, ['memory'])


STEPS: List[Callable] = [v1, v2, v3, v4, v5, v6, v7, v8, v9, v10]


def layout_dir():
    return os.path.join(os.path.dirname(__file__), 'layouts')


def seed_layouts(engine):
    with engine.begin() as c:
        existing = {r[0] for r in c.execute(sa.text('SELECT name FROM report_layout'))}
        for path in sorted(glob.glob(os.path.join(layout_dir(), '*.yml'))):
            name = os.path.basename(path).rsplit('.', 1)[0]
            if name in existing:
                continue
            c.execute(sa.insert(ReportLayout.__table__).values(
                name=name, content=open(path).read(), last_modified=now()))


def _ensure_version_table(engine):
    with engine.begin() as c:
        c.execute(sa.text('CREATE TABLE IF NOT EXISTS migrate_version ('
                          'repository_id VARCHAR(250) NOT NULL PRIMARY KEY, '
                          'repository_path TEXT, version INTEGER)'))
        row = c.execute(sa.text('SELECT version FROM migrate_version WHERE repository_id=:r'),
                        {'r': REPO_ID}).fetchone()
        if row is None:
            c.execute(sa.text('INSERT INTO migrate_version VALUES (:r, :p, 0)'),
                      {'r': REPO_ID, 'p': os.path.dirname(__file__)})


def current_version(engine) -> int:
    _ensure_version_table(engine)
    with engine.begin() as c:
        return int(c.execute(sa.text('SELECT version FROM migrate_version WHERE repository_id=:r'),
                             {'r': REPO_ID}).scalar())


def migrate(connection_string: str = None, target: int = LATEST) -> int:
    s = Session.create_session(connection_string=connection_string, key='migrate')
    engine = s.get_bind()
    v = current_version(engine)
    while v < target:
        STEPS[v](engine)
        v += 1
        with engine.begin() as c:
            c.execute(sa.text('UPDATE migrate_version SET version=:v WHERE repository_id=:r'),
                      {'v': v, 'r': REPO_ID})
    Session.cleanup('migrate')
    return v


__all__ = ['migrate', 'current_version', 'LATEST']
