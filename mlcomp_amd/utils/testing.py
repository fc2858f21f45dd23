"""Test fixture helper (`mlcomp/utils/tests.py:12-19`): a fresh ROOT_FOLDER with a migrated
SQLite DB and a new session, for user test suites of DAG code.

    from mlcomp_amd.utils.testing import session   # noqa  (pytest fixture)
"""
from __future__ import annotations

import pytest


@pytest.fixture
def session(tmp_path, monkeypatch):
    monkeypatch.setenv('MLCOMP_ROOT', str(tmp_path / 'mlcomp'))
    monkeypatch.setenv('ROOT_FOLDER', str(tmp_path / 'mlcomp'))
    from mlcomp_amd import broker, config
    from mlcomp_amd.db.core import Session
    from mlcomp_amd.db.migrate import migrate
    config.reset()
    Session.cleanup()
    broker.set_broker(broker.InProcBroker())
    migrate()
    s = Session.create_session(key='test')
    yield s
    broker.set_broker(None)
    Session.cleanup()
    config.reset()


__all__ = ['session']
