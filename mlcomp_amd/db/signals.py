"""Heartbeat-by-write ORM events (`mlcomp/db/signals.py:29-69` semantics).

* Task update -> its ``last_activity`` (and its parent's) = now
* Step insert/update, Log insert -> the owning task's ``last_activity`` = now
* ReportImg insert -> ``dag.img_size += size``

Unlike the reference (which opens a second session inside the event and commits it),
the updates are issued on the *same connection* that is flushing the triggering row,
so they join its transaction: no second writer, no SQLite lock contention.
"""
from __future__ import annotations

import sqlalchemy as sa
from sqlalchemy import event

from .models import Dag, Log, ReportImg, Step, Task, now

_task = Task.__table__
_dag = Dag.__table__
_step = Step.__table__


@event.listens_for(Task, 'before_update')
def _task_before_update(mapper, connection, target):
    target.last_activity = now()
    if target.parent:
        connection.execute(sa.update(_task).where(_task.c.id == target.parent)
                           .values(last_activity=target.last_activity))


@event.listens_for(Step, 'before_insert')
@event.listens_for(Step, 'before_update')
def _step_touch(mapper, connection, target):
    if target.task is not None:
        connection.execute(sa.update(_task).where(_task.c.id == target.task).values(last_activity=now()))


@event.listens_for(Log, 'before_insert')
def _log_touch(mapper, connection, target):
    task = target.task
    if task is None and target.step is not None:
        task = connection.execute(sa.select(_step.c.task).where(_step.c.id == target.step)).scalar()
    if task is not None:
        connection.execute(sa.update(_task).where(_task.c.id == task).values(last_activity=now()))


@event.listens_for(ReportImg, 'before_insert')
def _img_size(mapper, connection, target):
    if target.dag is not None:
        connection.execute(sa.update(_dag).where(_dag.c.id == target.dag)
                           .values(img_size=_dag.c.img_size + (target.size or 0)))


INSTALLED = True
