"""Persistence layer: schema-compatible ORM models, session registry, migrations,
providers, report-layout model and heartbeat signals."""
from .core import PaginatorOptions, Session  # noqa: F401
from . import signals  # noqa: F401  (installs the ORM events)
