"""DAG builders: YAML -> DB rows (standard, pipe, copy/restart, model add/start)."""
from .standard import dag_standard, dag_from_config, DagConfigError  # noqa: F401
