"""Executors: the units of work a DAG node runs (`mlcomp/worker/executors/**`)."""
from .base import Executor, StepWrap, TqdmWrapper  # noqa: F401

_LOADED = False


def load_builtin_executors():
    """Import (and thereby register) every executor shipped with the framework."""
    global _LOADED
    if _LOADED:
        return
    _LOADED = True
    from . import bash, click_, split  # noqa: F401
    for mod in ('train', 'model', 'kaggle', 'equation', 'valid', 'infer'):
        try:
            __import__(f'{__name__}.{mod}')
        except ImportError:
            pass
