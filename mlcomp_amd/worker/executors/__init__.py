"""Executors: the units of work a DAG node runs (`mlcomp/worker/executors/**`)."""
from .base import Executor, StepWrap, TqdmWrapper  # noqa: F401

_LOADED = False
# builtin executor type (lower case, no underscores) -> the module that registers it.  A task
# process imports only its own executor's module: a bash task does not pay the ~3 s import of
# torch and the training stack (the dispatch -> start latency of small tasks).
_BUILTIN = {'bash': 'bash', 'click': 'click_', 'split': 'split', 'train': 'train', 'catalyst': 'train',
            'modeladd': 'model', 'download': 'kaggle', 'submit': 'kaggle', 'equation': 'equation',
            'valid': 'valid', 'infer': 'infer'}


def load_builtin_executors(type_name: str = None):
    """Import (and thereby register) the executors shipped with the framework - only the
    one that registers ``type_name`` when it is a builtin, else all of them."""
    global _LOADED
    if type_name is not None:
        mod = _BUILTIN.get(str(type_name).lower().replace('_', ''))
        if mod is not None:
            __import__(f'{__name__}.{mod}')
            if Executor.is_registered(type_name):
                return
    if _LOADED:
        return
    _LOADED = True
    from . import bash, click_, split  # noqa: F401
    for mod in ('train', 'model', 'kaggle', 'equation', 'valid', 'infer'):
        try:
            __import__(f'{__name__}.{mod}')
        except ImportError:
            pass
