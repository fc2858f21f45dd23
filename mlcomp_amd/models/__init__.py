"""Model zoo.  Registry maps a name (as used in YAML ``model_params.model`` /
``variant``) to a constructor; mirrors the reference's catalyst registrations
(`mlcomp/contrib/catalyst/register.py:16-42`)."""
from __future__ import annotations

from typing import Callable, Dict

MODELS: Dict[str, Callable] = {}


def register(name: str = None):
    def deco(fn):
        MODELS[name or fn.__name__] = fn
        return fn
    return deco


def build_model(name: str, **kwargs):
    _populate()
    if name not in MODELS:
        raise KeyError(f'unknown model {name!r}; registered: {sorted(MODELS)}')
    return MODELS[name](**kwargs)


_POPULATED = False


def _populate():
    global _POPULATED
    if _POPULATED:
        return
    _POPULATED = True
    from . import resnet as _r
    for v in _r._SPECS:
        MODELS[v] = (lambda v: (lambda **kw: _r.resnet(v, **kw)))(v)
    from . import zoo, efficientnet, bert, cadene, nas, transformers  # noqa: F401  (register more families)
    import mlcomp_amd.contrib.segmentation  # noqa: F401
    import mlcomp_amd.contrib.video  # noqa: F401
