"""``register()`` - the reference's contrib/catalyst/register.py: makes the contrib
criterions, callbacks, schedulers and models resolvable by name from experiment YAML.
In this framework they are registered on import already; calling ``register()`` just
imports everything (kept for user code that calls it)."""
from __future__ import annotations


def register():
    import mlcomp_amd.contrib.criterion  # noqa: F401
    import mlcomp_amd.contrib.optim  # noqa: F401
    import mlcomp_amd.contrib.segmentation  # noqa: F401
    import mlcomp_amd.contrib.video  # noqa: F401
    import mlcomp_amd.train.callbacks  # noqa: F401
    from mlcomp_amd.models import _populate
    _populate()


__all__ = ['register']
