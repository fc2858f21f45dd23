"""mlcomp_amd: an MI355X-native distributed task-DAG execution engine for ML.

Same capabilities as deepalcoholic/mlcomp (DAG YAML schema, DB layout, scheduler,
worker pool, executors, reports, REST API, CLI) with a native compute path:
hand-written CDNA4 HIP kernels for the training hot path and RCCL data parallelism.
"""
from .__version__ import __version__  # noqa: F401
