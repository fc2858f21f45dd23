"""Report builders used by validation / inference executors
(`mlcomp/worker/reports/{classification,segmenation}.py`)."""
from .classification import ClassificationReportBuilder  # noqa: F401
from .segmentation import SegmentationReportBuilder  # noqa: F401
