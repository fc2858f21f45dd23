"""Transforms: RLE mask codec, test-time augmentation wrapper, tensor layout helpers
(`mlcomp/contrib/transform/{rle,tta,albumentations}.py`)."""
from .rle import mask2rle, rle2mask  # noqa: F401
from .tta import TtaWrap  # noqa: F401
from .layout import ChannelTranspose, Ensure4d  # noqa: F401
