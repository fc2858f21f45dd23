"""Segmentation models: U-Net, FPN, LinkNet, PSPNet over a family of encoders, and
DeepLab v3+ (`mlcomp/contrib/segmentation/**`).  Importing registers them in the model
registry (``model_params.model: Unet`` etc.)."""
from .encoders import get_encoder, get_encoder_names, get_preprocessing_params, preprocess_input  # noqa: F401
from .models import FPN, PSPNet, EncoderDecoder, Linknet, Unet, segmentation_model_pytorch  # noqa: F401
from .deeplab import DeepLab  # noqa: F401
