"""Encoder-decoder segmentation models (`mlcomp/contrib/segmentation/{base,unet,fpn,linknet,
pspnet}/model.py`) and the ``SegmentationModelPytorch`` factory
(`mlcomp/contrib/model/segmentation_model_pytorch.py:6-34`)."""
from __future__ import annotations

import torch
import torch.nn as nn

from mlcomp_amd.models import register
from .blocks import make_activation
from .decoders import FPNDecoder, LinknetDecoder, PSPDecoder, UnetDecoder
from .encoders import get_encoder


class EncoderDecoder(nn.Module):
    """``forward`` returns logits; ``predict`` = eval + no_grad + activation."""

    def __init__(self, encoder, decoder, activation):
        super().__init__()
        self.encoder = encoder
        self.decoder = decoder
        self.activation = make_activation(activation)

    def forward(self, x):
        return self.decoder(self.encoder(x))

    def predict(self, x):
        if self.training:
            self.eval()
        with torch.no_grad():
            x = self.forward(x)
            if self.activation is not None:
                x = self.activation(x)
        return x


@register('Unet')
class Unet(EncoderDecoder):
    def __init__(self, encoder_name='resnet34', encoder_weights=None, decoder_use_batchnorm=True,
                 decoder_channels=(256, 128, 64, 32, 16), classes=1, activation='sigmoid', center=False,
                 attention_type=None):
        enc = get_encoder(encoder_name, encoder_weights)
        dec = UnetDecoder(enc.out_shapes, decoder_channels, classes, decoder_use_batchnorm, center, attention_type)
        super().__init__(enc, dec, activation)
        self.name = f'u-{encoder_name}'


@register('FPN')
class FPN(EncoderDecoder):
    def __init__(self, encoder_name='resnet34', encoder_weights=None, decoder_pyramid_channels=256,
                 decoder_segmentation_channels=128, classes=1, dropout=0.2, activation='sigmoid'):
        enc = get_encoder(encoder_name, encoder_weights)
        dec = FPNDecoder(enc.out_shapes, decoder_pyramid_channels, decoder_segmentation_channels, classes, dropout)
        super().__init__(enc, dec, activation)
        self.name = f'fpn-{encoder_name}'


@register('Linknet')
class Linknet(EncoderDecoder):
    def __init__(self, encoder_name='resnet34', encoder_weights=None, decoder_use_batchnorm=True, classes=1,
                 activation='sigmoid'):
        enc = get_encoder(encoder_name, encoder_weights)
        dec = LinknetDecoder(enc.out_shapes, 32, classes, decoder_use_batchnorm)
        super().__init__(enc, dec, activation)
        self.name = f'link-{encoder_name}'


@register('PSPNet')
class PSPNet(EncoderDecoder):
    def __init__(self, encoder_name='resnet34', encoder_weights=None, psp_in_factor=8, psp_out_channels=512,
                 psp_use_batchnorm=True, psp_aux_output=False, classes=21, dropout=0.2, activation='softmax'):
        enc = get_encoder(encoder_name, encoder_weights)
        dec = PSPDecoder(enc.out_shapes, psp_in_factor, psp_use_batchnorm, psp_out_channels, classes,
                         psp_aux_output, dropout)
        super().__init__(enc, dec, activation)
        self.name = f'psp-{encoder_name}'


ARCHS = {'unet': Unet, 'fpn': FPN, 'linknet': Linknet, 'pspnet': PSPNet}


@register('SegmentationModelPytorch')
def segmentation_model_pytorch(arch: str, encoder: str = 'resnet34', num_classes: int = 1,
                               encoder_weights=None, activation='sigmoid', **kw):
    """Factory by architecture + encoder name."""
    a = arch.lower()
    if a == 'deeplab' or a == 'deeplabv3':
        from .deeplab import DeepLab
        return DeepLab(backbone=encoder, num_classes=num_classes, **kw)
    if a not in ARCHS:
        raise ValueError(f'unknown arch {arch}; one of {list(ARCHS)} or deeplab')
    return ARCHS[a](encoder_name=encoder, encoder_weights=encoder_weights, classes=num_classes,
                    activation=activation, **kw)


# catalyst-era registry names the reference's YAMLs use (`contrib/catalyst/register.py:16-42`)
def _alias(name, cls, **fixed):
    register(name)(lambda **kw: cls(**{**fixed, **kw}))


_alias('ResnetUnet', Unet)
_alias('MobileUnet', Unet, encoder_name='mobilenet_v2')
_alias('ResnetFPNUnet', FPN)
_alias('FPNUnet', FPN)
_alias('ResnetLinknet', Linknet)
_alias('ResNetLinknet', Linknet)
_alias('ResnetPSPnet', PSPNet)
_alias('PSPnet', PSPNet)

__all__ = ['EncoderDecoder', 'Unet', 'FPN', 'Linknet', 'PSPNet', 'segmentation_model_pytorch']
