"""Extra model families for config-driven training.

* ``Pretrained`` - the reference's classification wrapper
  (`mlcomp/contrib/model/pretrained.py:8-58`): a registered backbone (``variant``)
  with its classifier resized to ``num_classes`` and an optional output activation.
  There is no network access, so ``pretrained`` takes a local checkpoint path
  (loaded with ``weights_only=True``) instead of downloading.
* ``SimpleCNN`` - small LeNet-style net for MNIST/CIFAR-shaped smoke configs.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import MODELS, register


def _activation(a):
    if a is None or callable(a):
        return a
    if a == 'softmax':
        return nn.Softmax(dim=1)
    if a == 'sigmoid':
        return nn.Sigmoid()
    raise ValueError('activation should be "sigmoid"/"softmax"/callable/None')


@register('Pretrained')
class Pretrained(nn.Module):
    def __init__(self, variant: str, num_classes: int, pretrained=None, activation=None, **kw):
        super().__init__()
        self.model = MODELS[variant](num_classes=num_classes, **kw)
        if isinstance(pretrained, str):
            sd = torch.load(pretrained, map_location='cpu', weights_only=True)
            sd = sd.get('model_state_dict', sd)
            own = self.model.state_dict()
            sd = {k: v for k, v in sd.items() if k in own and own[k].shape == v.shape}
            self.model.load_state_dict(sd, strict=False)
        self.activation = _activation(activation)

    def forward(self, x):
        y = self.model(x)
        if isinstance(y, tuple):
            y = y[0]
        return self.activation(y) if self.activation else y


@register('LeNet')
class LeNet(nn.Module):
    """The digit-recognizer example net (`examples/digit-recognizer/model.py:8-25`):
    conv5(20) -> pool -> conv5(50) -> pool -> fc(500) -> fc(classes), log-softmax out."""

    def __init__(self, in_channels: int = 1, num_classes: int = 10, image_size: int = 28):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, 20, 5)
        self.conv2 = nn.Conv2d(20, 50, 5)
        s = ((image_size - 4) // 2 - 4) // 2
        self.fc1 = nn.Linear(50 * s * s, 500)
        self.fc2 = nn.Linear(500, num_classes)

    def forward(self, x):
        x = torch.nn.functional.max_pool2d(torch.relu(self.conv1(x)), 2)
        x = torch.nn.functional.max_pool2d(torch.relu(self.conv2(x)), 2)
        x = torch.relu(self.fc1(x.flatten(1)))
        return torch.log_softmax(self.fc2(x), dim=1)


@register('SimpleCNN')
class SimpleCNN(nn.Module):
    def __init__(self, in_channels: int = 3, num_classes: int = 10, width: int = 16, image_size: int = 32):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(in_channels, width, 3, padding=1), nn.BatchNorm2d(width), nn.ReLU(inplace=True),
            nn.MaxPool2d(2),
            nn.Conv2d(width, 2 * width, 3, padding=1), nn.BatchNorm2d(2 * width), nn.ReLU(inplace=True),
            nn.AdaptiveAvgPool2d(1))
        self.fc = nn.Linear(2 * width, num_classes)

    def forward(self, x):
        return self.fc(self.features(x).flatten(1))


class EncoderClassifier(nn.Module):
    """Any segmentation encoder (densenet / se_resnet / senet154 / dpn / vgg / mobilenet
    ...) as an image classifier: deepest feature -> global average pool -> linear.  Gives
    ``Pretrained`` / ``Timm`` the pretrainedmodels-style variants without that package."""

    def __init__(self, encoder_name: str, num_classes: int = 1000, in_channels: int = 3):
        super().__init__()
        from mlcomp_amd.contrib.segmentation.encoders import get_encoder
        self.encoder = get_encoder(encoder_name)
        self.fc = nn.Linear(self.encoder.out_shapes[0], num_classes)

    def forward(self, x):
        f = self.encoder(x)[0]
        return self.fc(torch.flatten(torch.nn.functional.adaptive_avg_pool2d(f, 1), 1))


def _register_encoder_classifiers():
    from mlcomp_amd.contrib.segmentation.encoders import ENCODERS
    for name in ENCODERS:
        if name not in MODELS:
            register(name)((lambda n: (lambda num_classes=1000, **kw: EncoderClassifier(n, num_classes, **kw)))(name))


_TIMM_ALIASES = {f'efficientnet_b{i}': f'efficientnet-b{i}' for i in range(8)}
_TIMM_ALIASES.update({f'tf_efficientnet_b{i}': f'efficientnet-b{i}' for i in range(8)})
_TIMM_ALIASES.update({'mobilenetv2_100': 'mobilenet_v2', 'seresnet50': 'se_resnet50',
                      'seresnext50_32x4d': 'se_resnext50_32x4d', 'dpn68b': 'dpn68'})


@register('Timm')
class Timm(Pretrained):
    """The reference's timm wrapper (`mlcomp/contrib/model/timm.py:5-40`): timm is not in
    this stack, so timm variant names are mapped onto the native registry."""

    def __init__(self, variant: str, num_classes: int, pretrained=None, activation=None, **kw):
        _register_encoder_classifiers()
        name = _TIMM_ALIASES.get(variant, variant)
        if name not in MODELS:
            raise KeyError(f'timm variant {variant!r} has no native equivalent; registered: {sorted(MODELS)}')
        super().__init__(name, num_classes, pretrained if isinstance(pretrained, str) else None, activation, **kw)


_register_encoder_classifiers()

__all__ = ['Pretrained', 'SimpleCNN', 'LeNet', 'EncoderClassifier', 'Timm']
