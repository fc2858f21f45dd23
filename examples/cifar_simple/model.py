"""A small CIFAR-10 convnet registered under the name the training config uses."""
import torch.nn as nn

from mlcomp_amd.models import register


@register('CifarNet')
class CifarNet(nn.Module):
    def __init__(self, num_classes: int = 10, width: int = 32):
        super().__init__()

        def block(cin, cout):
            return nn.Sequential(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout),
                                 nn.ReLU(inplace=True), nn.MaxPool2d(2))
        self.features = nn.Sequential(block(3, width), block(width, 2 * width), block(2 * width, 4 * width))
        self.head = nn.Linear(4 * width * 16, num_classes)

    def forward(self, x):
        return self.head(self.features(x).flatten(1))
