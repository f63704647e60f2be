"""Model zoo: the reference ConvNet and the ResNet-50 stress config."""
from .convnet import ConvNet  # noqa: F401
from .resnet import ResNet, resnet50  # noqa: F401
