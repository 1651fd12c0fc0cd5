"""Model zoo: the reference's EnhancedCNNModel (+ its small variant) and the
BASELINE.json configs (mlp2, mlp3, lenet5, resnet18)."""
from __future__ import annotations

import torch.nn as nn

from .cnn import EnhancedCNNModel, EnhancedCNNSmall, LeNet5, ResBlock  # noqa: F401
from .layers import CrossEntropyLoss, Linear  # noqa: F401
from .mlp import MLP, mlp2, mlp3  # noqa: F401
from .resnet import ResNet, resnet18  # noqa: F401

# name -> (constructor, input kind for the synthetic dataset)
REGISTRY = {
    "enhanced_cnn": (lambda nc=10: EnhancedCNNModel(nc), "cifar10"),
    "enhanced_cnn_small": (lambda nc=10: EnhancedCNNSmall(nc), "cifar10"),
    "lenet5": (lambda nc=10: LeNet5(nc), "mnist"),
    "mlp2": (lambda nc=10: mlp2(784, 1024, nc), "mnist"),
    "mlp3": (lambda nc=10: mlp3(784, 4096, nc), "mnist"),
    "mlp3_small": (lambda nc=10: mlp3(784, 1024, nc), "mnist"),
    "resnet18": (lambda nc=1000: resnet18(nc), "imagenet"),
    "resnet18_cifar": (lambda nc=10: resnet18(nc), "cifar10"),
}


def build_model(name: str, num_classes: int | None = None) -> nn.Module:
    ctor, _ = REGISTRY[name]
    return ctor() if num_classes is None else ctor(num_classes)


def dataset_for(name: str) -> str:
    return REGISTRY[name][1]


def xavier_init(model: nn.Module):
    """The reference's init (BAR/main.py:33-37): Xavier-uniform Conv2d/Linear
    weights, zero biases."""
    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.Linear)):
            nn.init.xavier_uniform_(m.weight)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
