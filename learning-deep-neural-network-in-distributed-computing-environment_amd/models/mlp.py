"""Multi-layer perceptrons of the BASELINE.json configs.

* ``mlp2``: 2-layer MLP on MNIST-shaped input (config #1, CPU plumbing).
* ``mlp3``: the flagship 3-layer MLP 784-4096-4096-10 (configs #2/#3), whose
  training step the static engine (train/static_mlp.py) runs on the native
  MFMA kernels with graph capture and overlapped RCCL gradient all-reduce.

Activations are fused into the Linear GEMM epilogue (ReLU or sigmoid, the
two activations BASELINE.json names).
"""
from __future__ import annotations

import torch.nn as nn

from .layers import Linear


class MLP(nn.Module):
    def __init__(self, in_features: int = 784, hidden=(4096, 4096), num_classes: int = 10,
                 activation: str = "relu"):
        super().__init__()
        dims = [in_features, *hidden, num_classes]
        self.in_features = in_features
        self.num_classes = num_classes
        self.activation = activation
        self.layers = nn.ModuleList(
            Linear(dims[i], dims[i + 1], activation=activation if i < len(dims) - 2 else "none")
            for i in range(len(dims) - 1)
        )

    def forward(self, x):
        x = x.flatten(1)
        for layer in self.layers:
            x = layer(x)
        return x


def mlp2(in_features=784, hidden=1024, num_classes=10, activation="relu"):
    return MLP(in_features, (hidden,), num_classes, activation)


def mlp3(in_features=784, hidden=4096, num_classes=10, activation="relu"):
    return MLP(in_features, (hidden, hidden), num_classes, activation)
