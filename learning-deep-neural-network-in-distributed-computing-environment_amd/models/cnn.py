"""CNN model families of the reference and of the BASELINE.json configs.

* ``EnhancedCNNModel`` -- the reference's CIFAR ResNet-style network
  (BAR/model.py:74-111): prep conv3x3 3->64 + BN + ReLU, four stages of two
  ``ResBlock``s (64->128->256->512->1024, first block stride 2), global average
  pool, fc 1024->10.  44,595,786 parameters; state_dict keys identical to the
  reference (prep.0.weight, layer1.0.conv1.weight, ..., fc.bias).
* ``EnhancedCNNSmall`` -- the commented-out three-stage variant
  (BAR/model.py:4-50): 4,829,258 parameters.
* ``LeNet5`` -- BASELINE.json config #4 (28x28 input).
"""
from __future__ import annotations

import torch.nn as nn

from ..ops import functional as LF
from .layers import AdaptiveAvgPool2d, AvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, pair_conv_bn


class ConvBNReLU(nn.Sequential):
    """Sequential(conv, bn, relu) -- same state_dict keys (prep.0 / prep.1) -- whose
    BN and ReLU run as one fused pass."""

    def __init__(self, *mods):
        super().__init__(*mods)
        pair_conv_bn(self[0], self[1])

    def forward(self, x):
        return self[1].act(self[0](x), relu=True)


class ResBlock(nn.Module):
    """conv3x3(stride)-BN-ReLU-conv3x3-BN + shortcut (1x1 conv + BN when the shape
    changes) -> add -> ReLU; convs without bias (BAR/model.py:52-72)."""

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_channels, out_channels, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNorm2d(out_channels)
        self.conv2 = Conv2d(out_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = BatchNorm2d(out_channels)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_channels != out_channels:
            self.shortcut = nn.Sequential(
                Conv2d(in_channels, out_channels, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(out_channels),
            )
        self.relu = ReLU()
        pair_conv_bn(self.conv1, self.bn1)
        pair_conv_bn(self.conv2, self.bn2)
        if len(self.shortcut):
            pair_conv_bn(self.shortcut[0], self.shortcut[1])

    def forward(self, x):
        # BAR/model.py:67-72 with BN+ReLU and BN+residual-add+ReLU each fused into one pass;
        # the shortcut reads x's twin (LF.shortcut_input), so the producer of x sums the two
        # branch gradients in its own backward kernels instead of a separate add
        if len(self.shortcut):
            # the 3x3 and the 1x1 shortcut conv of x in one launch, then conv2 and both BNs, the add
            # and the ReLU in one pass
            c1, sc = LF.conv2d_pair(x, LF.shortcut_input(x), self.conv1, self.shortcut[0])
            out = self.bn1.act(c1, relu=True)
            return LF.batch_norm_dual_act(self.conv2(out), self.bn2, sc, self.shortcut[1])
        out = self.bn1.act(self.conv1(x), relu=True)
        return self.bn2.act(self.conv2(out), residual=LF.shortcut_input(x), relu=True)


class EnhancedCNNModel(nn.Module):
    def __init__(self, num_classes: int = 10, in_channels: int = 3):
        super().__init__()
        self.prep = ConvBNReLU(
            Conv2d(in_channels, 64, kernel_size=3, stride=1, padding=1, bias=False),
            BatchNorm2d(64),
            ReLU(),
        )
        self.layer1 = nn.Sequential(ResBlock(64, 128, stride=2), ResBlock(128, 128, stride=1))
        self.layer2 = nn.Sequential(ResBlock(128, 256, stride=2), ResBlock(256, 256, stride=1))
        self.layer3 = nn.Sequential(ResBlock(256, 512, stride=2), ResBlock(512, 512, stride=1))
        self.layer4 = nn.Sequential(ResBlock(512, 1024, stride=2), ResBlock(1024, 1024, stride=1))
        self.pool = AdaptiveAvgPool2d(1)
        self.fc = Linear(1024, num_classes)

    def forward(self, x):
        x = self.prep(x)
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return LF.gap_linear(x, self.pool, self.fc)   # pool -> view -> fc (one fused launch each way on the GPU)


class EnhancedCNNSmall(nn.Module):
    """The reference's commented-out smaller model (BAR/model.py:4-50)."""

    def __init__(self, num_classes: int = 10, in_channels: int = 3):
        super().__init__()
        self.prep = ConvBNReLU(
            Conv2d(in_channels, 64, kernel_size=3, stride=1, padding=1, bias=False),
            BatchNorm2d(64),
            ReLU(),
        )
        self.layer1 = ResBlock(64, 128, stride=2)
        self.layer2 = ResBlock(128, 256, stride=2)
        self.layer3 = ResBlock(256, 512, stride=2)
        self.pool = AdaptiveAvgPool2d(1)
        self.fc = Linear(512, num_classes)

    def forward(self, x):
        x = self.prep(x)
        x = self.layer3(self.layer2(self.layer1(x)))
        return LF.gap_linear(x, self.pool, self.fc)


class LeNet5(nn.Module):
    """LeNet-5 for 28x28 (MNIST-shaped) input: conv5x5(pad 2)-ReLU-pool, conv5x5-ReLU-pool,
    fc 400-120-84-10 (ReLU activations fused into the Linear epilogues)."""

    def __init__(self, num_classes: int = 10, in_channels: int = 1, pool: str = "max"):
        super().__init__()
        P = MaxPool2d if pool == "max" else AvgPool2d
        self.features = nn.Sequential(
            Conv2d(in_channels, 6, kernel_size=5, padding=2, activation="relu"), ReLU(), P(2),
            Conv2d(6, 16, kernel_size=5, activation="relu"), ReLU(), P(2),
        )
        # the ReLUs are fused into the conv epilogues; the modules stay for the reference layout
        self.features[1] = nn.Identity()
        self.features[4] = nn.Identity()
        self.features[5].flatten_out = True   # native pool writes NCHW: the flatten below is a view
        self.fc1 = Linear(16 * 5 * 5, 120, activation="relu")
        self.fc2 = Linear(120, 84, activation="relu")
        self.fc3 = Linear(84, num_classes)

    def forward(self, x):
        x = self.features(x)
        x = x.flatten(1)
        return self.fc3(self.fc2(self.fc1(x)))
