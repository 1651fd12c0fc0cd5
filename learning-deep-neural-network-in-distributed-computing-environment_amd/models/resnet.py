"""ResNet-18 for 224x224 input (BASELINE.json config #5), torchvision layout and
state_dict keys (conv1, bn1, layer{1..4}.{0,1}.conv{1,2}/bn{1,2},
layer{2..4}.0.downsample.{0,1}, fc): 7x7/2 stem, 3x3/2 max-pool, four stages
of two BasicBlocks (64, 128, 256, 512), global average pool, fc 512->classes."""
from __future__ import annotations

import torch.nn as nn

from ..ops import functional as LF
from .layers import AdaptiveAvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, pair_conv_bn


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.relu = ReLU()
        self.conv2 = Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        pair_conv_bn(self.conv1, self.bn1)
        pair_conv_bn(self.conv2, self.bn2)
        if downsample is not None:
            pair_conv_bn(downsample[0], downsample[1])

    def forward(self, x):
        xs = LF.shortcut_input(x)   # (x's twin: see models/cnn.py ResBlock)
        if self.downsample is not None:
            # conv1 and the 1x1 shortcut conv of x in one launch; conv2's BN, the shortcut BN, the add
            # and the ReLU in one pass
            c1, sc = LF.conv2d_pair(x, xs, self.conv1, self.downsample[0])
            out = self.bn1.act(c1, relu=True)
            return LF.batch_norm_dual_act(self.conv2(out), self.bn2, sc, self.downsample[1])
        out = self.bn1.act(self.conv1(x), relu=True)
        return self.bn2.act(self.conv2(out), residual=xs, relu=True)


class ResNet(nn.Module):
    def __init__(self, layers=(2, 2, 2, 2), num_classes=1000, in_channels=3, width=64):
        super().__init__()
        self.inplanes = width
        self.conv1 = Conv2d(in_channels, width, 7, 2, 3, bias=False)
        self.bn1 = BatchNorm2d(width)
        self.relu = ReLU()
        self.maxpool = MaxPool2d(3, 2, 1)
        pair_conv_bn(self.conv1, self.bn1)
        self.layer1 = self._make(width, layers[0], 1)
        self.layer2 = self._make(width * 2, layers[1], 2)
        self.layer3 = self._make(width * 4, layers[2], 2)
        self.layer4 = self._make(width * 8, layers[3], 2)
        self.avgpool = AdaptiveAvgPool2d(1)
        self.fc = Linear(width * 8, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def _make(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes:
            down = nn.Sequential(Conv2d(self.inplanes, planes, 1, stride, bias=False), BatchNorm2d(planes))
        layers = [BasicBlock(self.inplanes, planes, stride, down)]
        self.inplanes = planes
        layers += [BasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = LF.bn_relu_maxpool(self.conv1(x), self.bn1, self.maxpool)   # maxpool(relu(bn1(conv1 x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = self.avgpool(x).flatten(1)
        return self.fc(x)


def resnet18(num_classes=1000, in_channels=3):
    return ResNet((2, 2, 2, 2), num_classes, in_channels)
