"""Plain torch.nn fp32 oracles with the same state_dict keys as ldnn's CNNs.

They contain no ldnn layer, so a model-level numerics check compares ldnn's bf16
native path against stock fp32 PyTorch (kernel-unit row): load the
ldnn model's state_dict, run the same (bf16-rounded) input in fp32, compare grads.
Architectures: torchvision-layout ResNet-18 (models/resnet.py) and the reference's
EnhancedCNNModel (Balanced All-Reduce/model.py:52-111)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class RefBasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + (x if self.downsample is None else self.downsample(x)))


class RefResNet18(nn.Module):
    def __init__(self, num_classes=1000, width=64):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        c = width
        for i, w in enumerate((width, width * 2, width * 4, width * 8)):
            s = 1 if i == 0 else 2
            setattr(self, f"layer{i + 1}", nn.Sequential(RefBasicBlock(c, w, s), RefBasicBlock(w, w, 1)))
            c = w
        self.fc = nn.Linear(c, num_classes)

    def stem(self, x):
        return self.maxpool(F.relu(self.bn1(self.conv1(x))))

    def trunk(self, x):
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(x.mean((2, 3)))

    def forward(self, x):
        return self.trunk(self.stem(x))


class RefResBlock(nn.Module):
    """BAR/model.py:52-72 (shortcut keys: shortcut.0 / shortcut.1)."""

    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = nn.Sequential()
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(out)) + self.shortcut(x))


class RefEnhancedCNN(nn.Module):
    def __init__(self, num_classes=10):
        super().__init__()
        self.prep = nn.Sequential(nn.Conv2d(3, 64, 3, 1, 1, bias=False), nn.BatchNorm2d(64), nn.ReLU())
        c = 64
        for i, w in enumerate((128, 256, 512, 1024)):
            setattr(self, f"layer{i + 1}", nn.Sequential(RefResBlock(c, w, 2), RefResBlock(w, w, 1)))
            c = w
        self.fc = nn.Linear(1024, num_classes)

    def forward(self, x):
        x = self.layer4(self.layer3(self.layer2(self.layer1(self.prep(x)))))
        return self.fc(x.mean((2, 3)))


def oracle_for(name: str, state_dict, device="cuda"):
    """fp32 torch.nn twin of ldnn's `name` model loaded with `state_dict`."""
    ref = {"resnet18": RefResNet18, "enhanced_cnn": RefEnhancedCNN}[name]()
    sd = {k: v.detach().float() if v.is_floating_point() else v for k, v in state_dict.items()}
    ref.load_state_dict(sd)
    return ref.to(device).float()


def rel(a, b):
    """||a - b|| / ||b|| in float64."""
    a, b = a.detach().double().flatten(), b.detach().double().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def bf16_grad_tol(depth: int, k: float = 2.0) -> float:
    """Relative-error budget for a gradient that passed through `depth` bf16 layers:
    each bf16 rounding contributes ~2^-9 relative error, random-walk accumulated
    (sqrt(depth)), times k for reductions that amplify it."""
    return k * (2.0 ** -8) * max(1.0, depth) ** 0.5
