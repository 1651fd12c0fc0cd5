"""Layer modules whose forward/backward run on the native gfx950 kernels.

They subclass the stock ``torch.nn`` layers, so parameter names, shapes,
``state_dict`` keys and init hooks are exactly those of the reference
(BAR/model.py uses nn.Conv2d / nn.BatchNorm2d / nn.Linear / nn.ReLU); only the
compute path changes.  A layer is bound to the model's FlatParams (bf16
shadow + flat gradient buffer) by ``ldnn.prepare`` / ``FlatParams(model)``.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..ops import functional as LF


class Linear(nn.Linear):
    """nn.Linear with an optional fused activation epilogue ('none'|'relu'|'sigmoid')."""

    def __init__(self, in_features, out_features, bias=True, activation: str = "none", device=None, dtype=None):
        super().__init__(in_features, out_features, bias=bias, device=device, dtype=dtype)
        assert activation in LF.ACTS
        self.activation = activation
        self._ldnn_flat = None

    def forward(self, x):
        return LF.linear_act(x, self.weight, self.bias, self.activation, self._ldnn_flat)

    def extra_repr(self):
        return super().extra_repr() + f", activation={self.activation}"


class ReLU(nn.ReLU):
    def forward(self, x):
        return LF.relu(x)


class Sigmoid(nn.Sigmoid):
    def forward(self, x):
        return LF.sigmoid(x)


class Flatten(nn.Flatten):
    pass


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """Mean cross-entropy (the reference's criterion, BAR/main.py:52) on the fused
    softmax-xent kernel.  Pass ``stats`` to accumulate loss-sum / #correct on device."""

    def forward(self, logits, labels, stats=None):
        return LF.cross_entropy(logits, labels, stats)


class Conv2d(nn.Conv2d):
    """nn.Conv2d (reference key names and init).  On the GPU the activations flow as
    NHWC bf16 through the native implicit-GEMM conv kernels (conv.hip), with the
    weights read from the FlatParams KRSC bf16 shadow; an optional ReLU is fused
    into the conv epilogue."""

    def __init__(self, *args, activation: str = "none", **kwargs):
        super().__init__(*args, **kwargs)
        assert activation in ("none", "relu")
        self.activation = activation
        self._ldnn_flat = None
        self.__dict__["_ldnn_stats_bn"] = None  # (not a submodule: state_dict keys unchanged)

    def forward(self, x):
        return LF.conv2d(x, self, relu=self.activation == "relu",
                         bn=self._ldnn_stats_bn if FUSE_BN_STATS else None)


# Conv-epilogue BatchNorm statistics (pair_conv_bn) are on by default since the
# finalize became parallel (8 accumulator copies summed into LDS, exchanges batched):
# alternated same-box A/B (scripts/ab_cnn.sh, profiles/cnn_fuse_stats_tapmajor_ab_r2.jsonl)
# with the tap-major conv K order: ResNet-18 b64 3.89 -> 3.82 ms, EnhancedCNN b64
# 2.45 -> 2.42 ms.  (Round 1, with a serial finalize, it lost: 3.80 vs 3.67 ms.)
# LDNN_FUSE_BN_STATS=0 turns it off.
FUSE_BN_STATS = os.environ.get("LDNN_FUSE_BN_STATS", "1") == "1"


def pair_conv_bn(conv: "Conv2d", bn: "BatchNorm2d") -> None:
    """Declare that `bn` consumes exactly `conv`'s output: in training mode the conv
    kernel's epilogue then accumulates and finalizes the BN's batch statistics
    (ldnn_conv_lds.h bn_stats_epilogue) and the BN runs only its apply pass.  Only for
    architectures where that dataflow is fixed (the BN also checks it is handed the
    very buffer the conv wrote before it trusts the statistics)."""
    conv.__dict__["_ldnn_stats_bn"] = bn


class BatchNorm2d(nn.BatchNorm2d):
    """Train-mode batch statistics + running-stat EMA exactly as nn.BatchNorm2d;
    on the GPU fp32 statistics over NHWC bf16 activations in the native kernels,
    with optional residual-add + ReLU fused into the same pass (``act``)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._ldnn_flat = None

    def forward(self, x):
        return LF.batch_norm_act(x, self)

    def act(self, x, residual=None, relu: bool = False):
        """relu?(bn(x) + residual) in one fused pass."""
        return LF.batch_norm_act(x, self, residual, relu)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        return LF.pool2d(x, self, True)


class AvgPool2d(nn.AvgPool2d):
    def forward(self, x):
        return LF.pool2d(x, self, False)


class AdaptiveAvgPool2d(nn.AdaptiveAvgPool2d):
    def forward(self, x):
        return LF.adaptive_avg_pool2d(x, self.output_size)
