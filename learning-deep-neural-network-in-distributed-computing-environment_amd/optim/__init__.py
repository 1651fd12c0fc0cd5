"""Fused optimizers and LR schedules (StepLR is torch's, as in BAR/main.py:54)."""
from torch.optim.lr_scheduler import StepLR  # noqa: F401

from .optimizers import SGD, Adam, AdamW, build_optimizer  # noqa: F401
