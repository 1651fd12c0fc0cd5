"""ldnn — an MI355X-native (gfx950 / CDNA4) distributed DNN training framework.

Capabilities mirror Sanasar1/Learning-Deep-Neural-Network-In-Distributed-Computing-Environment
(see SURVEY.md): a global/local-epoch training driver with the reference's
flags and 12 metric histories, data-parallel aggregation by all-reduce,
model averaging and ring / double-ring gossip (equal or self-weighted, on
gradients or weights), IID / class-skewed / speed-proportional sharding,
validation, test evaluation with precision/recall/F1, plots, plus what the
reference lacks: per-step bucketed all-reduce on RCCL overlapped with the
backward pass, hand-written bf16 MFMA kernels, checkpoint/resume, straggler
cutoff and failure detection.
"""
__version__ = "0.1.0"

from . import ops  # noqa: F401  (loads the native extension, loudly on GPU boxes)


def prepare(model, device=None):
    """Move `model` to `device` and lay its parameters out in one FlatParams buffer
    (fp32 master + flat grads + bf16 shadow on the GPU).  Returns the FlatParams."""
    import torch

    from .parallel.ddp import ensure_flat

    if device is not None:
        model.to(torch.device(device))
    return ensure_flat(model, device)
