"""Process-group bootstrap and device binding (fixes Q7/Q8).

The reference hard-codes MASTER_ADDR=localhost / MASTER_PORT=29500
(BAR/main.py:14-15), initialises the default group from env:// (:19) and puts
every rank on cuda:0 (:25) -- so with nccl on one multi-GPU host all ranks
collide on one device.  Here:

* one process per GPU: ``cuda:{LOCAL_RANK}``; backend "nccl" (= RCCL on ROCm,
  over xGMI inside a node) when GPUs are present, "gloo" on CPU;
* rendezvous from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*),
  defaulting to 127.0.0.1 for single-process runs;
* a collective timeout so a dead rank becomes an exception instead of a hang
  (failure detection).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str | None = None
    initialized_here: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 and dist.is_initialized()


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def setup(backend: str | None = None, timeout_s: float = 600.0, device: str | None = None) -> DistContext:
    """Initialise (if needed) the default process group and bind this rank's device."""
    rank = env_int("RANK", 0)
    world = env_int("WORLD_SIZE", 1)
    local = env_int("LOCAL_RANK", 0)
    ndev = torch.cuda.device_count()
    use_cuda = ndev > 0 and device != "cpu"
    if backend is None:
        backend = os.environ.get("LDNN_BACKEND") or None
    if device is None or device == "auto":
        # one process per GPU; more ranks than GPUs (test oversubscription) wrap around
        dev = torch.device(f"cuda:{local % ndev}") if use_cuda else torch.device("cpu")
    else:
        dev = torch.device(device if device != "cuda" else f"cuda:{local}")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    if backend is None or backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    ctx = DistContext(rank, world, local, dev, backend)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
        ctx.initialized_here = True
    if dist.is_initialized():
        ctx.rank, ctx.world_size = dist.get_rank(), dist.get_world_size()
        ctx.backend = dist.get_backend()
    return ctx


def teardown(ctx: DistContext | None = None):
    if dist.is_initialized() and (ctx is None or ctx.initialized_here):
        dist.destroy_process_group()


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, group=None):
    """Broadcast every state_dict entry from `src` (reference A6, BAR/main.py:40-42):
    parameters AND buffers (BN running stats, num_batches_tracked), coalesced
    into one flat message per dtype instead of 128 separate broadcasts."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    tensors = [t for t in module.state_dict().values() if torch.is_tensor(t)]
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dt, ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off: off + n].view_as(t))
            off += n
