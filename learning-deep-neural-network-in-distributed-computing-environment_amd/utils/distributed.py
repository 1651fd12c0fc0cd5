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


def _first_env(names, default: int) -> int:
    for n in names:
        if n in os.environ:
            return env_int(n, default)
    return default


# Launchers the reference's variants are started with: torchrun (BAR/DAR) and
# `mpirun -np N` (BR/DR/BDR/DDR, BR/main.py:15-17 -- Open MPI, MPICH / Hydra PMI,
# PMIx, Slurm).  No mpi4py: the ranks rendezvous over the c10d TCP store.
_RANK_VARS = ("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK", "SLURM_PROCID")
_SIZE_VARS = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS")
_LOCAL_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID", "PMI_LOCAL_RANK", "SLURM_LOCALID")


def launch_env() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torchrun, mpirun or Slurm environment variables."""
    rank = _first_env(_RANK_VARS, 0)
    world = _first_env(_SIZE_VARS, 1)
    local = _first_env(_LOCAL_VARS, -1)
    if local < 0:
        local = rank  # single node: ranks are local
    return rank, world, local


def setup(backend: str | None = None, timeout_s: float = 600.0, device: str | None = None) -> DistContext:
    """Initialise (if needed) the default process group and bind this rank's device."""
    rank, world, local = launch_env()
    if world > 1:  # env:// rendezvous reads these (mpirun does not set them)
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        os.environ.setdefault("LOCAL_RANK", str(local))
        # a failed / timed-out RCCL collective aborts the communicator and raises in
        # the caller instead of leaving the other ranks hung
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
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
            # RCCL's kernels on a HIGH-priority stream: the compute stream's GEMM / conv grids
            # fill every CU, and a freed CU then goes to the collective's waiting workgroups
            # first instead of the next compute tile (without it a bucket's reduce-scatter
            # waits for the whole overlapping GEMM: profiles/r5/overlap_probe.jsonl)
            if os.environ.get("LDNN_RCCL_HIGH_PRIO", "1") != "0":
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
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
