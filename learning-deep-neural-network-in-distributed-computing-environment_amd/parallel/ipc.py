"""One-shot intra-node all-reduce over IPC-mapped peer buffers (the
small-message path "that reads from all 7 peers").

RCCL's ring / tree all-reduce pays N-1 dependent link hops; inside one MI355X
node every GPU has its own xGMI link to each peer, so for small messages (metric
vectors, the schedule digest, small gradient buckets, the MLP configs' gradients)
one kernel that reads every peer's copy at once over all links is latency-optimal.
The native side (``csrc/kernels/ipc.hip``, ``OneShotComm`` in the bindings) owns
this rank's staging and signal regions; their IPC handles are exchanged once
through the process group, after which a call is one stream-ordered device copy
plus one kernel with a single cross-rank barrier -- no host synchronisation.

Requirements: every rank of the group on one node, one GPU per rank (a rank may
map a peer on the same device too: that is how the one-GPU test box runs it),
fp32 or bf16 tensors with numel % 8 == 0.  Anything else falls back to the
process group's all-reduce.  Every wait in the kernel has a 5 s wall-clock limit;
``check()`` raises if a peer never arrived.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _ext


class OneShotAllReduce:
    def __init__(self, max_bytes: int = 4 << 20, group=None, device: torch.device | None = None, blocks: int = 64):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.max_bytes = int(max_bytes)
        self._c = _ext.C().OneShotComm(self.rank, self.world_size, self.max_bytes, device.index, blocks)
        mine = tuple(bytes(h) for h in self._c.handles())
        allh: list = [None] * self.world_size
        dist.all_gather_object(allh, mine, group=group)  # the one host exchange: IPC handles
        self._c.connect([(a, b) for a, b in allh])
        dist.barrier(group=group)  # every rank mapped every peer before the first kernel

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.device and t.is_contiguous()
                and t.dtype in (torch.float32, torch.bfloat16) and t.numel() % 8 == 0
                and t.numel() * t.element_size() <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor) -> None:
        """In-place sum over the group's ranks, ordered on the current stream."""
        self._c.all_reduce(t)

    def check(self) -> None:
        if self._c.error():
            raise RuntimeError("one-shot all-reduce: a peer rank never reached the barrier (5 s limit)")
