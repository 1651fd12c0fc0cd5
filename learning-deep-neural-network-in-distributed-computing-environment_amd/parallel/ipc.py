"""One-shot intra-node all-reduce over IPC-mapped peer buffers (the
small-message path "that reads from all 7 peers").

RCCL's ring / tree all-reduce pays N-1 dependent link hops; inside one MI355X
node every GPU has its own xGMI link to each peer, so for small messages (metric
vectors, the schedule digest, small gradient buckets, the MLP configs' gradients)
one kernel that reads every peer's copy at once over all links is latency-optimal.
The native side (``csrc/kernels/ipc.hip``, ``OneShotComm`` in the bindings) owns
this rank's staging, signal and per-block epoch-counter regions; their IPC handles
are exchanged once through the process group, after which a call is ONE
stream-ordered kernel (stage, one cross-rank barrier, sum) -- no host
synchronisation, and no host-side call number in its arguments, so a call
captured into a hipGraph is a correct call on every replay.

Requirements: every rank of the group on one node, one GPU per rank (a rank may
map a peer on the same device too: that is how the one-GPU test box runs it),
fp32 or bf16 tensors with numel % 8 == 0.  Anything else falls back to the
process group's all-reduce.  Every wait in the kernel has a 5 s wall-clock limit;
a timed-out call sets a sticky error word and leaves its tensor (and every later
call's) unsummed: ``check()`` raises then, and ``Comm.check_schedule`` -- run every
global epoch and every few hundred per-step-DP steps -- gathers every rank's flag and
raises on all of them.  Because of that limit the path is opt-in for training
(``default_comm``), on for lock-step loops such as bench.py.

``self_test()`` (run when the communicator is enabled) sums a rank-dependent
vector through the kernel and compares with the process group's all-reduce; any
mismatch or timeout on any rank disables the path on every rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _ext


class OneShotAllReduce:
    def __init__(self, max_bytes: int = 4 << 20, group=None, device: torch.device | None = None, blocks: int = 64):
        """Collective.  Every rank runs the same collective sequence whatever fails
        locally (allocation, IPC export / import): one all_gather_object + one barrier
        here, then self_test()'s three all-reduces -- a rank whose setup failed takes
        part with ok = False and the path is then off on every rank."""
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.max_bytes = int(max_bytes)
        self.connect_error = None
        self._c, mine = None, None
        try:
            self._c = _ext.C().OneShotComm(self.rank, self.world_size, self.max_bytes, device.index, blocks)
            mine = tuple(bytes(h) for h in self._c.handles())
        except Exception as e:  # noqa: BLE001 -- reported by self_test on every rank
            self.connect_error = e
        allh: list = [None] * self.world_size
        dist.all_gather_object(allh, mine, group=group)  # the one host exchange: IPC handles
        if self.connect_error is None and any(h is None for h in allh):
            self.connect_error = RuntimeError("a peer rank could not export its IPC buffers")
        if self.connect_error is None:
            try:
                self._c.connect([(a, b) for a, b in allh])
            except Exception as e:  # noqa: BLE001
                self.connect_error = e
        dist.barrier(group=group)  # every rank mapped every peer before the first kernel

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.device and t.is_contiguous()
                and t.dtype in (torch.float32, torch.bfloat16) and t.numel() % 8 == 0
                and t.numel() * t.element_size() <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor) -> None:
        """In-place sum over the group's ranks, ordered on the current stream."""
        self._c.all_reduce(t)

    def error(self) -> str | None:
        if self._c is not None and self._c.error():
            return ("one-shot all-reduce: a peer rank never reached the barrier (5 s limit); the tensors of "
                    "that call and of every later one-shot call were left unsummed")
        return None

    def check(self) -> None:
        err = self.error()
        if err:
            raise RuntimeError(err)

    def self_test(self) -> bool:
        """Collective: True on every rank iff the kernel summed correctly on every rank."""
        ok = self._agree(self.connect_error is None)   # no kernel waits on a peer that failed to map
        for dt in (torch.float32, torch.bfloat16):
            n = 4096
            t = (torch.arange(n, device=self.device, dtype=torch.float32) % 7 + self.rank + 1).to(dt)
            ref = t.float().clone()
            dist.all_reduce(ref, group=self.group)
            for _ in range(3 if ok else 0):   # consecutive calls: both staging halves, epoch counters advance
                u = t.clone()
                self.all_reduce(u)
                torch.cuda.synchronize(self.device)
                ok = ok and not self._c.error() and torch.allclose(u.float(), ref, rtol=1e-2 if dt != torch.float32 else 0)
        return self._agree(ok)

    def _agree(self, ok: bool) -> bool:
        flag = torch.tensor([1.0 if ok else 0.0], device=self.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        return bool(flag.item() == 1.0)
