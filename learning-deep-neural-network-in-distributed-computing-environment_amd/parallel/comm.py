"""Communicator abstraction over the collectives the reference uses.

The reference talks to two backends: torch.distributed (gloo/nccl; AR
variants) and mpi4py with host-staged numpy buffers (ring variants,
BR/communication.py:1-30).  Here one interface serves every topology:

* ``TorchComm``  -- torch.distributed on the default (or a given) group.  With
  backend "nccl" this is RCCL over xGMI inside an MI355X node: device buffers
  are sent directly (no host staging), point-to-point gossip uses grouped
  ``batch_isend_irecv`` (one ncclGroupStart/End) so the ring and double-ring
  exchanges use distinct xGMI links concurrently.
* ``FakeWorld`` / ``FakeComm`` -- an in-process world of N ranks run as
  threads, used by the tests to check aggregation formulas and whole training
  loops deterministically without any process group (SURVEY §4 "FakeGroup").

Every collective the training driver issues goes through ``Comm.record`` so a
schedule checker can hash the op sequence and detect rank divergence.
"""
from __future__ import annotations

import hashlib
import os
import threading

import torch
import torch.distributed as dist

SUM, MAX, MIN = "sum", "max", "min"


class RankDivergenceError(RuntimeError):
    """The ranks issued different collective sequences (different op counts / kinds /
    shapes).  Raised by Comm.check_schedule instead of letting a mismatched collective
    hang until the process-group timeout."""
_TORCH_OPS = {SUM: dist.ReduceOp.SUM, MAX: dist.ReduceOp.MAX, MIN: dist.ReduceOp.MIN}


class Comm:
    rank: int = 0
    world_size: int = 1
    # True when collectives run on device buffers ordered by HIP streams (RCCL):
    # they may then be issued from a side stream behind in-graph events
    device_collectives: bool = False

    def __init__(self):
        self._sched = hashlib.sha1()
        self._nops = 0

    # -- schedule bookkeeping (race / divergence detection)
    def record(self, op: str, t: torch.Tensor | None = None):
        desc = op if t is None else f"{op}:{tuple(t.shape)}:{t.dtype}"
        self._sched.update(desc.encode())
        self._nops += 1

    def schedule_digest(self) -> tuple[int, str]:
        return self._nops, self._sched.hexdigest()

    def check_schedule(self, where: str = "", device=None):
        """Cross-check every rank's collective schedule (op count + running hash of
        op / shape / dtype) AND every rank's device-side error flag (one-shot IPC
        timeout) with one small all-gather; raise on EVERY rank at the same point:
        RankDivergenceError on the first schedule mismatch, RuntimeError if any rank
        recorded a collective failure.  The error is usually set on the rank(s) that
        timed out only, so a local check would leave the others waiting in the next
        collective.  The training driver calls it once per global epoch and every
        ``check_every`` steps of per-step synchronisation -- the class of bug the
        reference's dead time-limit break would cause."""
        if self.world_size <= 1:
            return
        n, h = self.schedule_digest()
        err = self.local_error()
        v = torch.tensor([n, int(h[:15], 16), 1 if err else 0], dtype=torch.int64,
                         device=device if device is not None else "cpu")
        got = [t.cpu() for t in self.all_gather(v)]
        bad = [r for r, g in enumerate(got) if int(g[2]) != 0]
        if bad:
            raise RuntimeError(f"collective failure on rank(s) {bad}{' at ' + where if where else ''}"
                               f"{': ' + err if err else ''}")
        if any(not torch.equal(got[0][:2], g[:2]) for g in got):
            desc = ", ".join(f"rank {r}: {int(g[0])} ops #{int(g[1]):015x}" for r, g in enumerate(got))
            raise RankDivergenceError(f"collective schedules diverged{' at ' + where if where else ''}: {desc}")

    def local_error(self) -> str | None:
        """Description of a failure a device-side collective path recorded on THIS rank
        (one-shot IPC timeout), else None.  Never raises, never communicates."""
        return None

    def check_errors(self):
        """Raise (locally) if this rank's device-side collective path recorded a failure."""
        err = self.local_error()
        if err:
            raise RuntimeError(err)

    # -- API (implemented by subclasses)
    def all_reduce(self, t: torch.Tensor, op: str = SUM, async_op: bool = False):
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int = 0):
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> list[torch.Tensor]:
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def sendrecv(self, sends: list[tuple[torch.Tensor, int]], recvs: list[tuple[torch.Tensor, int]],
                 async_op: bool = False):
        """Grouped point-to-point: post every send and receive, wait for all.  ``async_op``:
        return a handle whose ``wait()`` orders the current stream after them (RCCL) --
        the sends' buffers must not change before it."""
        raise NotImplementedError

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """SUM-reduce ``inp`` (world_size * out.numel() elements) over the ranks; rank r
        receives slice r into ``out``.  ``inp`` may be clobbered."""
        raise NotImplementedError

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        """``out`` (world_size * inp.numel() elements) <- every rank's ``inp``, in rank order.
        ``inp`` may be ``out``'s own slot (in place)."""
        raise NotImplementedError


class _Done:
    def wait(self):
        return None


class _Works:
    """Several in-flight c10d works behind one ``wait()`` (a grouped send/recv)."""

    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        for w in self.works:
            w.wait()


class LocalComm(Comm):
    """World of one: every collective is the identity."""

    def all_reduce(self, t, op=SUM, async_op=False):
        self.record("all_reduce", t)
        return _Done() if async_op else None

    def broadcast(self, t, src=0):
        self.record("broadcast", t)

    def all_gather(self, t):
        self.record("all_gather", t)
        return [t.clone()]

    def barrier(self):
        self.record("barrier")

    def sendrecv(self, sends, recvs, async_op=False):
        self.record("sendrecv")
        for (rt, src), (st, dst) in zip(recvs, sends):
            rt.copy_(st)
        return _Done() if async_op else None

    def reduce_scatter(self, out, inp, async_op=False):
        self.record("reduce_scatter", inp)
        out.copy_(inp)
        return _Done() if async_op else None

    def all_gather_into(self, out, inp, async_op=False):
        self.record("all_gather_into", out)
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)
        return _Done() if async_op else None


class TorchComm(Comm):
    def __init__(self, group=None):
        super().__init__()
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device_collectives = self.backend == "nccl"

    def _global(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def enable_oneshot(self, max_bytes: int, device=None, self_test: bool = True):
        """Route SUM all-reduces of at most ``max_bytes`` (fp32 / bf16 device tensors)
        through the one-shot IPC path (parallel/ipc.py).  Collective: every rank calls it
        and every rank reaches the same decision (the path is on everywhere or nowhere:
        a rank routing a bucket through IPC while a peer uses RCCL would hang).  With
        ``self_test`` the path is verified against RCCL first and left off (on every
        rank, with a warning) if it fails anywhere -- e.g. a node whose GPUs cannot map
        each other's memory.  Only for groups inside one node (IPC handles do not cross
        hosts): a multi-node world leaves it off without any setup."""
        from .ipc import OneShotAllReduce

        if not single_node():
            return None
        os_ = OneShotAllReduce(max_bytes, group=self.group, device=device)   # never raises; collective
        ok = os_.self_test() if self_test else os_._agree(os_.connect_error is None)
        if not ok:
            import warnings

            warnings.warn(f"one-shot IPC all-reduce unavailable or failed its self-test on some rank "
                          f"({os_.connect_error!r} here); using RCCL for every message")
            return None
        self.oneshot = os_
        return os_

    oneshot = None

    def local_error(self):
        if self.oneshot is not None:
            return self.oneshot.error()
        return None

    def all_reduce(self, t, op=SUM, async_op=False):
        self.record("all_reduce", t)
        if op == SUM and self.oneshot is not None and self.oneshot.eligible(t):
            self.oneshot.all_reduce(t)  # stream-ordered: nothing to wait for on the host
            return _Done() if async_op else None
        return dist.all_reduce(t, op=_TORCH_OPS[op], group=self.group, async_op=async_op)

    def broadcast(self, t, src=0):
        self.record("broadcast", t)
        dist.broadcast(t, src=self._global(src), group=self.group)

    def all_gather(self, t):
        self.record("all_gather", t)
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return out

    def barrier(self):
        self.record("barrier")
        if dist.get_backend(self.group) == "nccl" and torch.cuda.is_available():
            dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=self.group)

    def sendrecv(self, sends, recvs, async_op=False):
        self.record("sendrecv")
        # gloo moves GPU tensors point-to-point through a slow per-op path (measured: a
        # 178 MB ring exchange ~10 s vs 0.1 s for the same bytes from host memory), so the
        # plumbing backend stages them through host buffers; RCCL sends device-direct
        stage = self.backend == "gloo" and any(t.is_cuda for t, _ in list(sends) + list(recvs))
        if stage:
            sends = [(t.detach().cpu(), dst) for t, dst in sends]
            dev_recvs, recvs = recvs, [(torch.empty(t.shape, dtype=t.dtype), src) for t, src in recvs]
        ops = [dist.P2POp(dist.irecv, t, self._global(src), self.group) for t, src in recvs]
        ops += [dist.P2POp(dist.isend, t, self._global(dst), self.group) for t, dst in sends]
        works = dist.batch_isend_irecv(ops)
        if async_op and not stage:
            return _Works(works)   # RCCL: wait() = stream waits, no host sync
        for w in works:
            w.wait()
        if stage:
            for (t, _), (c, _) in zip(dev_recvs, recvs):
                t.copy_(c)
        return _Done() if async_op else None

    def reduce_scatter(self, out, inp, async_op=False):
        self.record("reduce_scatter", inp)
        if self.backend == "nccl":
            return dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)
        # gloo has no reduce-scatter of device tensors: all-reduce, keep this rank's slice
        dist.all_reduce(inp, group=self.group)
        n = out.numel()
        out.copy_(inp[self.rank * n: (self.rank + 1) * n])
        return _Done() if async_op else None

    def all_gather_into(self, out, inp, async_op=False):
        self.record("all_gather_into", out)
        if self.backend == "nccl":   # in place when inp is out's slot r (the RCCL convention)
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)
        src = inp.clone()
        dist.all_gather(list(out.chunk(self.world_size)), src, group=self.group)
        return _Done() if async_op else None


# ------------------------------------------------------------------ fake world
class FakeWorld:
    """N ranks as threads of one process; collectives meet at a barrier."""

    def __init__(self, n: int, timeout: float = 60.0):
        self.n = n
        self._bar = threading.Barrier(n, timeout=timeout)
        self._slots: list = [None] * n
        self._p2p: dict = {}
        self._lock = threading.Lock()

    def comm(self, rank: int) -> "FakeComm":
        return FakeComm(self, rank)

    def run(self, fn, *args, **kwargs) -> list:
        """Run fn(comm, *args) on every rank; return per-rank results (re-raises errors)."""
        results: list = [None] * self.n
        errors: list = []

        def body(r):
            try:
                results[r] = fn(self.comm(r), *args, **kwargs)
            except BaseException as e:  # pragma: no cover - surfaced below
                errors.append(e)
                self._bar.abort()

        ts = [threading.Thread(target=body, args=(r,)) for r in range(self.n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errors:
            raise errors[0]
        return results


class FakeComm(Comm):
    def __init__(self, world: FakeWorld, rank: int):
        super().__init__()
        self.w = world
        self.rank = rank
        self.world_size = world.n

    def _exchange(self, value):
        w = self.w
        w._slots[self.rank] = value
        w._bar.wait()
        vals = list(w._slots)
        w._bar.wait()
        return vals

    def all_reduce(self, t, op=SUM, async_op=False):
        self.record("all_reduce", t)
        vals = self._exchange(t.detach().clone())
        if op == SUM:
            res = torch.stack(vals).sum(0)
        elif op == MAX:
            res = torch.stack(vals).amax(0)
        else:
            res = torch.stack(vals).amin(0)
        t.copy_(res.to(t.dtype))
        return _Done() if async_op else None

    def broadcast(self, t, src=0):
        self.record("broadcast", t)
        vals = self._exchange(t.detach().clone())
        t.copy_(vals[src])

    def all_gather(self, t):
        self.record("all_gather", t)
        return [v.clone() for v in self._exchange(t.detach().clone())]

    def barrier(self):
        self.record("barrier")
        self._exchange(None)

    def sendrecv(self, sends, recvs, async_op=False):
        self.record("sendrecv")
        msgs = {(self.rank, dst): st.detach().clone() for st, dst in sends}
        allm = self._exchange(msgs)
        merged = {}
        for m in allm:
            merged.update(m)
        for rt, src in recvs:
            rt.copy_(merged[(src, self.rank)])
        return _Done() if async_op else None

    def reduce_scatter(self, out, inp, async_op=False):
        self.record("reduce_scatter", inp)
        tot = torch.stack(self._exchange(inp.detach().clone())).sum(0)
        n = out.numel()
        out.copy_(tot[self.rank * n: (self.rank + 1) * n].to(out.dtype))
        return _Done() if async_op else None

    def all_gather_into(self, out, inp, async_op=False):
        self.record("all_gather_into", out)
        vals = self._exchange(inp.detach().clone())
        out.copy_(torch.cat(vals).to(out.dtype))
        return _Done() if async_op else None


ONESHOT_DEFAULT_BYTES = 4 << 20


def single_node() -> bool:
    """Every rank of the default world on this host (torchrun / mpirun local-size env)."""
    world = os.environ.get("WORLD_SIZE") or os.environ.get("OMPI_COMM_WORLD_SIZE") or os.environ.get("PMI_SIZE")
    local = (os.environ.get("LOCAL_WORLD_SIZE") or os.environ.get("OMPI_COMM_WORLD_LOCAL_SIZE")
             or os.environ.get("MPI_LOCALNRANKS"))
    if world is None or local is None:
        return False
    return int(local) == int(world)


def default_comm(oneshot_bytes: int | None = None) -> Comm:
    """TorchComm over the default group (LocalComm for a world of one).  With RCCL on
    one node, SUM all-reduces of at most ``oneshot_bytes`` use the one-shot IPC kernel
    that reads every peer's copy over its own xGMI link (SURVEY §5 small-message path:
    metric vectors, small gradient buckets such as LeNet-5's whole 0.25 MB gradient).
    Opt-in (default 0 = off, env LDNN_ONESHOT_BYTES): its device-side barrier gives up
    after a fixed wall-clock limit, so ranks skewed by more than that (a rank-0
    checkpoint write, unequal validation shards) would fail the call where RCCL just
    waits; lock-step loops (bench.py, per-step DP) turn it on.  Collective: every rank
    must pass the same value."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        c = TorchComm()
        if oneshot_bytes is None:
            oneshot_bytes = int(os.environ.get("LDNN_ONESHOT_BYTES", "0"))
        if oneshot_bytes > 0 and c.backend == "nccl" and torch.cuda.is_available():
            c.enable_oneshot(oneshot_bytes)
        return c
    return LocalComm()
