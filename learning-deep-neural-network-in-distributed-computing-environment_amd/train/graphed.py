"""A whole training step replayed from one hipGraph (HIP graphs instead of a
tracing compiler).

The reference's hot loop (BAR/trainer.py:194-223) launches every op from
Python each step: zero_grad, the forward modules, the loss, autograd's
backward, the optimizer, then three ``.item()`` host syncs.  For small
models (LeNet-5 at batch 1024, the MLPs) that host-side launch stream, not
the GPU, sets the step time.  ``GraphedStep`` runs the same eager step a few
times on a side stream (so lazily allocated state -- momentum buffers,
workspaces, BN counters -- exists), then captures ONE step into a
torch.cuda.CUDAGraph (= hipGraph on ROCm) and replays it: one host call per
step, every kernel of the forward, backward and fused optimizer in one graph
launch.

What makes the ldnn step capturable:
* inputs are copied into static device buffers before each replay;
* loss / #correct accumulate on the device (CrossEntropyLoss ``stats``), read
  whenever the caller wants them (no per-step sync);
* the fused optimizers read lr (and Adam's step count) from a device tensor;
  the graph does NOT capture the host->device lr write, ``GraphedStep``
  refreshes it before a replay whenever ``param_groups[..]['lr']`` changed
  (so StepLR & co. keep working);
* every native op writes into caller-provided / caching-allocator tensors
  (graph-pool allocations during capture).

Limitations (checked): one process (no per-step gradient collectives inside
the graph -- those are issued from Python between graph segments, see
train/static_mlp.py), static shapes (the last, smaller batch of an epoch runs
eagerly), CUDA tensors only.
"""
from __future__ import annotations

import torch

from ..optim.optimizers import _FlatOptimizer
from .static_mlp import no_gc


# Optimizer overlapped with the backward (GraphedStep overlap_optimizer): the flat
# buffer is laid out in gradient-ready order, so the parameters whose gradients are
# final form a growing prefix of it.  When an op notifies new gradients, every
# parameter that became ready BEFORE it is past its last backward read (its own dgrad
# / BN backward ran earlier on the main stream), so that prefix is updated on a side
# stream -- forked from the main stream at that point -- while the backward goes on;
# the rest is updated on the main stream after the backward and the side stream joins.
# OFF by default: measured on MI355X (profiles/overlap_optimizer_ab_r2.jsonl, same box,
# alternated) EnhancedCNN b64 2.21-2.24 ms without it vs 2.32-2.44 ms with it, and
# 3.27 ms with a 32-block side grid -- the side-stream branch of the replayed graph does
# not run beside the backward kernels here, it adds to them (as in
# profiles/graph_branch_concurrency_r2.jsonl).  LDNN_OVERLAP_OPT=1 turns it on,
# LDNN_OVERLAP_OPT_ELEMS sets the launch granularity, LDNN_OVERLAP_OPT_BLOCKS the side grid.
# (Assumes every parameter's gradient is written by one op per step -- true of the
# models here; tied / shared weights need overlap_optimizer=False.)
_OVERLAP_OPT = __import__("os").environ.get("LDNN_OVERLAP_OPT", "0") != "0"
_OVERLAP_ELEMS = int(__import__("os").environ.get("LDNN_OVERLAP_OPT_ELEMS", str(4 << 20)))
_OVERLAP_BLOCKS = int(__import__("os").environ.get("LDNN_OVERLAP_OPT_BLOCKS", "0"))  # side launches' grid cap


class _OverlapUpdate:
    def __init__(self, upd, flat, side: torch.cuda.Stream, min_elems: int):
        self.upd, self.flat, self.side, self.min_elems = upd, flat, side, min_elems
        self.segs = flat.segments          # buffer (gradient-ready) order
        self.idx, self.lo = 0, 0           # [0, lo) updated / launched
        self.ready: set = set()

    def on_ready(self, params):
        # (a native op notifies its parameters while its backward still runs; autograd's
        # AccumulateGrad then re-notifies each one after the op returned -- a repeat is
        # that echo.  Each parameter's gradient must come from ONE op per step: shared
        # weights need overlap_optimizer=False.)
        j = self.idx
        while j < len(self.segs) and id(self.segs[j].param) in self.ready:
            j += 1
        self.ready.update(id(p) for p in params)
        hi = self.segs[j].offset if j < len(self.segs) else self.flat.numel
        if j > self.idx and hi - self.lo >= self.min_elems:
            cur = torch.cuda.current_stream()
            self.side.wait_stream(cur)     # everything issued so far (the readers of [lo, hi))
            with torch.cuda.stream(self.side):
                if _OVERLAP_BLOCKS:
                    from ..ops import _ext
                    _ext.C().set_opt_max_blocks(_OVERLAP_BLOCKS)
                try:
                    self.upd.update(self.lo, hi)
                finally:
                    if _OVERLAP_BLOCKS:
                        _ext.C().set_opt_max_blocks(0)
            self.lo, self.idx = hi, j

    def finish(self):
        self.flat.finalize_grads()         # gradients no op wrote this step (outside [0, lo))
        self.upd.update(self.lo, self.flat.numel)
        torch.cuda.current_stream().wait_stream(self.side)
        self.upd.end()


class GraphedStep:
    def __init__(self, model, criterion, optimizer, x_example: torch.Tensor, y_example: torch.Tensor,
                 warmup: int = 3, stats: torch.Tensor | None = None, overlap_optimizer: bool | None = None):
        if not x_example.is_cuda:
            raise ValueError("GraphedStep needs GPU tensors")
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        if overlap_optimizer is None:
            overlap_optimizer = _OVERLAP_OPT
        self._ov_side, self._ov = None, None
        if overlap_optimizer and isinstance(optimizer, _FlatOptimizer) and optimizer.supports_ranges():
            self._ov_flat = optimizer._flat_for_group(optimizer.param_groups[0])
            self._ov_side = torch.cuda.Stream(device=x_example.device)
            self._ov_flat.add_ready_group_hook(self._on_ready)
        self.x = x_example.detach().clone()
        self.y = y_example.detach().clone()
        self.stats = stats if stats is not None else torch.zeros(2, dtype=torch.float32, device=self.x.device)
        self._lrs = None
        # persistent d(loss)/d(loss) = 1: the captured backward needs no seed fill launch
        self._one = torch.ones((), dtype=torch.float32, device=self.x.device)
        s = torch.cuda.Stream(device=self.x.device)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):  # warmup=0: the caller already ran eager steps
                self._eager()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize(self.x.device)
        self.stats.zero_()
        self.graph = torch.cuda.CUDAGraph()
        self._set_capture(True)
        try:
            # captured on the warmup stream: the per-stream native workspaces (conv
            # split-K counters, xent accumulators) exist already, so no fill lands in the graph
            with no_gc(), torch.cuda.graph(self.graph, stream=s):
                self.loss = self._eager()
        finally:
            self._set_capture(False)
        self._sync_lr(force=True)

    # ------------------------------------------------------------------ helpers
    def _set_capture(self, on: bool):
        if isinstance(self.optimizer, _FlatOptimizer):
            self.optimizer._ldnn_capturing = on

    def _eager(self):
        # (zero_grad stays IN the graph: clearing the gradients inside the optimizer
        # kernel instead -- step(clear_grads=True) -- measured slower on MI355X, its
        # extra 178 MB of zero writes cost more than the fill launch it replaces)
        self.optimizer.zero_grad()
        out = self.model(self.x)
        try:
            loss = self.criterion(out, self.y, self.stats)
        except TypeError:  # a stock criterion without the stats argument
            loss = self.criterion(out.float(), self.y)
        seed = self._one if loss.dtype == torch.float32 and loss.dim() == 0 else None
        if self._ov_side is not None:
            self._ov = _OverlapUpdate(self.optimizer.range_updater(), self._ov_flat, self._ov_side, _OVERLAP_ELEMS)
            try:
                loss.backward(seed)
                self._ov.finish()
            finally:
                self._ov = None
        else:
            loss.backward(seed)
            self.optimizer.step()
        return loss

    def _on_ready(self, params):
        if self._ov is not None:
            self._ov.on_ready(params)

    def _sync_lr(self, force: bool = False):
        lrs = [g["lr"] for g in self.optimizer.param_groups]
        if force or lrs != self._lrs:
            if isinstance(self.optimizer, _FlatOptimizer):
                self.optimizer.sync_hyperparams()
            self._lrs = lrs

    # ---------------------------------------------------------------------- API
    def flush_stats(self, into: torch.Tensor):
        """Move the [loss_sum, correct] the replays accumulated into ``into`` (device add)."""
        into.add_(self.stats)
        self.stats.zero_()

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """One training step on (x, y); returns the (device) loss tensor of this step."""
        if x.shape != self.x.shape or y.shape != self.y.shape:
            return self._eager_step(x, y)
        self.x.copy_(x, non_blocking=True)
        self.y.copy_(y, non_blocking=True)
        self._sync_lr()
        self.graph.replay()
        return self.loss

    def _eager_step(self, x, y):
        """Odd-shaped batch (e.g. the last one of an epoch): run it without the graph."""
        self.optimizer.zero_grad()
        out = self.model(x)
        try:
            loss = self.criterion(out, y, self.stats)
        except TypeError:
            loss = self.criterion(out.float(), y)
        loss.backward()
        self.optimizer.step()
        return loss.detach()


class GraphedDPStep:
    """A data-parallel training step (per-step gradient all-reduce) replayed from
    hipGraphs, with the bucket all-reduces overlapping the backward pass.

    The reference's DP hot loop (BAR/trainer.py:194-223 + communication.py:21-25)
    is the eager step plus 65 blocking per-tensor all-reduces.  ``DataParallel``
    (parallel/ddp.py) already buckets the flat gradient and launches each bucket's
    all-reduce from backward hooks -- but eagerly, one Python launch per kernel.

    mode "in_graph" (default with RCCL): ONE graph per step.  The bucket-readiness
    hooks fire once during capture; at each the capture forks onto a side stream
    and captures that bucket's RCCL all-reduce there (after the bucket's bf16
    staging copy when comm_dtype is bf16), so in every replay bucket i travels over
    xGMI while the backward nodes of buckets i+1.. still run; the capture joins the
    side stream before the (widen +) fused optimizer nodes.  1/N averaging is
    folded into the optimizer (flat.grad_scale).
    mode "after" (host-staged backends such as gloo, or on request): graph G1 =
    zero_grad + forward + backward, then the bucket collectives from Python, then
    graph G2 = (widen +) optimizer.

    ``comm_fn(i, buf)`` (tests) replaces the collective of bucket i and is issued
    exactly where the collective would be.
    """

    def __init__(self, dp, criterion, optimizer, x_example: torch.Tensor, y_example: torch.Tensor,
                 stats: torch.Tensor | None = None, mode: str | None = None, comm_fn=None):
        from ..parallel.comm import SUM

        if not x_example.is_cuda:
            raise ValueError("GraphedDPStep needs GPU tensors")
        self.dp, self.model, self.criterion, self.optimizer = dp, dp.module, criterion, optimizer
        self.bk, self.flat, self.comm = dp.bucketer, dp.flat, dp.comm
        self._SUM = SUM
        self.comm_fn = comm_fn
        self.x = x_example.detach().clone()
        self.y = y_example.detach().clone()
        self.stats = stats if stats is not None else torch.zeros(2, dtype=torch.float32, device=self.x.device)
        self._lrs = None
        if mode is None:
            mode = "in_graph" if (getattr(self.comm, "device_collectives", False) or comm_fn is not None) else "after"
        if mode not in ("in_graph", "after"):
            raise ValueError(f"unknown GraphedDPStep mode {mode!r}")
        self.mode = mode
        nb = len(self.bk.buckets)
        self.side = torch.cuda.Stream(device=self.x.device) if mode == "in_graph" else None
        self._cap = None
        self.flat.add_ready_hook(self._on_ready)
        torch.cuda.synchronize(self.x.device)
        self.stats.zero_()
        self.g1 = torch.cuda.CUDAGraph()
        self.g2 = torch.cuda.CUDAGraph() if mode == "after" else None
        self._set_capture(True)
        try:
            self._cap = {"pending": [len(b["params"]) for b in self.bk.buckets], "fired": [False] * nb,
                         "seen": set(), "works": []}
            with no_gc(), torch.cuda.graph(self.g1):
                self.optimizer.zero_grad()
                out = self.model(self.x)
                try:
                    loss = self.criterion(out, self.y, self.stats)
                except TypeError:
                    loss = self.criterion(out.float(), self.y)
                loss.backward()
                for i in range(nb):  # buckets whose parameters got no gradient
                    if not self._cap["fired"][i]:
                        self._fire(i)
                if mode == "in_graph":
                    for w in self._cap["works"]:
                        if w is not None:
                            w.wait()
                    torch.cuda.current_stream().wait_stream(self.side)
                    self._widen_and_step()
            self._cap = None
            self.loss = loss
            if mode == "after":
                with no_gc(), torch.cuda.graph(self.g2, pool=self.g1.pool()):
                    self._widen_and_step()
        finally:
            self._cap = None
            self._set_capture(False)
        self._sync_lr(force=True)

    # ---------------------------------------------------------------- capture
    def _set_capture(self, on: bool):
        if isinstance(self.optimizer, _FlatOptimizer):
            self.optimizer._ldnn_capturing = on

    def _widen_and_step(self):
        if self.bk._stage is not None:
            for i, b in enumerate(self.bk.buckets):
                self.flat.grad[b["begin"]: b["end"]].copy_(self.bk._stage[i])
        self.optimizer.step()

    def _fire(self, i):
        """(capture) bucket i's gradients are complete at this point of the graph."""
        self._cap["fired"][i] = True
        if self.bk._stage is not None:
            b = self.bk.buckets[i]
            self.bk._stage[i].copy_(self.flat.grad[b["begin"]: b["end"]])
        if self.mode == "in_graph":
            self.side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.side):
                self._cap["works"].append(self._collective(i, async_op=True))

    def _on_ready(self, p):
        c = self._cap
        if c is None or id(p) in c["seen"]:
            return
        c["seen"].add(id(p))
        i = self.bk.of_param.get(id(p))
        if i is None:
            return
        c["pending"][i] -= 1
        if c["pending"][i] == 0 and not c["fired"][i]:
            self._fire(i)

    def _sync_lr(self, force: bool = False):
        lrs = [g["lr"] for g in self.optimizer.param_groups]
        if force or lrs != self._lrs:
            if isinstance(self.optimizer, _FlatOptimizer):
                self.optimizer.sync_hyperparams()
            self._lrs = lrs

    def _buf(self, i):
        if self.bk._stage is not None:
            return self.bk._stage[i]
        b = self.bk.buckets[i]
        return self.flat.grad[b["begin"]: b["end"]]

    def _collective(self, i, async_op=False):
        buf = self._buf(i)
        if self.comm_fn is not None:
            self.comm_fn(i, buf)
            return None
        return self.comm.all_reduce(buf, self._SUM, async_op=async_op)

    # -------------------------------------------------------------------- API
    def flush_stats(self, into: torch.Tensor):
        into.add_(self.stats)
        self.stats.zero_()

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if x.shape != self.x.shape or y.shape != self.y.shape:
            return self._eager_step(x, y)
        self.x.copy_(x, non_blocking=True)
        self.y.copy_(y, non_blocking=True)
        self._sync_lr()
        self.g1.replay()
        if self.mode == "after":
            if not getattr(self.comm, "device_collectives", False):
                torch.cuda.current_stream().synchronize()  # a host-staged backend reads the buffers
            works = [self._collective(i, async_op=True) for i in range(len(self.bk.buckets))]
            for w in works:
                if w is not None:
                    w.wait()
            self.g2.replay()
        return self.loss

    def _eager_step(self, x, y):
        """Odd-shaped batch (the last one of an epoch): the eager bucketed DP step."""
        self.optimizer.zero_grad()
        out = self.dp(x)
        try:
            loss = self.criterion(out, y, self.stats)
        except TypeError:
            loss = self.criterion(out.float(), y)
        loss.backward()
        self.dp.finish_gradient_sync()
        self.optimizer.step()
        return loss.detach()
