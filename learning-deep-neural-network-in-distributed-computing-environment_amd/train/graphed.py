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


class GraphedStep:
    def __init__(self, model, criterion, optimizer, x_example: torch.Tensor, y_example: torch.Tensor,
                 warmup: int = 3, stats: torch.Tensor | None = None):
        if not x_example.is_cuda:
            raise ValueError("GraphedStep needs GPU tensors")
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.x = x_example.detach().clone()
        self.y = y_example.detach().clone()
        self.stats = stats if stats is not None else torch.zeros(2, dtype=torch.float32, device=self.x.device)
        self._lrs = None
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
            with no_gc(), torch.cuda.graph(self.graph):
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
        loss.backward()
        self.optimizer.step()
        return loss

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
