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

Limitations (checked): one process (per-step gradient collectives are issued
from Python between the graphs of a chain: GraphedDPStep below), static shapes
(the last, smaller batch of an epoch runs eagerly), CUDA tensors only.
"""
from __future__ import annotations

import os

import torch

from ..optim.optimizers import _FlatOptimizer
from .static_mlp import no_gc

# LDNN_NHWC_INPUT=0: the graph's static input stays an NCHW copy of the batch (A/B knob)
NHWC_INPUT = os.environ.get("LDNN_NHWC_INPUT", "1") == "1"
# LDNN_STAGE_S2D=0: a 7x7 / 2 stem packs its space-to-depth image itself instead of the staging
# pass writing it (A/B knob)
STAGE_S2D = os.environ.get("LDNN_STAGE_S2D", "1") == "1"


def _stem_s2d_image(first, x, cp, C_):
    """The packed space-to-depth image [N][H/2+3][W/2+3][16] the staging pass writes for a first
    layer that is a 7x7 / 2 / pad-3 bias-free stem the s2d forward takes (conv_stem.hip), or None."""
    N, C, H, W = x.shape
    fl = getattr(first, "_ldnn_flat", None)
    if not (STAGE_S2D and fl is not None and fl.shadow is not None and cp == 8 and C <= 4 and H % 2 == 0
            and W % 2 == 0 and first.bias is None and getattr(first, "activation", "none") != "relu"
            and first.groups == 1 and first.dilation == (1, 1) and tuple(first.kernel_size) == (7, 7)
            and tuple(first.stride) == (2, 2) and tuple(first.padding) == (3, 3) and first.in_channels == C):
        return None
    kp = fl.shadow_storage(first.weight).shape[0]
    if not C_.stem_s2d_fwd_ok(N, H, W, cp, kp, 7, 7, 2, 3, C):
        return None
    return torch.empty(N, H // 2 + 3, W // 2 + 3, 16, dtype=torch.bfloat16, device=x.device)


def unit_seed(device) -> torch.Tensor:
    """A persistent fp32 scalar 1 for ``loss.backward(seed)``: no fill launch for the seed, and
    marked so the native loss backward skips multiplying its gradient by it."""
    one = torch.ones((), dtype=torch.float32, device=device)
    one._ldnn_unit = True
    return one


def static_input(model, x_example: torch.Tensor):
    """The graph's static input buffer and its per-step staging function.

    For a conv net whose first layer is an ldnn Conv2d (it reads dense NHWC bf16 with the
    channels padded to 8), the buffer IS that padded NHWC image, seen as a logical NCHW view:
    the per-step staging is one native pass from the caller's NCHW batch (layout + cast +
    zeroed pad channels, the labels copied in the same launch) and the replayed graph starts at
    the first conv -- no device copy of the batch and no layout pass inside the graph (ResNet-18
    b256: a 77 MB copy and a 56 us conversion became one pass).  Anything else: plain copies
    into a clone.  The staging function takes (x, y, y_static)."""
    from ..models.layers import Conv2d
    from ..ops import _ext
    from ..ops import functional as LF

    x = x_example
    first = next((m for m in model.modules() if next(m.children(), None) is None), None)
    if (NHWC_INPUT and x.dim() == 4 and x.is_contiguous() and x.dtype in (torch.float32, torch.bfloat16)
            and isinstance(first, Conv2d) and _ext.use_native(x)):
        N, C, H, W = x.shape
        fl = getattr(first, "_ldnn_flat", None)   # the channel padding the conv's weight shadow uses
        cp = fl.shadow_storage(first.weight).shape[3] if fl is not None and fl.shadow is not None else LF._up8(C)
        buf = torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=x.device)
        C_ = _ext.C()
        # a 7x7 / 2 stem: the same pass also writes its space-to-depth image, which the conv then
        # reads instead of packing it from buf (ResNet-18 b256: one 313 MB pass less)
        img = _stem_s2d_image(first, x, cp, C_) if x.data_ptr() % 8 == 0 else None
        C_.nchw_to_nhwc(x, buf, s2d=img)
        xs = LF.nchw_view(buf, C)
        xs._ldnn_zpad = True   # the staging pass writes the pad channels' zeros
        if img is not None:   # (with x's version: an in-place change of x after staging voids the image)
            xs._ldnn_s2d = (img, xs._version)

        def stage(xn: torch.Tensor, yn: torch.Tensor, ys: torch.Tensor):
            if xn.device != buf.device or xn.dtype not in (torch.float32, torch.bfloat16):
                xn = xn.to(buf.device, torch.float32)   # (a host batch, fp16 / uint8: what copy_ accepted)
            xn = xn if xn.is_contiguous() and xn.data_ptr() % 8 == 0 else xn.clone()
            if (yn.is_cuda and yn.is_contiguous() and yn.dtype == ys.dtype and yn.nbytes % 8 == 0
                    and yn.data_ptr() % 8 == 0):   # the labels ride along in the same launch
                C_.nchw_to_nhwc(xn, buf, yn, ys, s2d=img)
            else:
                C_.nchw_to_nhwc(xn, buf, s2d=img)
                ys.copy_(yn, non_blocking=True)
        return xs, stage

    xs = x.detach().clone()

    def copy(xn: torch.Tensor, yn: torch.Tensor, ys: torch.Tensor):
        xs.copy_(xn, non_blocking=True)
        ys.copy_(yn, non_blocking=True)
    return xs, copy


# (An optimizer overlapped with the backward on a side-stream branch of the step
# graph was built in round 2 and measured slower -- EnhancedCNN b64 2.21-2.24 vs
# 2.32-2.44 ms, profiles/overlap_optimizer_ab_r2.jsonl: a replayed graph's branches
# run one after the other on this stack -- and removed.)


class GraphedStep:
    def __init__(self, model, criterion, optimizer, x_example: torch.Tensor, y_example: torch.Tensor,
                 warmup: int = 3, stats: torch.Tensor | None = None):
        if not x_example.is_cuda:
            raise ValueError("GraphedStep needs GPU tensors")
        self.model, self.criterion, self.optimizer = model, criterion, optimizer
        self.x, self._stage_x = static_input(model, x_example)
        self.y = y_example.detach().clone()
        self.stats = stats if stats is not None else torch.zeros(2, dtype=torch.float32, device=self.x.device)
        self._lrs = None
        # persistent d(loss)/d(loss) = 1: the captured backward needs no seed fill launch, and
        # the loss backward knows it scales by exactly 1 (no scaling pass: _SoftmaxXentNative)
        self._one = unit_seed(self.x.device)
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
        loss.backward(seed)
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
        self._stage_x(x, y, self.y)
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

    mode "segmented" (default with RCCL): the step is captured as a CHAIN of
    graphs cut at the bucket-ready points of the backward -- G_0 = zero_grad +
    forward + loss + backward up to the moment bucket b_0's last gradient is
    written, G_1 = the backward on to b_1's, ... -- plus G_opt = (widen / mix +)
    fused optimizer.  A replay launches G_0, issues b_0's RCCL all-reduce from the
    host (RCCL's own stream waits on an event behind G_0), launches G_1 at once,
    and so on; the host then makes the compute stream wait for every collective
    (no host sync) and launches G_opt.  So bucket i travels over xGMI on its own
    HIP stream / hardware queue while G_{i+1}.. run on the compute stream.
    (Putting the collectives on a side-stream branch INSIDE one graph does not
    overlap on this stack: a replayed graph's branches execute one after the
    other, profiles/graph_branch_concurrency_r2.jsonl -- separate streams do.)
    mode "after" (host-staged backends such as gloo, or on request): one backward
    graph, then the bucket collectives from Python, then G_opt.

    With ``DataParallel(shard_optimizer=True)`` a bucket's collective is a
    reduce-scatter, G_opt widens + updates only this rank's shards (and the
    replicated 1-D tail), and after G_opt the host issues the in-place bf16 weight
    all-gathers in forward order; the next replay's stream waits for them first.

    1/N averaging is folded into the optimizer (flat.grad_scale); the weighted
    all-reduce's mix and the bf16 stage widen run in G_opt (GradBucketer
    post_collective).  Every replay issues its collectives through ``comm`` -- the
    same ops, in the same order, as the eager fallback for an odd-shaped batch --
    so the runtime schedule check (Comm.check_schedule) sees identical sequences
    on ranks whose last batch is short and on ranks whose is not.

    ``comm_fn(i, buf)`` (tests, overlap probes) replaces the collective of bucket i;
    it is called on the host where the collective would be issued and may return
    an object with ``wait()`` (called before G_opt, e.g. a cross-stream join).
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
        self.x, self._stage_x = static_input(self.model, x_example)
        self.y = y_example.detach().clone()
        self._one = unit_seed(self.x.device)
        self.stats = stats if stats is not None else torch.zeros(2, dtype=torch.float32, device=self.x.device)
        self._lrs = None
        self.device_collectives = bool(getattr(self.comm, "device_collectives", False))
        if mode is None:
            mode = "segmented" if (self.device_collectives or comm_fn is not None) else "after"
        if mode not in ("segmented", "after"):
            raise ValueError(f"unknown GraphedDPStep mode {mode!r}")
        self.mode = mode
        nb = len(self.bk.buckets)
        self._cap = None
        self.flat.add_ready_group_hook(self._on_ready)
        torch.cuda.synchronize(self.x.device)
        self.stats.zero_()
        self.graphs: list = []     # the backward chain G_0 .. G_k
        self.issue: list = []      # buckets whose collective is issued after G_j
        self._empty: list = []     # G_j captured no work (not replayed)
        self._pool = torch.cuda.graph_pool_handle()
        self._stream = torch.cuda.Stream(device=self.x.device)
        self._stream.wait_stream(torch.cuda.current_stream())
        # sharded DP: the forward is cut too, right before the first module that reads a
        # sharded bucket's weights; a replay waits for that bucket's all-gather (issued
        # after the previous step's optimizer, in forward order) only there, so the
        # gathers of the deep layers' big weights run beside the shallow layers' forward
        self.waits: list = []      # buckets whose weight all-gather graph G_j waits for
        self._fwd_hooks = []
        self._fwd_seen: set = set()
        if self.bk.shard:
            for mod in self.model.modules():
                own = [p for p in mod.parameters(recurse=False)]
                if own and self.bk.buckets_of(own):
                    self._fwd_hooks.append(mod.register_forward_pre_hook(self._on_forward))
        self._set_capture(True)
        try:
            self._cap = {"pending": [len(b["params"]) for b in self.bk.buckets], "fired": [False] * nb,
                         "seen": set()}
            with no_gc(), torch.cuda.stream(self._stream):
                self._begin()
                self.optimizer.zero_grad()
                out = self.model(self.x)
                try:
                    loss = self.criterion(out, self.y, self.stats)
                except TypeError:
                    loss = self.criterion(out.float(), self.y)
                loss.backward(self._one if loss.dtype == torch.float32 and loss.dim() == 0 else None)
                rest = [i for i in range(nb) if not self._cap["fired"][i]]   # params with no gradient
                if rest:
                    self._fire(rest)
                self._end()
                if self.mode == "after":
                    self.issue[-1] = list(range(nb))
                self._capture_opt()
            self.loss = loss
        finally:
            self._cap = None
            self._set_capture(False)
            for h in self._fwd_hooks:
                h.remove()
            self._fwd_hooks = []
        torch.cuda.current_stream().wait_stream(self._stream)
        self._sync_lr(force=True)

    # ---------------------------------------------------------------- capture
    def _set_capture(self, on: bool):
        if isinstance(self.optimizer, _FlatOptimizer):
            self.optimizer._ldnn_capturing = on

    def _on_forward(self, mod, args):
        """(capture) module ``mod`` is about to read its weights: cut the chain before it
        when one of its sharded buckets has not been waited for in this forward yet."""
        if self._cap is None:
            return
        need = [b for b in self.bk.buckets_of(mod.parameters(recurse=False)) if b not in self._fwd_seen]
        if not need:
            return
        self._fwd_seen.update(need)
        self._end()
        self._begin()
        self.waits[-1] = need   # waited before the link that starts here

    def _begin(self):
        # relaxed: a link of the chain begins on one thread (main / autograd) and may end
        # on the other, which a thread_local capture refuses
        # (hipErrorStreamCaptureWrongThread); RCCL's watchdog and gloo's progress
        # threads keep querying the HIP runtime meanwhile, which a global capture refuses
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self._pool, capture_error_mode="relaxed")
        self._cur = g
        self.waits.append([])

    def _end(self):
        import warnings

        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            self._cur.capture_end()
        self.graphs.append(self._cur)
        self.issue.append([])
        self._empty.append(any("empty" in str(w.message).lower() for w in ws))
        self._cur = None

    def _capture_opt(self):
        """G_opt = widen / mix + the fused optimizer.  Sharded: one graph PER BUCKET in
        GradBucketer.opt_order (the sharded buckets in the order their reduce-scatters
        complete, then the replicated tail), so a replay waits for each bucket's own
        collective right before its update: the deep buckets update while the last
        bucket's reduce-scatter is still in flight.  (self.g_opts: [(graph, bucket or None)])"""
        self.g_opts = []
        order = self.bk.opt_order() if (self.bk.shard and isinstance(self.optimizer, _FlatOptimizer)) else None

        def begin(i):
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=self._pool, capture_error_mode="relaxed")
            self.g_opts.append((g, i))

        if order is None:
            begin(None)
            for i in range(len(self.bk.buckets)):
                self.bk.post_collective(i)
            self.optimizer.step()
            self.g_opts[-1][0].capture_end()
            return

        def parts(update):
            for k, i in enumerate(order):
                if k > 0:
                    self.g_opts[-1][0].capture_end()
                    begin(i)
                else:
                    self.g_opts[-1] = (self.g_opts[-1][0], i)
                self.bk.post_collective(i)
                update(*self.bk.update_range(i))

        begin(None)   # (the optimizer's per-step prologue, e.g. Adam's step count, lands in the first)
        self.bk.step_parts = parts
        try:
            self.optimizer.step()
        finally:
            self.bk.step_parts = None
        self.g_opts[-1][0].capture_end()

    def _fire(self, idx):
        """(capture) buckets ``idx``'s gradients are complete at this point of the backward."""
        for i in idx:
            self._cap["fired"][i] = True
            self.bk.pre_collective(i)   # own-gradient copy / bf16 stage: captured before the cut
        if self.mode == "segmented":
            # cut the chain here: the autograd thread runs this hook with the forward's
            # (= capture) stream current, so the next backward kernels land in G_{j+1}
            if torch.cuda.current_stream() != self._stream:
                raise RuntimeError("GraphedDPStep: a gradient-ready hook ran off the capture stream")
            self._end()
            self.issue[-1].extend(idx)
            self._begin()

    def _on_ready(self, params):
        c = self._cap
        if c is None:
            return
        for p in params:
            if id(p) in c["seen"]:
                continue
            c["seen"].add(id(p))
            i = self.bk.of_param.get(id(p))
            if i is not None:
                c["pending"][i] -= 1
        # fire in bucket order, as GradBucketer launches them (same schedule on every path)
        done = []
        nxt = c.setdefault("next", 0)
        while nxt < len(c["pending"]) and c["pending"][nxt] == 0:
            done.append(nxt)
            nxt += 1
        c["next"] = nxt
        if done:
            self._fire(done)

    def _sync_lr(self, force: bool = False):
        lrs = [g["lr"] for g in self.optimizer.param_groups]
        if force or lrs != self._lrs:
            if isinstance(self.optimizer, _FlatOptimizer):
                self.optimizer.sync_hyperparams()
            self._lrs = lrs

    def _collective(self, i):
        if self.comm_fn is not None:
            w = self.comm_fn(i, self.bk.comm_buffer(i))
            return w if hasattr(w, "wait") else None
        return self.bk.collective(i)   # reduce-scatter (sharded bucket) or all-reduce

    @property
    def n_segments(self) -> int:
        return len(self.graphs)

    # -------------------------------------------------------------------- API
    def flush_stats(self, into: torch.Tensor):
        into.add_(self.stats)
        self.stats.zero_()

    def __call__(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        if x.shape != self.x.shape or y.shape != self.y.shape:
            return self._eager_step(x, y)
        self._stage_x(x, y, self.y)
        self._sync_lr()
        works = {}
        for j, g in enumerate(self.graphs):
            if self.waits[j]:
                self.bk.wait_gathers(self.waits[j])   # this link's first reads of those buckets' weights
            if not self._empty[j]:
                g.replay()
            issue = self.issue[j]
            if issue and not self.device_collectives and self.comm_fn is None:
                torch.cuda.current_stream().synchronize()  # a host-staged backend reads the buffers
            for i in issue:
                works[i] = self._collective(i)
        self.bk.wait_gathers()   # (any gather no forward link waited for) before the optimizer writes
        host_staged = not self.device_collectives and self.comm_fn is None
        # each optimizer graph waits only for ITS bucket's collective (a stream wait): the deep
        # buckets, reduced first, update while the last bucket's reduce-scatter is still on
        # the wire; the weight all-gathers then go out in forward order.  (The round-4 order --
        # each gather right after its own update -- measured neutral, 0.34-0.35 vs 0.36 ms
        # exposed, and was removed in round 6.)
        for g, i in self.g_opts:
            for k in (list(works) if i is None else [i]):
                w = works.pop(k, None)
                if w is not None:
                    w.wait()
            g.replay()
        for w in works.values():   # (buckets without an optimizer graph of their own)
            if w is not None:
                w.wait()
        if self.bk.shard:
            self.bk.master_whole = False
            if any(i is not None for _, i in self.g_opts):
                if host_staged:
                    torch.cuda.current_stream().synchronize()   # a host-staged backend reads the shadow
                self.bk.issue_gathers()
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
