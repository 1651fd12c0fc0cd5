"""Flat parameter / gradient / bf16-shadow storage for a model.

The reference keeps 65 separate parameter tensors and aggregates them with 65
separate collectives (BAR/communication.py:4-31).  On MI355X
that is the wrong shape: every collective and every optimizer launch has a
fixed cost, and RCCL over xGMI wants few, large messages.  FlatParams moves a
model's parameters into ONE contiguous fp32 master buffer (each
``nn.Parameter`` becomes a view into it, so ``state_dict()`` keeps the
reference key names such as ``prep.0.weight`` / ``fc.bias``), with

* ``grad``   -- one fp32 gradient buffer; ``param.grad`` is a view into it,
* ``shadow`` -- one bf16 copy of the weights that the MFMA kernels read
  (refreshed by the fused optimizer in the same pass that updates the master),
* per-parameter padded *storage* views: a parameter whose leading dim is not a
  multiple of 8 (e.g. the 10-class classifier) gets zero rows of padding so the
  GEMM never needs a scalar tail; the padding stays exactly zero because its
  gradient is always zero.  Conv weights are stored KRSC (channels innermost,
  K and C padded to 8) -- the layout the implicit-GEMM conv kernels read --
  while the Parameter keeps the reference's [K][C][R][S] shape as a permuted view.

Segments are 64-element aligned (256 B fp32 / 128 B bf16) so every view is
16-byte aligned for vector loads.  The order of segments is the order in which
gradients become ready during backward (reverse of registration), which is
what gradient bucketing wants.
"""
from __future__ import annotations

from dataclasses import dataclass

import weakref

import torch
import torch.nn as nn

_ALIGN = 64

# id(param) -> FlatParams that owns it (lets optimizers find the flat buffers)
_OWNER: "weakref.WeakValueDictionary[int, FlatParams]" = weakref.WeakValueDictionary()


def owner_of(p: nn.Parameter):
    return _OWNER.get(id(p))


def storage_numel(shape, pad_rows: bool = True) -> int:
    """Elements a parameter of `shape` occupies in the flat buffers (padding + 64-alignment)."""
    sshape = _pad_rows(torch.Size(shape)) if (pad_rows and len(shape) >= 1) else tuple(shape)
    n = 1
    for d in sshape:
        n *= d
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _pad_rows(shape: torch.Size, multiple: int = 8) -> tuple:
    """Padded storage shape: leading dim to a multiple of 8 and, for 2-D
    (Linear) weights, the inner dim too, so every GEMM operand row is a whole
    number of 16-byte vectors."""
    if len(shape) == 0:
        return tuple(shape)
    up = lambda v: (v + multiple - 1) // multiple * multiple  # noqa: E731
    if len(shape) == 2:
        return (up(shape[0]), up(shape[1]))
    if len(shape) == 4:  # conv weight [K][C][R][S] stored KRSC with K and C padded
        k, c, r, s = shape
        return (up(k), r, s, up(c))
    return (up(shape[0]),) + tuple(shape[1:])


@dataclass
class Segment:
    name: str
    param: nn.Parameter
    offset: int        # element offset of the padded storage in the flat buffers
    numel: int         # logical elements
    storage_shape: tuple  # padded shape
    storage_numel: int


class FlatParams:
    """Owns flat master/grad/shadow buffers for ``module``'s parameters."""

    def __init__(self, module: nn.Module, device: torch.device | str | None = None, pad_rows: bool = True,
                 shadow: bool | None = None, grad_ready_order: bool = True, order: list | None = None,
                 align_after: dict | None = None):
        self.module = module
        params = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        if device is None:
            device = params[0][1].device if params else torch.device("cpu")
        self.device = torch.device(device)
        if shadow is None:
            shadow = self.device.type == "cuda"
        if order is not None:  # explicit layout (e.g. a static engine's bucket plan)
            names = {id(p): n for n, p in params}
            ordered = [(names[id(p)], p) for p in order]
            assert len(ordered) == len(params), "order must list every trainable parameter once"
        else:
            ordered = list(reversed(params)) if grad_ready_order else params
        segs = []
        off = 0
        for name, p in ordered:
            sshape = _pad_rows(p.shape) if (pad_rows and p.dim() >= 1) else tuple(p.shape)
            snumel = 1
            for d in sshape:
                snumel *= d
            segs.append(Segment(name, p, off, p.numel(), sshape, snumel))
            off += (snumel + _ALIGN - 1) // _ALIGN * _ALIGN
            if align_after and id(p) in align_after:  # e.g. a bucket boundary that must split N ways
                a = int(align_after[id(p)])
                off = (off + a - 1) // a * a
        self.numel = off
        self.segments = segs
        self.by_param = {id(s.param): s for s in segs}
        self.master = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=self.device) if shadow else None
        with torch.no_grad():
            for s in segs:
                st = self.storage_view(s, self.master)
                st.zero_()
                self._logical(s, st).copy_(s.param.detach().to(self.device, torch.float32))
                s.param.data = self._logical(s, st)
                s.param.grad = self._logical(s, self.storage_view(s, self.grad))
        # gradient-readiness notification: native ops call notify() after writing a
        # weight gradient; params handled by stock torch ops signal through autograd.
        self._ready_hooks: list = []
        self._ready_group_hooks: list = []
        # first-write gradients: native ops ask grad_beta() before writing a gradient;
        # after a lazy zero_grad the first writer overwrites (beta 0) instead of
        # accumulating onto a zero-filled buffer -- no fill pass, and the fp32 wgrad
        # epilogues store without reading.
        self._native: set = set()   # params whose gradients native ops write
        self._stale: set = set()    # params whose gradient is logically zero, not cleared
        self.grad_scale = 1.0  # set to 1/N by data parallelism; consumed by the fused optimizers
        for s in segs:
            _OWNER[id(s.param)] = self
        for s in segs:
            s.param.register_post_accumulate_grad_hook(lambda p: self.notify(p))
        for m in module.modules():
            if hasattr(m, "_ldnn_flat"):
                m._ldnn_flat = self
        self.refresh_shadow()

    def add_ready_hook(self, fn):
        self._ready_hooks.append(fn)

    def add_ready_group_hook(self, fn):
        """fn(params): called once per notify() with every parameter it names (the
        gradients one op wrote together; the op may still read those weights after)."""
        self._ready_group_hooks.append(fn)

    def notify(self, *params):
        ps = [p for p in params if p is not None]
        for p in ps:
            for fn in self._ready_hooks:
                fn(p)
        if ps:
            for fn in self._ready_group_hooks:
                fn(ps)

    # ---- views ---------------------------------------------------------------
    @staticmethod
    def storage_view(seg: Segment, flat: torch.Tensor) -> torch.Tensor:
        return flat[seg.offset: seg.offset + seg.storage_numel].view(seg.storage_shape)

    @staticmethod
    def _logical(seg: Segment, storage: torch.Tensor) -> torch.Tensor:
        shape = tuple(seg.param.shape)
        if len(shape) == 0:
            return storage
        if len(shape) == 2:
            return storage[: shape[0], : shape[1]]
        if len(shape) == 4:  # KRSC storage -> the reference's [K][C][R][S] view
            return storage[: shape[0], :, :, : shape[1]].permute(0, 3, 1, 2)
        return storage[: shape[0]]

    def seg(self, p: nn.Parameter) -> Segment:
        return self.by_param[id(p)]

    def master_storage(self, p):
        return self.storage_view(self.seg(p), self.master)

    def grad_storage(self, p):
        return self.storage_view(self.seg(p), self.grad)

    def shadow_storage(self, p):
        if self.shadow is None:
            raise RuntimeError("FlatParams was built without a bf16 shadow")
        return self.storage_view(self.seg(p), self.shadow)

    def params(self):
        return [s.param for s in self.segments]

    # ---- maintenance --------------------------------------------------------
    @torch.no_grad()
    def refresh_shadow(self):
        """Re-derive the bf16 shadow after the master changed outside the optimizer
        (initial broadcast, load_state_dict, weight averaging without fused mix)."""
        if self.shadow is None:
            return
        from ..ops import _ext

        if _ext.use_native(self.master):
            _ext.C().cast_f32_bf16(self.master, self.shadow)
            # (a native write leaves the version counter alone: bump it, readers that keep
            # derived copies of the shadow -- StaticMLPEngine's transposed W -- key on it)
            torch.autograd.graph.increment_version(self.shadow)
        else:
            self.shadow.copy_(self.master)

    def grad_beta(self, p) -> float:
        """0.0 when ``p``'s gradient is logically zero (lazy zero_grad, not written yet
        this step): the caller overwrites; else 1.0 (accumulate)."""
        i = id(p)
        self._native.add(i)
        if i in self._stale:
            self._stale.discard(i)
            return 0.0
        return 1.0

    def grad_fresh(self, p) -> bool:
        """Whether ``p``'s gradient is still logically zero this step (grad_beta would return
        0.0), without consuming that state."""
        return id(p) in self._stale

    @torch.no_grad()
    def zero_grad(self, lazy: bool = False):
        """lazy: gradients that native ops write are only marked zero (their first
        writer overwrites, grad_beta); the rest are cleared now."""
        if not lazy or not self._native:
            self.grad.zero_()
            self._stale.clear()
            return
        others = [s.param for s in self.segments if id(s.param) not in self._native]
        for b, e in (self.ranges(others) if others else []):
            self.grad[b:e].zero_()
        self._stale = set(self._native)

    @torch.no_grad()
    def finalize_grads(self):
        """Clear gradients still marked zero (their op did not run this step) before a
        consumer reads the flat buffer (optimizer, aggregation)."""
        if self._stale:
            for s in self.segments:
                if id(s.param) in self._stale:
                    self.storage_view(s, self.grad).zero_()
            self._stale.clear()

    def reattach_grads(self):
        """Point every ``param.grad`` back at its flat view (after user code set it to None)."""
        for s in self.segments:
            if s.param.grad is None or s.param.grad.data_ptr() != self._logical(s, self.storage_view(s, self.grad)).data_ptr():
                s.param.grad = self._logical(s, self.storage_view(s, self.grad))

    def ranges(self, params) -> list[tuple[int, int]]:
        """Merged [begin, end) element ranges of the given parameters' storage."""
        rs = sorted((self.seg(p).offset, self.seg(p).offset + self.seg(p).storage_numel) for p in params)
        merged: list[list[int]] = []
        for b, e in rs:
            e = (e + _ALIGN - 1) // _ALIGN * _ALIGN
            if merged and b <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], e)
            else:
                merged.append([b, e])
        return [(b, min(e, self.numel)) for b, e in merged]
