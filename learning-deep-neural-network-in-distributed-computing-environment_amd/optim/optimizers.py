"""Fused optimizers (reference BAR/main.py:53 uses torch.optim.Adam,
BASELINE configs use SGD-momentum).

They are ``torch.optim.Optimizer`` subclasses (so the reference's
``StepLR(optimizer, step_size=25)`` and ``optimizer.param_groups[..]['lr']``
work unchanged), but when the parameters live in a FlatParams buffer the
update is ONE fused kernel over the whole model (fp32 master + momentum /
moments + bf16 shadow refresh, with the data-parallel 1/N folded in) instead
of a per-tensor loop.  Learning rate and Adam's step count are handed to the
kernel through a small device tensor, so the update can sit inside a captured
hipGraph.  Without FlatParams (or on CPU) the same math runs as torch ops.
"""
from __future__ import annotations

import math

import torch

from ..ops import _ext
from ..utils.flat_params import owner_of




def _refuse_partial_sharded(params):
    """A param group that does not map onto one whole FlatParams would take the per-tensor
    update path; on a sharded DataParallel buffer (only this rank's shard of flat.grad is
    reduced, and nothing all-gathers the result) that silently diverges the replicas."""
    for p in params:
        f = owner_of(p)
        if f is not None and getattr(f, "shard_sync", None) is not None:
            raise RuntimeError("DataParallel(shard_optimizer=True): the optimizer's param group must hold "
                               "every parameter of the model's flat buffer (one group, built AFTER the "
                               "DataParallel wrapper)")


class _FlatOptimizer(torch.optim.Optimizer):
    def _ls(self) -> dict:
        """Fused (flat-buffer) optimizer state: momentum / moments / step / hp."""
        return self.__dict__.setdefault("_ldnn_state", {})

    def state_dict(self):
        sd = super().state_dict()
        sd["ldnn_flat_state"] = {k: v for k, v in self._ls().items() if k != "hp"}
        return sd

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        flat_state = state_dict.pop("ldnn_flat_state", {})
        super().load_state_dict(state_dict)
        ls = self._ls()
        ls.clear()
        for k, v in flat_state.items():
            ls[k] = v.clone() if torch.is_tensor(v) else v
        # re-home buffers onto the parameters' device
        for group in self.param_groups:
            f = self._flat_for_group(group)
            if f is not None:
                for k, v in list(ls.items()):
                    if torch.is_tensor(v):
                        ls[k] = v.to(f.master.device)

    def _flat_for_group(self, group):
        ps = group["params"]
        if not ps:
            return None
        f = owner_of(ps[0])
        if f is None or any(owner_of(p) is not f for p in ps) or len(ps) != len(f.segments):
            _refuse_partial_sharded(ps)
            return None
        return f

    def _hp(self, flat, lr):
        st = self._ls()
        hp = st.get("hp")
        if hp is None or hp.device != flat.master.device:
            if getattr(self, "_ldnn_capturing", False):
                raise RuntimeError("run an eager optimizer step before capturing it into a graph")
            hp = torch.zeros(2, dtype=torch.float32, device=flat.master.device)
            hp[1] = float(st.get("step", 0))
            st["hp"] = hp
        # inside a hipGraph capture the lr write is NOT recorded: the graph reads hp,
        # and GraphedStep refreshes it (sync_hyperparams) whenever the lr changes
        if not getattr(self, "_ldnn_capturing", False):
            hp[0].fill_(lr)
        return hp

    @torch.no_grad()
    def sync_hyperparams(self):
        """Write the current learning rate into the device hyper-parameter tensor."""
        hp = self._ls().get("hp")
        if hp is not None:
            hp[0].fill_(self.param_groups[0]["lr"])

    def _buf(self, name, like):
        st = self._ls()
        b = st.get(name)
        if b is None or b.shape != like.shape or b.device != like.device:
            b = torch.zeros_like(like)
            st[name] = b
        return b

    # ---- range updates (optimizer overlapped with the backward, train/graphed.py) ----
    def range_updater(self):
        """A ``_RangeUpdate`` for ONE step of a single flat-buffer group on the GPU
        (None when the optimizer cannot update by ranges: several groups, no
        FlatParams, CPU).  ``update(lo, hi)`` runs the fused kernel on flat elements
        [lo, hi) on the current stream; ``end()`` closes the step.  Every element must
        be covered exactly once per step."""
        if not self.supports_ranges():
            return None
        group = self.param_groups[0]
        return _RangeUpdate(self, self._flat_for_group(group), group)

    def supports_ranges(self) -> bool:
        if len(self.param_groups) != 1 or type(self)._update_range is _FlatOptimizer._update_range:
            return False
        f = self._flat_for_group(self.param_groups[0])
        return f is not None and _ext.use_native(f.master)

    def _begin_ranges(self, f, group):  # per-step setup on the current stream (subclasses)
        return {}

    def _update_range(self, f, group, ctx, lo, hi):
        raise NotImplementedError

    def _sharded_step(self, f, group) -> bool:
        """DataParallel(shard_optimizer=True) owns ``f``: update only this rank's flat
        ranges (its shard of every reduce-scattered bucket + the replicated tail), then
        let the data-parallel wrapper start the weight all-gathers.  False otherwise."""
        sh = getattr(f, "shard_sync", None)
        if sh is None:
            return False
        if len(self.param_groups) != 1:
            # the full-replica update below would read flat.grad, of which only this rank's
            # shards hold reduced values, and no weight all-gather would follow: replicas
            # would silently diverge
            raise RuntimeError("DataParallel(shard_optimizer=True) needs ONE param group holding the whole "
                               f"flat buffer; this optimizer has {len(self.param_groups)}")
        f.finalize_grads()
        ctx = self._begin_ranges(f, group)
        parts = getattr(sh, "step_parts", None)
        if parts is not None:   # the caller interleaves its own work per bucket (GraphedDPStep capture)
            parts(lambda lo, hi: self._update_range(f, group, ctx, lo, hi) if hi > lo else None)
        else:
            for lo, hi in sh.update_ranges():
                if hi > lo:
                    self._update_range(f, group, ctx, lo, hi)
        st = self._ls()
        st["step"] = st.get("step", 0) + 1
        sh.after_update()
        return True

    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            f = self._flat_for_group(group)
            if f is not None:
                # (set_to_none: the next backward's first write overwrites instead of a fill)
                f.zero_grad(lazy=set_to_none)
            else:
                for p in group["params"]:
                    if p.grad is not None:
                        if set_to_none and owner_of(p) is None:
                            p.grad = None
                        else:
                            p.grad.zero_()


class SGD(_FlatOptimizer):
    def __init__(self, params, lr=0.01, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    @torch.no_grad()
    def step(self, closure=None, clear_grads: bool = False):
        """clear_grads: the update kernel also zeroes the flat gradient after reading it
        (one pass instead of a later zero_grad fill; on MI355X the zero writes inside
        the bandwidth-bound update cost about what the fill launch does)."""
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            lr, mu, damp, wd, nest = (group[k] for k in ("lr", "momentum", "dampening", "weight_decay", "nesterov"))
            f = self._flat_for_group(group)
            if f is not None and self._sharded_step(f, group):
                continue
            if f is not None:
                f.finalize_grads()
                st = self._ls()
                first = st.get("step", 0) == 0
                mom = self._buf("momentum", f.master) if mu != 0 else f.master
                if _ext.use_native(f.master):
                    _ext.C().sgd_step(f.master, f.grad, mom, f.shadow, self._hp(f, lr), f.grad_scale, mu, damp, wd,
                                      nest, first, zero_ranges=[(0, f.grad.numel())] if clear_grads else [])
                else:
                    self._sgd_torch(f.master, f.grad * f.grad_scale, mom if mu != 0 else None, lr, mu, damp, wd,
                                    nest, first)
                    if f.shadow is not None:
                        f.shadow.copy_(f.master)
                    if clear_grads:
                        f.grad.zero_()
                st["step"] = st.get("step", 0) + 1
            else:
                for p in group["params"]:
                    if p.grad is None:
                        continue
                    ps = self.state.setdefault(p, {})
                    first = "momentum_buffer" not in ps
                    if mu != 0 and first:
                        ps["momentum_buffer"] = torch.zeros_like(p)
                    self._sgd_torch(p.data, p.grad, ps.get("momentum_buffer"), lr, mu, damp, wd, nest, first)
        return loss

    def _begin_ranges(self, f, group):
        mu = group["momentum"]
        hp = self._hp(f, group["lr"]) if _ext.use_native(f.master) else None
        return dict(hp=hp, first=self._ls().get("step", 0) == 0,
                    mom=self._buf("momentum", f.master) if mu != 0 else f.master)

    def _update_range(self, f, group, ctx, lo, hi):
        sh = f.shadow[lo:hi] if f.shadow is not None else None
        if not _ext.use_native(f.master):
            mu = group["momentum"]
            self._sgd_torch(f.master[lo:hi], f.grad[lo:hi] * f.grad_scale, ctx["mom"][lo:hi] if mu != 0 else None,
                            group["lr"], mu, group["dampening"], group["weight_decay"], group["nesterov"], ctx["first"])
            if sh is not None:
                sh.copy_(f.master[lo:hi])
            return
        _ext.C().sgd_step(f.master[lo:hi], f.grad[lo:hi], ctx["mom"][lo:hi], sh, ctx["hp"], f.grad_scale,
                          group["momentum"], group["dampening"], group["weight_decay"], group["nesterov"],
                          ctx["first"])

    @staticmethod
    def _sgd_torch(p, g, buf, lr, mu, damp, wd, nest, first):
        if wd != 0:
            g = g + wd * p
        if mu != 0:
            if first:
                buf.copy_(g)
            else:
                buf.mul_(mu).add_(g, alpha=1 - damp)
            g = g + mu * buf if nest else buf
        p.add_(g, alpha=-lr)


class Adam(_FlatOptimizer):
    decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None, clear_grads: bool = False):
        """clear_grads: as SGD.step."""
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            f = self._flat_for_group(group)
            if f is not None and self._sharded_step(f, group):
                continue
            if f is not None:
                f.finalize_grads()
                st = self._ls()
                m, v = self._buf("exp_avg", f.master), self._buf("exp_avg_sq", f.master)
                if _ext.use_native(f.master):
                    hp = self._hp(f, lr)
                    _ext.C().bump_step(hp)
                    _ext.C().adam_step(f.master, f.grad, m, v, f.shadow, hp, f.grad_scale, b1, b2, eps, wd,
                                       self.decoupled, zero_ranges=[(0, f.grad.numel())] if clear_grads else [])
                    st["step"] = st.get("step", 0) + 1
                else:
                    st["step"] = st.get("step", 0) + 1
                    self._adam_torch(f.master, f.grad * f.grad_scale, m, v, st["step"], lr, b1, b2, eps, wd)
                    if f.shadow is not None:
                        f.shadow.copy_(f.master)
                    if clear_grads:
                        f.grad.zero_()
            else:
                for p in group["params"]:
                    if p.grad is None:
                        continue
                    ps = self.state.setdefault(p, {})
                    if "exp_avg" not in ps:
                        ps["exp_avg"] = torch.zeros_like(p)
                        ps["exp_avg_sq"] = torch.zeros_like(p)
                        ps["step"] = 0
                    ps["step"] += 1
                    self._adam_torch(p.data, p.grad, ps["exp_avg"], ps["exp_avg_sq"], ps["step"], lr, b1, b2, eps,
                                     wd)
        return loss

    def _begin_ranges(self, f, group):
        hp = None
        if _ext.use_native(f.master):
            hp = self._hp(f, group["lr"])
            _ext.C().bump_step(hp)   # once per step, before any range reads the step count
        return dict(hp=hp, m=self._buf("exp_avg", f.master), v=self._buf("exp_avg_sq", f.master),
                    t=self._ls().get("step", 0) + 1)

    def _update_range(self, f, group, ctx, lo, hi):
        b1, b2 = group["betas"]
        sh = f.shadow[lo:hi] if f.shadow is not None else None
        if not _ext.use_native(f.master):
            self._adam_torch(f.master[lo:hi], f.grad[lo:hi] * f.grad_scale, ctx["m"][lo:hi], ctx["v"][lo:hi],
                             ctx["t"], group["lr"], b1, b2, group["eps"], group["weight_decay"])
            if sh is not None:
                sh.copy_(f.master[lo:hi])
            return
        _ext.C().adam_step(f.master[lo:hi], f.grad[lo:hi], ctx["m"][lo:hi], ctx["v"][lo:hi], sh, ctx["hp"],
                           f.grad_scale, b1, b2, group["eps"], group["weight_decay"], self.decoupled)

    def _adam_torch(self, p, g, m, v, t, lr, b1, b2, eps, wd):
        if wd != 0:
            if self.decoupled:
                p.mul_(1 - lr * wd)
            else:
                g = g + wd * p
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)


class AdamW(Adam):
    decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, lr, betas, eps, weight_decay)


def build_optimizer(name: str, params, lr: float, momentum: float = 0.9, weight_decay: float = 0.0):
    name = name.lower()
    if name == "sgd":
        return SGD(params, lr=lr, momentum=momentum, weight_decay=weight_decay)
    if name == "adam":
        return Adam(params, lr=lr, weight_decay=weight_decay)
    if name == "adamw":
        return AdamW(params, lr=lr, weight_decay=weight_decay)
    raise ValueError(f"unknown optimizer {name!r}")


class _RangeUpdate:
    """One optimizer step applied as several flat-range launches (see
    ``_FlatOptimizer.range_updater``)."""

    def __init__(self, opt, flat, group):
        self.opt, self.flat, self.group = opt, flat, group
        self.ctx = opt._begin_ranges(flat, group)
        self.done = 0

    @torch.no_grad()
    def update(self, lo: int, hi: int):
        if hi > lo:
            self.opt._update_range(self.flat, self.group, self.ctx, lo, hi)
            self.done += hi - lo

    def end(self):
        if self.done != self.flat.numel:
            raise RuntimeError(f"range updates covered {self.done} of {self.flat.numel} flat elements")
        st = self.opt._ls()
        st["step"] = st.get("step", 0) + 1
