"""The static MLP engine behind the reference's training API.

The reference drives one model through ``train_global`` -> ``train_local_epoch``
(BAR/main.py:57-59, BAR/trainer.py:11,194-223) with an ``optimizer`` and a
``StepLR`` scheduler.  ``StaticMLPEngine`` (train/static_mlp.py) is the fast
MI355X step for the MLP configs -- graph-replayed native kernels, fused loss,
fused optimizer and, with per-step data parallelism, its own bucketed RCCL
reduce-scatter / sharded update / all-gather -- but it owns its optimizer state
and steps a fixed batch shape.  Two adapters let the unchanged driver run it:

* ``EngineModule`` -- an ``nn.Module`` holding the MLP (whose parameters are
  views of the engine's flat fp32 master) and the engine.  ``forward`` is the
  MLP's own forward on the engine's bf16 shadow (validate / evaluate / probe);
  ``state_dict`` gathers a sharded master first and returns the MLP's own keys
  (``layers.0.weight`` ...), so checkpoints load into a plain ``mlp3``.
* ``EngineOptimizer`` -- a ``torch.optim.Optimizer`` over the same parameters:
  ``StepLR`` and ``param_groups[0]['lr']`` work as in the reference; its
  ``state_dict`` carries the engine's momentum / Adam moments (gathered from the
  shards) and ``load_state_dict`` puts them back.  ``step()`` is a no-op: the
  engine's fused update runs inside its step.

``train_local_epoch`` recognises an ``EngineModule`` and runs ``engine_local_epoch``:
one ``load_batch`` + ``step`` per full batch, the per-batch losses read from the
engine's on-device statistics (one small reduction per step, one host read per
epoch).  A trailing partial batch is trained too, as the reference does
(BAR/trainer.py:202-216): the engine's shapes are static, so it runs
``StaticMLPEngine.eager_step`` (autograd on the same flat parameters + the fused
update).  A data-parallel engine runs the same number of full steps on every rank
(the minimum over the ranks), then ONE tail step on every rank
(``StaticMLPEngine.dp_tail_step``: each rank's next batch of any size -- its
partial batch, or none -- weighted by its sample count, so the update is the mean
over all ranks' samples).  Batches beyond that (shards of unequal length) are
reported as ``engine_local_epoch.last_skipped``.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .static_mlp import OptimConfig, StaticMLPEngine
from .straggler import StopLocalTraining


class EngineModule(nn.Module):
    def __init__(self, model: nn.Module, engine: StaticMLPEngine):
        super().__init__()
        self.module = model
        self.__dict__["engine"] = engine   # not a submodule: state_dict keys stay the MLP's

    def forward(self, x):
        self.engine.sync()   # the previous step's weight all-gathers (sharded DP)
        return self.module(x)

    def state_dict(self, *args, **kwargs):
        self.engine.gather_master()
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        r = self.module.load_state_dict(state_dict, strict=strict)
        self.engine.flat.refresh_shadow()
        return r

    def prepare_collective_read(self):
        """Collective (every rank): make the sharded master / optimizer state whole, so a
        rank-0-only state_dict() / checkpoint afterwards issues no collective."""
        self.engine.gather_master()

    def full_batches(self, loader) -> int:
        return int(loader.num_samples) // self.engine.B if hasattr(loader, "num_samples") else len(loader)


class EngineOptimizer(torch.optim.Optimizer):
    def __init__(self, engine: StaticMLPEngine, params):
        o = engine.optim
        defaults = dict(lr=o.lr)
        if o.name == "sgd":
            defaults.update(momentum=o.momentum, dampening=o.dampening, weight_decay=o.weight_decay,
                            nesterov=o.nesterov)
        else:
            defaults.update(betas=o.betas, eps=o.eps, weight_decay=o.weight_decay)
        super().__init__(params, defaults)
        self.__dict__["engine"] = engine

    @torch.no_grad()
    def step(self, closure=None):   # the engine's step runs the fused update
        return closure() if closure is not None else None

    def zero_grad(self, set_to_none: bool = True):   # the update kernels clear the gradients
        pass

    def sync_hyperparams(self):
        self.engine.set_lr(self.param_groups[0]["lr"])

    def state_dict(self):
        sd = super().state_dict()
        sd["ldnn_engine_state"] = self.engine.optimizer_state()
        return sd

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        es = state_dict.pop("ldnn_engine_state", None)
        super().load_state_dict(state_dict)
        if es is not None:
            self.engine.load_optimizer_state(es)
        self.sync_hyperparams()


def build_engine(model, batch_size: int, optimizer: str, lr: float, device, *, momentum: float = 0.9,
                 weight_decay: float = 0.0, world_size: int = 1, process_group=None, use_graphs: bool = True,
                 bucket_cap_elems: int = 8 << 20, grad_mix: tuple | None = None):
    """(EngineModule, EngineOptimizer) for an ldnn MLP.  ``world_size`` > 1 = per-step
    data parallelism inside the engine (reduce-scatter + sharded update + all-gather
    over RCCL); 1 = an independent replica (the reference's global-epoch schedule
    aggregates it through the Aggregator like any other model).  ``grad_mix`` =
    (hops, local_weight): per-step ring / double-ring gossip or the self-weighted
    all-reduce inside the engine (StaticMLPEngine)."""
    name = optimizer.lower()
    oc = (OptimConfig("sgd", lr=lr, momentum=momentum, weight_decay=weight_decay) if name == "sgd"
          else OptimConfig(name, lr=lr, weight_decay=weight_decay))
    eng = StaticMLPEngine(model, batch_size, oc, device=device, world_size=world_size, process_group=process_group,
                          use_graphs=use_graphs, bucket_cap_elems=bucket_cap_elems, grad_mix=grad_mix)
    return EngineModule(model, eng), EngineOptimizer(eng, model.parameters())


def engine_local_epoch(model: EngineModule, trainloader, optimizer, scheduler=None, *, cutoff=None,
                       max_steps: int | None = None, step_scheduler: bool = True, check_comm=None,
                       check_every: int = 50):
    """train_local_epoch for an EngineModule: (mean loss, accuracy %, per-batch losses)."""
    eng = model.engine
    dev = eng.device
    if isinstance(optimizer, EngineOptimizer):
        optimizer.sync_hyperparams()
    else:
        eng.set_lr(optimizer.param_groups[0]["lr"])
    model.train()
    nb = model.full_batches(trainloader)
    if max_steps is not None:
        nb = min(nb, max_steps)
    dist_ = eng.distributed
    # cum[i] = running (loss sum, #correct) after step i -- one tiny reduction per step
    cum = torch.zeros(max(nb, 1) + 2, 2, dtype=torch.float64, device=dev)
    sizes = []
    eng.reset_stats()
    done, skipped, tail, steps = 0, 0, False, 0

    def record(n):
        nonlocal done
        sizes.append(n)
        torch.sum(eng.stats, 0, dtype=torch.float64, out=cum[len(sizes)])
        done += 1

    def after_step():
        # (counts every step incl. a sample-less tail step: the collective checks stay aligned)
        nonlocal steps
        steps += 1
        if cutoff is not None:
            cutoff.step(steps - 1)
        if check_comm is not None and steps % check_every == 0:
            check_comm.check_schedule(f"step {steps}", dev if check_comm.device_collectives else None)

    total = int(trainloader.num_samples) if hasattr(trainloader, "num_samples") else None
    seen = 0
    try:
        for x, y in trainloader:
            seen += y.numel()
            if done < nb and y.numel() == eng.B:
                eng.load_batch(x, y)
                eng.step()
                record(y.numel())
                after_step()
                continue
            # the first batch past the full steps: the trailing partial batch (or, under
            # data parallelism, this rank's next batch of any size) -- at most one tail step
            tail = True
            if dist_:
                eng.dp_tail_step(x, y)   # collective: every rank runs exactly one
                record(y.numel())
                after_step()
            elif y.numel() != eng.B:
                eng.eager_step(x, y)
                record(y.numel())
                after_step()
            else:
                seen -= y.numel()
            break
        if dist_ and not tail:   # this rank's shard ran out: take part in the tail step with no samples
            tail = True
            eng.dp_tail_step(None, None)
            after_step()
        skipped = (total - sum(sizes)) if total is not None else max(seen - sum(sizes), 0)
    except StopLocalTraining:
        if isinstance(optimizer, EngineOptimizer):
            optimizer.step()   # a no-op; keeps torch's scheduler-order check quiet
        if step_scheduler and scheduler is not None:
            scheduler.step()
        _finish(model, done, skipped, sizes)
        raise
    if isinstance(optimizer, EngineOptimizer):
        optimizer.step()   # a no-op (the engine's fused update ran): keeps the scheduler-order contract
    if step_scheduler and scheduler is not None:
        scheduler.step()
    return _finish(model, done, skipped, sizes, cum)


def _finish(model, done, skipped, sizes, cum=None):
    engine_local_epoch.last_skipped = skipped
    engine_local_epoch.last_samples = sum(sizes)
    if cum is None or done == 0:
        return 0.0, 0.0, []
    c = cum[: done + 1].cpu()   # the one host sync of the epoch
    model.engine.sync()
    per = (c[1:, 0] - c[:-1, 0]) / torch.tensor(sizes, dtype=torch.float64)
    losses = per.tolist()
    correct = float(c[done, 1])
    return float(per.mean()), 100.0 * correct / max(sum(sizes), 1), losses


engine_local_epoch.last_skipped = 0
engine_local_epoch.last_samples = 0
