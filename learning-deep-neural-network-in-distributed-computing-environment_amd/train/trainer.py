"""The global / local-epoch training driver (§3.2-3.4).

``train_global`` keeps the reference's signature and its 12-history return
contract (BAR/trainer.py:11-192):

   1 all_workers_losses         [N][*]        per-batch train losses per worker (rank 0)
   2 all_epochs_losses          [Eg*El][*]    all workers' batch losses per local epoch (rank 0)
   3 global_epoch_losses        [Eg][*]       all batch losses of each global epoch (rank 0)
   4 global_epoch_accuracies    [Eg][El]      worker-mean train accuracy per local epoch (rank 0)
   5-8 global_{train,val}_{losses,accuracies}  [Eg] means over workers and local epochs (all ranks)
   9-12 worker_specific_{train,val}_{losses,accuracies}  [Eg*El] rank-0 values (rank 0)

What changes is how it runs on MI355X:
* the hot loop (train_local_epoch, BAR/trainer.py:194-223) has no host syncs:
  loss / correct counts / per-batch losses accumulate on the device and are
  read once per local epoch;
* metric exchange is batched: instead of 6 collectives per local epoch
  (C3-C6) every rank packs its local-epoch metrics and batch
  losses and ONE all-gather per global epoch delivers everything;
* aggregation is either the reference schedule (``sync_every="global_epoch"``:
  once per global epoch on gradients or weights, with all-reduce, ring or
  double-ring topology) or real data parallelism (``sync_every="step"``:
  bucketed RCCL all-reduce -- or ring / double-ring gossip -- of gradients every
  step, overlapped with backward);
* the straggler time limit works (train/straggler.py);
* re-partitioning uses a seeded RNG and a selectable share rule.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..data.loader import get_subset_loaders
from ..models.layers import CrossEntropyLoss as LdnnCE
from ..parallel.aggregation import Aggregator
from ..utils.tracing import PhaseTimer, null_timer, trace_range
from ..parallel.comm import MAX, MIN, SUM, Comm, default_comm
from .straggler import StopLocalTraining, StragglerCutoff
from .validator import validate


def _progress(it, enabled, desc):
    if not enabled:
        return it
    try:
        from tqdm import tqdm

        return tqdm(it, desc=desc)
    except Exception:  # pragma: no cover
        return it


def train_local_epoch(model, trainloader, criterion, optimizer, device, scheduler=None, *, dp=None,
                      step_aggregator=None, cutoff: StragglerCutoff | None = None, max_steps: int | None = None,
                      step_scheduler: bool = True, timer: PhaseTimer | None = None, graphs: bool = False,
                      check_comm=None, check_every: int = 50, dp_tail: bool = False):
    """One pass over the rank's shard.  Returns (mean loss, accuracy %, per-batch losses).

    ``timer`` (utils.tracing.PhaseTimer) brackets forward / backward / grad_sync /
    optimizer with roctx ranges and HIP events (BAR/trainer.py:194-223 has none).
    ``graphs``: replay each full-size step from hipGraphs (train/graphed.py): one graph
    for a single-process step; with per-step data parallelism (``dp``) one graph whose
    side-stream branch runs the bucket RCCL all-reduces beside the backward
    (GraphedDPStep).
    ``check_comm``: with per-step synchronisation, cross-check the ranks' collective
    schedules every ``check_every`` steps (Comm.check_schedule).
    ``dp_tail`` (per-step DP, shards of unequal batch counts): after the ``max_steps``
    common steps every rank runs ONE more sample-count-weighted step on its next batch,
    or -- its shard exhausted -- a zero-weight step that only takes part in the
    collectives, so no rank's samples are dropped beyond one batch (the reference trains
    every batch of its shard, BAR/trainer.py:202-216).
    """
    from .engine_adapter import EngineModule, engine_local_epoch

    if isinstance(model, EngineModule):   # the static MLP engine (train/engine_adapter.py)
        out = engine_local_epoch(model, trainloader, optimizer, scheduler, cutoff=cutoff, max_steps=max_steps,
                                 step_scheduler=step_scheduler, check_comm=check_comm, check_every=check_every)
        train_local_epoch.last_samples = engine_local_epoch.last_samples
        return out
    tm = timer or null_timer()
    model.train()
    dev = torch.device(device)
    nb = len(trainloader) if max_steps is None else min(len(trainloader), max_steps)
    losses = torch.zeros(max(nb, 1), dtype=torch.float32, device=dev)
    stats = torch.zeros(2, dtype=torch.float32, device=dev)
    total, done = 0, 0
    ldnn_ce = isinstance(criterion, LdnnCE)
    use_graph = (graphs and dev.type == "cuda" and step_aggregator is None and ldnn_ce and timer is None)
    # equal-average per-step DP: the epoch's LAST step may be short on some ranks (shards of
    # unequal length, the trailing partial batch).  Every rank exchanges its sample count
    # there and scales its loss by n_rank * N / n_total, so the 1/N-averaged gradient is the
    # mean over all ranks' samples -- what one process on the concatenated batch computes
    # (static-engine twin: StaticMLPEngine.dp_tail_step).
    weigh_last = (dp is not None and dp.comm.world_size > 1 and step_aggregator is None
                  and getattr(dp.bucketer, "averaging", False))

    def weight_of(n):
        cnt = torch.tensor([float(n)], dtype=torch.float32, device=dev)
        dp.comm.all_reduce(cnt, SUM)
        return n * dp.comm.world_size / max(float(cnt.item()), 1.0)

    dp_tail = dp_tail and weigh_last
    it = iter(trainloader)
    batches = ((i, b) for i, b in enumerate(it))
    last = pending = None
    try:
        for i, (x, y) in batches:
            if i >= nb:
                pending = (x, y)   # (the tail step's batch, already drawn from the iterator)
                break
            last = (x, y)
            scale = 1.0
            if weigh_last and i == nb - 1:
                scale = weight_of(y.numel())
            if use_graph and scale == 1.0 and (i > 0 or getattr(model, "_ldnn_graphed", None) is not None):
                # the first batch ran eagerly (momentum / optimizer state exist), so the
                # capture needs no extra warmup steps and training semantics are unchanged
                gs = _graphed_step(model, criterion, optimizer, x, y, dp)
                if x.shape == gs.x.shape:
                    losses[i] = gs(x, y).detach().float()
                    total += y.numel()
                    done += 1
                    if cutoff is not None:
                        cutoff.step(i)
                    if check_comm is not None and (i + 1) % check_every == 0:
                        check_comm.check_schedule(f"step {i + 1}", dev if check_comm.device_collectives else None)
                    continue
            optimizer.zero_grad()
            with tm.phase("forward"):
                out = model(x)
                if ldnn_ce:
                    loss = criterion(out, y, stats)
                else:
                    loss = criterion(out.float(), y)
                    with torch.no_grad():
                        stats[1] += (out.argmax(1) == y).sum()
            with tm.phase("backward"):
                (loss if scale == 1.0 else loss * scale).backward()
            if dp is not None or step_aggregator is not None:
                with tm.phase("grad_sync"):
                    if dp is not None:
                        dp.finish_gradient_sync()
                    if step_aggregator is not None:
                        step_aggregator(model)
            with tm.phase("optimizer"):
                optimizer.step()
            losses[i] = loss.detach().float()
            total += y.numel()
            done += 1
            if cutoff is not None:
                cutoff.step(i)
            if check_comm is not None and (i + 1) % check_every == 0:
                check_comm.check_schedule(f"step {i + 1}", dev if check_comm.device_collectives else None)
        if dp_tail and last is not None:
            nxt = pending if pending is not None else next(it, None)
            x, y = nxt if nxt is not None else last
            n = y.numel() if nxt is not None else 0
            scale = weight_of(n)
            if n:
                optimizer.zero_grad()
                out = model(x)
                loss = criterion(out, y, stats) if ldnn_ce else criterion(out.float(), y)
                if not ldnn_ce:
                    with torch.no_grad():
                        stats[1] += (out.argmax(1) == y).sum()
                (loss * scale).backward()
            else:
                # shard exhausted: a zero-weight step that only joins the collectives -- no
                # forward (BatchNorm running statistics would see a duplicate batch) and no
                # loss * 0 backward (a non-finite loss would put NaN into every rank's sum)
                optimizer.zero_grad(set_to_none=False)
                dp.flat.zero_grad(lazy=False)
                dp.wait_gathers()
                dp.bucketer.prepare()
            dp.finish_gradient_sync()
            optimizer.step()
            if n:
                losses = torch.cat([losses[:done], loss.detach().float().reshape(1)])
                total += n
                done += 1
    except StopLocalTraining:
        if step_scheduler and scheduler is not None:
            scheduler.step()
        if dp is not None:
            dp.wait_gathers()
        raise
    if step_scheduler and scheduler is not None:
        scheduler.step()
    if dp is not None:
        dp.wait_gathers()   # sharded DP: the last step's weight all-gathers land before any reader
    gs = getattr(model, "_ldnn_graphed", None) if use_graph else None
    if gs is not None:
        gs.flush_stats(stats)
    batch_losses = losses[:done].tolist()  # the one host sync of the epoch
    correct = stats[1].item()
    train_local_epoch.last_samples = total
    train_loss = float(np.mean(batch_losses)) if batch_losses else 0.0
    return train_loss, 100.0 * correct / max(total, 1), batch_losses


train_local_epoch.last_samples = 0


def _graphed_step(model, criterion, optimizer, x, y, dp=None):
    """The model's cached GraphedStep / GraphedDPStep (captured on the first graphed batch)."""
    from .graphed import GraphedDPStep, GraphedStep

    gs = getattr(model, "_ldnn_graphed", None)
    if gs is None or gs.optimizer is not optimizer or gs.criterion is not criterion or getattr(gs, "dp", None) is not dp:
        if dp is not None:
            gs = GraphedDPStep(dp, criterion, optimizer, x, y)
        else:
            gs = GraphedStep(model, criterion, optimizer, x, y, warmup=0)
        model._ldnn_graphed = gs
    return gs


def loader_seed(seed: int, rank: int, global_epoch: int) -> int:
    """Seed of a rank's training loader for a global epoch (augmentation draws): a
    pure function of (seed, rank, epoch), so a resumed run replays the same draws."""
    return (seed * 1_000_003 + rank * 10_007 + global_epoch * 101) & 0x7FFFFFFF


def _plain(x):
    """Checkpoint round trip (weights_only) turns numpy RNG state leaves into tensors / str keys."""
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    if torch.is_tensor(x):
        return x.item() if x.numel() == 1 else x.tolist()
    return x


_HDR = 2   # [n local epochs done, samples trained this global epoch]


def _pack(local_records, batch_losses_per_epoch, E_l, max_len, device, samples: int = 0):
    """[n_done, samples, (loss, acc, vloss, vacc) x E_l, (len, losses padded to max_len) x E_l]"""
    buf = torch.full((_HDR + 4 * E_l + E_l * (1 + max_len),), -1.0, dtype=torch.float64)
    buf[0] = len(local_records)
    buf[1] = samples
    for e, rec in enumerate(local_records):
        buf[_HDR + 4 * e: _HDR + 4 + 4 * e] = torch.tensor(rec, dtype=torch.float64)
    base = _HDR + 4 * E_l
    for e, bl in enumerate(batch_losses_per_epoch):
        o = base + e * (1 + max_len)
        buf[o] = len(bl)
        if bl:
            buf[o + 1: o + 1 + len(bl)] = torch.tensor(bl, dtype=torch.float64)
    return buf.to(device)


def _unpack(buf, E_l, max_len):
    """-> (records, batch losses per local epoch, samples)"""
    buf = buf.cpu()
    n = int(buf[0].item())
    recs = [tuple(buf[_HDR + 4 * e: _HDR + 4 + 4 * e].tolist()) for e in range(n)]
    base = _HDR + 4 * E_l
    bls = []
    for e in range(n):
        o = base + e * (1 + max_len)
        ln = int(buf[o].item())
        bls.append(buf[o + 1: o + 1 + ln].tolist())
    return recs, bls, int(buf[1].item())


def train_global(model, trainloader, val_loader, trainset, valset, indices_train, indices_val, criterion, optimizer,
                 scheduler, device, rank, world_size, num_local_epochs, num_global_epochs, timelimit, batch_size,
                 prev_fraction, next_fraction, local_weight=0.5, aggregation_type="equal",
                 aggregation_by="gradients", *, comm: Comm | None = None, topology: str = "allreduce",
                 fixed_classes=None, fixed_ratio=None, sync_every: str = "global_epoch", dp=None,
                 partition_rule: str = "reference_duration", repartition: bool = True, replace: bool = False,
                 seed: int = 0, legacy_gossip: bool = False, average_buffers: bool = False,
                 check_every: int = 20, progress: bool = True, logger=None, checkpointer=None,
                 start_global_epoch: int = 0, histories=None, dtype=torch.float32, verbose: bool = True,
                 timer: PhaseTimer | None = None, graphs: bool = False, rng_state=None,
                 ref_samples_per_s: float | None = None):
    """``rng_state`` (resume): the re-partition RNG state saved in the checkpoint's
    ``extra`` -- with it, a resumed run draws the same shards as an uninterrupted one.

    Throughput reporting (``logger``): every global epoch logs the samples trained
    by all ranks, whole-job samples/s over the epoch's wall time (training,
    validation, exchange, aggregation, barrier) and, given ``ref_samples_per_s``
    (one GPU's measured rate for the same model / batch), the data-parallel scaling
    efficiency = samples/s / (N x ref)."""
    comm = comm or default_comm()
    tm = timer or null_timer()
    N = comm.world_size
    dev = torch.device(device)
    rng = np.random.default_rng(seed * 7919 + rank)
    if rng_state is not None:
        rng.bit_generator.state = _plain(rng_state)
    H = histories or {
        "all_workers_losses": [[] for _ in range(N)],
        "all_epochs_losses": [],
        "global_epoch_losses": [],
        "global_epoch_accuracies": [],
        "global_train_losses": [],
        "global_train_accuracies": [],
        "global_val_losses": [],
        "global_val_accuracies": [],
        "worker_specific_train_losses": [],
        "worker_specific_train_accuracies": [],
        "worker_specific_val_losses": [],
        "worker_specific_val_accuracies": [],
    }
    aggregator = Aggregator(topology, aggregation_type, aggregation_by, local_weight, comm, legacy_gossip,
                            average_buffers)
    step_aggregator = None
    if sync_every == "step" and dp is None:
        # per-step decentralised SGD without a DataParallel wrapper (CPU / legacy_gossip
        # runs): gossip (or all-reduce) the whole gradient every step, eagerly
        step_aggregator = Aggregator(topology, aggregation_type, "gradients", local_weight, comm, legacy_gossip)
    cutoff = StragglerCutoff(comm, timelimit, check_every, dev)

    for global_epoch in _progress(range(start_global_epoch, num_global_epochs), progress and rank == 0,
                                  "Global Epochs"):
        t_start = time.perf_counter()
        cutoff.reset()
        max_steps = None
        dp_tail = False
        if sync_every == "step" and N > 1 or getattr(model, "engine", None) is not None and model.engine.distributed:
            # per-step collectives need the same number of steps on every rank
            nsteps = model.full_batches(trainloader) if hasattr(model, "full_batches") else len(trainloader)
            t = torch.tensor([float(nsteps), -float(nsteps)], device=dev)
            comm.all_reduce(t, MIN)
            max_steps = int(t[0].item())
            dp_tail = -int(t[1].item()) > max_steps   # a rank holds more batches: one weighted tail step
        records, batch_losses, samples = [], [], 0
        for local_epoch in range(num_local_epochs):
            try:
                loss, acc, bl = train_local_epoch(model, trainloader, criterion, optimizer, dev, scheduler, dp=dp,
                                                  step_aggregator=step_aggregator, cutoff=cutoff,
                                                  max_steps=max_steps, timer=timer, graphs=graphs,
                                                  check_comm=comm if (sync_every == "step" and N > 1) else None,
                                                  check_every=max(check_every, 1) * 5, dp_tail=dp_tail)
            except StopLocalTraining:
                # cut by the collective time limit: keep LR schedules aligned across ranks
                for _ in range(num_local_epochs - local_epoch - 1):
                    if scheduler is not None:
                        scheduler.step()
                break
            samples += train_local_epoch.last_samples
            with tm.phase("validate"):
                val_loss, val_acc = validate(model, val_loader, criterion, dev)
            records.append((loss, acc, val_loss, val_acc))
            batch_losses.append(bl)
            if verbose:
                print(f"Rank {rank}, Global Epoch {global_epoch + 1}, Local Epoch {local_epoch + 1}, "
                      f"Loss: {loss}, Accuracy: {acc}")
                print(f"Worker {rank}, Global Epoch {global_epoch + 1}, Validation Loss: {val_loss:.4f}, "
                      f"Validation Accuracy: {val_acc:.2f}%")
        cutoff.finish()
        if dp is not None and getattr(dp, "sharded", False):
            dp.gather_master(optimizer)   # sharded DP: whole master for aggregation / checkpoint / eval

        # ---- one metric exchange per global epoch (replaces C3-C6 per local epoch)
        lt = torch.tensor([float(max([len(b) for b in batch_losses] + [0]))], device=dev)
        comm.all_reduce(lt, MAX)
        max_len = int(lt.item())
        packed = _pack(records, batch_losses, num_local_epochs, max_len, dev, samples)
        gathered = comm.all_gather(packed) if N > 1 else [packed]
        per_rank = [_unpack(g, num_local_epochs, max_len) for g in gathered]
        samples_per_rank = [pr[2] for pr in per_rank]
        total_samples = sum(samples_per_rank)
        # every rank must have issued the same collectives so far (RankDivergenceError otherwise)
        comm.check_schedule(f"global epoch {global_epoch + 1}", dev if getattr(comm, "device_collectives", False)
                            else None)

        if rank == 0:
            cur_losses, cur_accs = [], []
            for e in range(num_local_epochs):
                ranks_e = [r for r in range(N) if len(per_rank[r][0]) > e]
                if not ranks_e:
                    continue
                ep_losses = []
                for r in ranks_e:
                    H["all_workers_losses"][r].extend(per_rank[r][1][e])
                    ep_losses.extend(per_rank[r][1][e])
                H["all_epochs_losses"].append(ep_losses)
                cur_losses.extend(ep_losses)
                cur_accs.append(float(np.mean([per_rank[r][0][e][1] for r in ranks_e])))
            for rec in per_rank[0][0]:
                H["worker_specific_train_losses"].append(rec[0])
                H["worker_specific_train_accuracies"].append(rec[1])
                H["worker_specific_val_losses"].append(rec[2])
                H["worker_specific_val_accuracies"].append(rec[3])
            H["global_epoch_losses"].append(cur_losses)
            H["global_epoch_accuracies"].append(cur_accs)
        all_recs = [rec for r in range(N) for rec in per_rank[r][0]]
        if all_recs:
            arr = np.asarray(all_recs, dtype=np.float64)
            means = arr.mean(0)
        else:
            means = np.zeros(4)
        H["global_train_losses"].append(float(means[0]))
        H["global_train_accuracies"].append(float(means[1]))
        H["global_val_losses"].append(float(means[2]))
        H["global_val_accuracies"].append(float(means[3]))

        # ---- end-of-global-epoch aggregation (reference schedule, A27)
        prep = getattr(model, "prepare_collective_read", None)
        if prep is not None:   # e.g. a sharded static engine: whole master on every rank
            prep()
        if sync_every == "global_epoch" or (sync_every == "step" and aggregation_by == "weights"):
            with tm.phase("aggregate"):
                aggregator(model)

        if rank == 0 and progress and verbose:
            print(f"[global epoch {global_epoch + 1}] train loss {means[0]:.4f} acc {means[1]:.2f}% | "
                  f"val loss {means[2]:.4f} acc {means[3]:.2f}%")

        # ---- sync + timing + re-partition (A30, A15/A16)
        with trace_range("barrier"):
            comm.barrier()
        duration = time.perf_counter() - t_start
        if repartition and prev_fraction + next_fraction > 0:
            if partition_rule == "reference_duration":
                td = torch.tensor([duration], dtype=torch.float64, device=dev)
                comm.all_reduce(td, SUM)
                share = duration / max(td.item(), 1e-12)
            else:
                dts = comm.all_gather(torch.tensor([duration], dtype=torch.float64, device=dev))
                from ..data.partition import shares_from_durations

                share = shares_from_durations([float(d.item()) for d in dts], partition_rule)[rank]
            trainloader, val_loader, indices_train, indices_val = get_subset_loaders(
                trainset, valset, indices_train, indices_val, batch_size, prev_fraction, next_fraction, share, dev,
                rng, replace, fixed_classes, fixed_ratio, dtype=dtype,
                augment=getattr(trainloader, "augment", False), augment_val=bool(getattr(val_loader, "mode", 0)),
                loader_seed=loader_seed(seed, rank, global_epoch + 1))
        if logger is not None:
            logger.log(kind="global_epoch", global_epoch=global_epoch + 1, duration_s=duration,
                       train_loss=H["global_train_losses"][-1], train_acc=H["global_train_accuracies"][-1],
                       val_loss=H["global_val_losses"][-1], val_acc=H["global_val_accuracies"][-1],
                       n_local_epochs_done=len(records), cut_by_time_limit=cutoff.cut,
                       shard_size=len(indices_train), samples=total_samples,
                       samples_per_s=total_samples / max(duration, 1e-12),
                       train_samples_per_s_per_rank=[s_ / max(duration, 1e-12) for s_ in samples_per_rank],
                       **({"scaling_efficiency": total_samples / max(duration, 1e-12) / (N * ref_samples_per_s)}
                          if ref_samples_per_s else {}))
        if checkpointer is not None:
            checkpointer.save(global_epoch + 1, model, optimizer, scheduler, H,
                              extra=dict(indices_train=np.asarray(indices_train),
                                         indices_val=np.asarray(indices_val), fixed_classes=fixed_classes,
                                         rng_state=rng.bit_generator.state))
    train_global.last_loaders = (trainloader, val_loader, indices_train, indices_val)
    return (H["all_workers_losses"], H["all_epochs_losses"], H["global_epoch_losses"], H["global_epoch_accuracies"],
            H["global_train_losses"], H["global_train_accuracies"], H["global_val_losses"],
            H["global_val_accuracies"], H["worker_specific_train_losses"], H["worker_specific_train_accuracies"],
            H["worker_specific_val_losses"], H["worker_specific_val_accuracies"])
