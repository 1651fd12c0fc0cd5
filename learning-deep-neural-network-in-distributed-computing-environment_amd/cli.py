"""Command line entry point: the reference's flags (BAR/main.py:83-97,
DAR/main.py:87-103, BR/main.py:77-92, BDR/main.py:77-93) plus the MI355X-native
extensions (SURVEY §5 config row, §7.4 decisions).

Launch (one process per GPU, RCCL over xGMI):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py [flags]
CPU / gloo plumbing runs the same way with --device cpu.

Reference flags kept verbatim: --local-rank, --backend {nccl,gloo,mpi}, --epochs_local,
--epochs_global, --batch_size, --lr, --time_limit, --prev_fraction, --next_fraction,
--aggregation_type {equal,weighted}, --aggregation_by {gradients,weights},
--local_weight, --fixed_ratio, --gpu_weight (accepted, unused as in the reference),
--dist-url (accepted, unused).
"""
from __future__ import annotations

import argparse
import json
import math
import os

import torch


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="ldnn: MI355X-native distributed DNN training")
    # ---- reference flags
    p.add_argument("--local-rank", "--local_rank", type=int, dest="local_rank", default=None)
    p.add_argument("--backend", type=str, default="auto", choices=["auto", "nccl", "gloo", "mpi"],
                   help="process-group backend; nccl = RCCL on ROCm; mpi maps to the default backend")
    p.add_argument("--epochs_local", type=int, default=5)
    p.add_argument("--epochs_global", type=int, default=20)
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--time_limit", type=float, default=60.0)
    p.add_argument("--prev_fraction", type=float, default=0.5)
    p.add_argument("--next_fraction", type=float, default=0.5)
    p.add_argument("--aggregation_type", type=str, default="equal", choices=["equal", "weighted"])
    p.add_argument("--aggregation_by", type=str, default="gradients", choices=["gradients", "weights"])
    p.add_argument("--local_weight", type=float, default=0.5)
    p.add_argument("--fixed_ratio", type=float, default=None,
                   help="class-skewed ('disbalanced') partition with this fraction of fixed classes")
    p.add_argument("--gpu_weight", type=float, default=10, help="accepted for compatibility (unused)")
    p.add_argument("--dist-url", type=str, default=None, help="accepted for compatibility (unused)")
    # ---- extensions
    p.add_argument("--topology", type=str, default="allreduce", choices=["allreduce", "ring", "double_ring"])
    p.add_argument("--partition", type=str, default=None, choices=["balanced", "skewed"],
                   help="skewed requires --fixed_ratio (default 0.5)")
    p.add_argument("--partition_rule", type=str, default="reference_duration",
                   choices=["reference_duration", "throughput", "equal"])
    p.add_argument("--sync_every", type=str, default="global_epoch", choices=["global_epoch", "step"],
                   help="global_epoch = reference schedule (SURVEY Q1); step = per-step data parallelism")
    p.add_argument("--model", type=str, default="enhanced_cnn")
    p.add_argument("--dataset", type=str, default=None, help="cifar10 | mnist | imagenet | imagenet64 (synthetic "
                   "unless the CIFAR-10 binary files exist under --data_root)")
    p.add_argument("--n_train", type=int, default=None)
    p.add_argument("--n_test", type=int, default=None)
    p.add_argument("--data_root", type=str, default="data")
    p.add_argument("--optimizer", type=str, default="adam", choices=["adam", "adamw", "sgd"])
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--step_size", type=int, default=25, help="StepLR step (local epochs), BAR/main.py:54")
    p.add_argument("--gamma", type=float, default=0.1)
    p.add_argument("--dtype", type=str, default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", type=str, default="auto", help="auto | cpu | cuda")
    p.add_argument("--legacy_gossip", action="store_true", help="reproduce the reference's lost GPU gossip update")
    p.add_argument("--average_buffers", action="store_true", help="also average BN buffers in weight averaging")
    p.add_argument("--replace", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                   help="sample the per-global-epoch re-partition with replacement.  auto (default) follows the "
                        "reference variant: on for class-skewed shards (DAR/DR/DDR dataloader.py:123,129) and for "
                        "the balanced double ring (BDR/dataloader.py:94,100), off for BAR/BR")
    p.add_argument("--no_repartition", action="store_true")
    p.add_argument("--check_every", type=int, default=20, help="steps between straggler-cutoff rounds")
    p.add_argument("--bucket_mb", type=float, default=32.0)
    p.add_argument("--grad_comm_dtype", choices=["fp32", "bf16"], default="fp32",
                   help="dtype of the per-step gradient all-reduce (bf16 halves the xGMI bytes)")
    p.add_argument("--shard_optimizer", choices=["auto", "on", "off"], default="auto",
                   help="per-step all-reduce DP of autograd models: reduce-scatter each gradient bucket, run the "
                        "fused optimizer on this rank's 1/N shard, all-gather the bf16 weights (ZeRO-1 style, "
                        "parallel/ddp.py); auto = on for GPU runs with --aggregation_type equal")
    p.add_argument("--oneshot_bytes", type=int, default=None,
                   help="RCCL runs on one node: SUM all-reduces of at most this many bytes use the one-shot IPC "
                        "kernel that reads every peer's copy over its own xGMI link (parallel/ipc.py); opt-in, "
                        "default 0 = off (env LDNN_ONESHOT_BYTES); 4194304 covers LeNet-5's whole gradient")
    p.add_argument("--augment", nargs="?", const="autoaugment", default="none",
                   choices=["none", "autoaugment", "flipcrop", "autoaugment+flipcrop"],
                   help="training-set augmentation in the native input kernel (augment.hip); bare --augment = "
                        "AutoAugment(CIFAR10), the reference's train transform (BAR/dataloader.py:16)")
    p.add_argument("--augment_val", action="store_true",
                   help="also augment the validation shard: the reference's split of an augmented train set "
                        "(BAR/dataloader.py:29-35) does that")
    p.add_argument("--out_dir", type=str, default="runs/latest")
    p.add_argument("--plots", type=str, default="Graphs", help="output folder of the six plots ('' to skip)")
    p.add_argument("--checkpoint_every", type=int, default=0)
    p.add_argument("--resume", type=str, default=None, help="checkpoint path or 'latest'")
    p.add_argument("--timeout", type=float, default=600.0, help="collective timeout (s): failure detection")
    p.add_argument("--no_eval", action="store_true")
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--graphs", dest="graphs", action="store_true", default=True,
                   help="(default) on a GPU, replay each training step from hipGraphs; with --sync_every step the "
                        "backward is a chain of graphs cut at the gradient buckets, each bucket's RCCL all-reduce "
                        "issued between two links (train/graphed.py GraphedDPStep).  CPU runs are always eager")
    p.add_argument("--no_graphs", dest="graphs", action="store_false", help="eager steps (one launch per kernel)")
    p.add_argument("--engine", choices=["auto", "autograd", "static"], default="auto",
                   help="static: MLP models run on the graph-captured static engine (train/static_mlp.py: native "
                        "kernels, fused loss + optimizer, per-step DP = its own RCCL reduce-scatter / sharded update "
                        "/ all-gather); autograd: the generic module path; auto: static for MLPs on a GPU whenever "
                        "the topology / schedule allows it")
    p.add_argument("--ref_samples_per_s", type=float, default=None,
                   help="one GPU's measured samples/s for this model and batch: metrics.jsonl then also logs the "
                        "data-parallel scaling efficiency per global epoch")
    p.add_argument("--trace", action="store_true",
                   help="roctx ranges per phase + HIP-event phase timers (summary in metrics.jsonl)")
    return p


def resolve_replace(flag: str, fixed_ratio, topology: str) -> bool:
    """--replace auto -> the reference variant's sampling (see the flag's help)."""
    if flag == "auto":
        return fixed_ratio is not None or topology == "double_ring"
    return flag == "on"


def resolve_engine(args, model, dev, world: int) -> bool:
    """--engine auto|autograd|static -> run the static MLP engine?"""
    from .models.mlp import MLP
    from .ops import _ext

    why = None
    if not isinstance(model, MLP):
        why = f"--model {args.model} is not an MLP"
    elif dev.type != "cuda" or not _ext.use_native(torch.empty(0, device=dev)):
        why = "the static engine needs the native extension on a GPU"
    elif args.grad_comm_dtype != "fp32":
        why = "--grad_comm_dtype bf16 runs on the autograd path"
    elif args.legacy_gossip and args.sync_every == "step" and args.topology != "allreduce" and world > 1:
        # the static engine's grad_mix always applies the combine (no reference-Q2 mode)
        why = "--legacy_gossip runs on the autograd path"
    if args.engine == "static" and why is not None:
        raise SystemExit(f"--engine static: {why}")
    return args.engine != "autograd" and why is None


def main(argv=None):
    args = build_parser().parse_args(argv)
    from . import prepare
    from .data.loader import get_loaders
    from .models import CrossEntropyLoss, build_model, dataset_for, xavier_init
    from .optim import StepLR, build_optimizer
    from .parallel.comm import default_comm
    from .parallel.ddp import DataParallel
    from .train.trainer import train_global
    from .train.validator import evaluate
    from .utils import distributed as D
    from .utils.checkpoint import Checkpointer, load_checkpoint
    from .utils.metrics import MetricsLogger

    backend = None if args.backend in ("auto", "mpi") else args.backend
    ctx = D.setup(backend, timeout_s=args.timeout, device=None if args.device == "auto" else args.device)
    rank, world = ctx.rank, ctx.world_size
    dev = ctx.device
    torch.manual_seed(args.seed)
    comm = default_comm(args.oneshot_bytes)

    dataset = args.dataset or dataset_for(args.model)
    model = build_model(args.model)
    xavier_init(model)
    use_engine = resolve_engine(args, model, dev, world)
    if use_engine:
        from .train.engine_adapter import build_engine

        step_dp = args.sync_every == "step" and world > 1
        hops = {"allreduce": 0, "ring": 1, "double_ring": 2}[args.topology]
        lw = args.local_weight if args.aggregation_type == "weighted" else None
        net, optimizer = build_engine(model.to(dev), args.batch_size, args.optimizer, args.lr, dev,
                                      momentum=args.momentum, weight_decay=args.weight_decay,
                                      world_size=world if step_dp else 1, use_graphs=True,
                                      bucket_cap_elems=int(args.bucket_mb * (1 << 20)) // 4,
                                      grad_mix=(hops, lw) if step_dp else None)
        flat = net.engine.flat
    else:
        flat = prepare(model, dev)
    fixed_ratio = args.fixed_ratio
    if args.partition == "skewed" and fixed_ratio is None:
        fixed_ratio = 0.5
    if args.partition == "balanced":
        fixed_ratio = None

    replace = resolve_replace(args.replace, fixed_ratio, args.topology)

    dp = None
    if use_engine:   # the engine synchronises its own gradients (per-step DP) or is a plain replica
        D.broadcast_module(model)
        flat.refresh_shadow()
    elif args.sync_every == "step" and world > 1:
        # (--grad_comm_dtype bf16: all-reduce / reduce-scatter buckets and the gossip exchange travel
        # as bf16 copies of the fp32 gradient)
        weighted = args.aggregation_type == "weighted"
        gossip = {"allreduce": 0, "ring": 1, "double_ring": 2}[args.topology]
        if args.shard_optimizer == "on" and (weighted or gossip):
            raise SystemExit("--shard_optimizer on needs --topology allreduce --aggregation_type equal (the "
                             "weighted mix and gossip give every rank its own update)")
        shard = not weighted and not gossip and (args.shard_optimizer == "on" or (args.shard_optimizer == "auto"
                                                                                   and dev.type == "cuda"))
        dp = DataParallel(model, comm, bucket_cap_mb=args.bucket_mb,
                          local_weight=args.local_weight if weighted else None,
                          comm_dtype=torch.bfloat16 if args.grad_comm_dtype == "bf16" else None,
                          shard_optimizer=shard, gossip=gossip, legacy_gossip=args.legacy_gossip)
        flat = dp.flat   # (sharding re-lays the flat buffers out)
    else:  # reference A6: broadcast every state_dict entry from rank 0
        D.broadcast_module(model)
        flat.refresh_shadow()
    if not use_engine:
        net = dp if dp is not None else model

    dtype = torch.bfloat16 if (args.dtype == "bf16" and dev.type == "cuda") else torch.float32
    loaders = get_loaders(args.batch_size, world, rank, net, dev, fixed_ratio, dataset=dataset, comm=comm,
                          seed=args.seed, partition_rule=args.partition_rule, n_train=args.n_train,
                          n_test=args.n_test, dtype=dtype, augment=args.augment, data_root=args.data_root,
                          augment_val=args.augment_val)
    train_loader, val_loader, test_loader, trainset, valset, tr_idx, va_idx = loaders[:7]
    fixed_classes = loaders[7] if len(loaders) > 7 else None

    criterion = CrossEntropyLoss()
    if not use_engine:
        optimizer = build_optimizer(args.optimizer, model.parameters(), args.lr, args.momentum, args.weight_decay)
    scheduler = StepLR(optimizer, step_size=args.step_size, gamma=args.gamma)

    os.makedirs(args.out_dir, exist_ok=True)
    logger = MetricsLogger(os.path.join(args.out_dir, "metrics.jsonl"), rank)
    logger.log(kind="config", world_size=world, pg_backend=ctx.backend, resolved_device=str(dev),
               resolved_engine="static" if use_engine else "autograd", **vars(args))
    per_rank = args.topology != "allreduce" or args.sync_every == "global_epoch"
    ckpt = Checkpointer(os.path.join(args.out_dir, "ckpt"), rank, per_rank=per_rank,
                        every=args.checkpoint_every) if args.checkpoint_every > 0 else None
    start, hist, rng_state = 0, None, None
    if args.resume:
        path = args.resume
        if path == "latest":
            path = Checkpointer(os.path.join(args.out_dir, "ckpt"), rank, per_rank=per_rank).latest()
        if path:
            sd = load_checkpoint(path, net if use_engine else model, optimizer, scheduler, rank=rank)
            flat.refresh_shadow()
            start, hist = sd["global_epoch"], sd["histories"]
            ex = sd.get("extra", {})
            rng_state = ex.get("rng_state")
            if "indices_train" in ex:
                from .data.loader import DeviceLoader
                from .train.trainer import loader_seed

                tr_idx, va_idx = ex["indices_train"].numpy(), ex["indices_val"].numpy()
                train_loader = DeviceLoader(trainset, tr_idx, args.batch_size, dev, dtype=dtype, augment=args.augment,
                                            seed=loader_seed(args.seed, rank, start))
                val_loader = DeviceLoader(valset, va_idx, args.batch_size, dev, dtype=dtype,
                                          augment=args.augment if args.augment_val else False,
                                          seed=(loader_seed(args.seed, rank, start) * 31 + 7) & 0x7FFFFFFF)
            if ex.get("fixed_classes") is not None:
                fc = ex["fixed_classes"]
                fixed_classes = fc.tolist() if torch.is_tensor(fc) else list(fc)

    from .utils import tracing

    timer = None
    if args.trace:
        tracing.enable(True)
        timer = tracing.PhaseTimer(dev, enabled=True)
    timelimit = args.time_limit if args.time_limit and args.time_limit > 0 else math.inf
    histories = train_global(
        net, train_loader, val_loader, trainset, valset, tr_idx, va_idx, criterion, optimizer, scheduler, dev, rank,
        world, args.epochs_local, args.epochs_global, timelimit, args.batch_size, args.prev_fraction,
        args.next_fraction, args.local_weight, args.aggregation_type, args.aggregation_by, comm=comm,
        topology=args.topology, fixed_classes=fixed_classes, fixed_ratio=fixed_ratio, sync_every=args.sync_every,
        dp=dp, partition_rule=args.partition_rule, repartition=not args.no_repartition, replace=replace,
        seed=args.seed, legacy_gossip=args.legacy_gossip, average_buffers=args.average_buffers,
        check_every=args.check_every, progress=not args.quiet, logger=logger, checkpointer=ckpt,
        start_global_epoch=start, histories=hist, dtype=dtype, verbose=not args.quiet, timer=timer,
        graphs=args.graphs, rng_state=rng_state, ref_samples_per_s=args.ref_samples_per_s)
    if timer is not None:
        phases = timer.summary()
        logger.log(kind="phase_times", phases=phases)
        if not args.quiet:
            for k, v in sorted(phases.items(), key=lambda kv: -kv[1]["total_ms"]):
                print(f"[rank {rank}] {k:10s} {v['total_ms']:10.2f} ms total  {v['mean_ms']:8.3f} ms x {v['count']}")

    result = {"histories": [list(h) if not isinstance(h, list) else h for h in histories]}
    if rank == 0 and not args.no_eval:
        loss, acc, _, _ = evaluate(net, test_loader, criterion, dev, rank, num_classes=trainset.num_classes,
                                   verbose=not args.quiet)
        rep = {k: v for k, v in evaluate.last_report.items() if k != "confusion_matrix"}
        result.update(test_loss=loss, test_acc=acc, **rep)
        logger.log(kind="test", test_loss=loss, test_acc=acc, **rep)
    if rank == 0 and args.plots:
        from .utils.viz import plot_all

        plot_all(histories, args.epochs_global, args.epochs_local, 0, args.plots)
    if rank == 0:
        with open(os.path.join(args.out_dir, "histories.json"), "w") as f:
            json.dump(result, f)
    logger.close()
    D.teardown(ctx)
    return result


if __name__ == "__main__":
    main()
