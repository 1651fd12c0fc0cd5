"""Headline benchmark: samples/sec of the whole node for the flagship 3-layer MLP.

BASELINE.json metric: "samples/sec (whole node) + DP scaling eff., 3-layer MLP
at 1/2/4/8 MI355X".  Config (weak scaling, fixed per-GPU work):

  model      mlp3: 784 -> 4096 -> 4096 -> 10, ReLU, 19.99 M params (MNIST-shaped input)
  batch      16384 samples per GPU (global = 16384 x N).  Sized for MI355X: the
             per-step gradient bytes are fixed by the model (20 M params), so a
             bigger per-GPU batch amortises the xGMI reduce-scatter/all-gather
             over more MFMA work, and the 16384-row GEMMs run at a higher
             fraction of peak (measured 1 GPU: 7.04 M samples/s at 4096,
             7.58 M at 8192, 7.98 M at 16384, before the library dgrad)
  compute    bf16 MFMA GEMMs, fp32 accumulation, fp32 master weights + grads
  optimizer  SGD momentum 0.9 (fused kernel, full update every step)
  comm       fp32 gradient reduce-scatter on RCCL every step, bucketed and
             overlapped with the backward pass, sharded SGD, bf16 weight all-gather
  data       synthetic (device-generated Gaussian inputs, uniform labels),
             random-init (Xavier) weights; no dataset download exists here

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
                 --master-port P bench.py --gpus N
Rank 0 prints ONE JSON line; `value` is the whole-job samples/sec (max step time
over ranks).  `--compare-stock` also times a stock PyTorch-ROCm eager
implementation (nn.Linear + DDP + torch.optim.SGD) of the same config.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import ldnn  # noqa: E402
from ldnn.models.mlp import mlp3  # noqa: E402
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine  # noqa: E402
from ldnn.utils import distributed as D  # noqa: E402

METRIC = "samples/sec (whole node) + DP scaling eff., 3-layer MLP at 1/2/4/8 MI355X"


def xavier_init(model):
    for m in model.modules():
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.xavier_uniform_(m.weight)
            torch.nn.init.zeros_(m.bias)


def make_batches(nb, B, in_features, classes, device, seed):
    from ldnn.ops import _ext

    C = _ext.C()
    xs, ys = [], []
    for i in range(nb):
        x = torch.empty(B, in_features, dtype=torch.bfloat16, device=device)
        y = torch.empty(B, dtype=torch.long, device=device)
        C.synth_normal(x, seed * 1000 + i, 1.0)
        C.synth_labels(y, classes, seed * 1000 + i)
        xs.append(x)
        ys.append(y)
    return xs, ys


def timed(ctx, step_fn, steps, warmup):
    for i in range(warmup):
        step_fn(i)
    if ctx.distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step_fn(warmup + i)
    torch.cuda.synchronize()
    if ctx.distributed:
        dist.barrier()
    el = time.perf_counter() - t0
    if ctx.distributed:
        t = torch.tensor([el], device=ctx.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    return el


def run_ldnn(ctx, args):
    torch.manual_seed(1234)
    model = mlp3(args.in_features, args.hidden, args.classes)
    xavier_init(model)
    eng = StaticMLPEngine(model, args.batch, OptimConfig("sgd", lr=args.lr, momentum=0.9),
                          device=ctx.device, world_size=ctx.world_size, use_graphs=not args.no_graphs,
                          bucket_cap_elems=args.bucket_elems, shard_optimizer=False if args.no_shard else None,
                          library_gemms=args.gemms == "library",
                          early_optimizer={"on": True, "off": False, "auto": None}[args.early_opt],
                          fuse_head_dgrad=False if args.no_fuse_head_dgrad else None,
                          concurrent_wgrad=args.concurrent_wgrad, overlap_optimizer=args.overlap_opt,
                          pad_input=args.pad_input, head_dgrad_mode=args.head_dgrad_mode)
    if ctx.distributed:
        dist.broadcast(eng.flat.master, src=0)
        eng.flat.refresh_shadow()
    xs, ys = make_batches(args.nbatches, args.batch, args.in_features, args.classes, ctx.device, 17 + ctx.rank)

    def step(i):
        j = i % len(xs)
        eng.load_batch(xs[j], ys[j])
        eng.step()

    el = timed(ctx, step, args.steps, args.warmup)
    loss, acc = eng.read_stats(args.batch * (args.steps + args.warmup))
    return el, dict(train_loss=round(loss, 4), n_params=sum(p.numel() for p in model.parameters()),
                    in_pad=eng.in_pad, gemm_kernels=eng.describe())


def run_stock(ctx, args):
    """Stock PyTorch-ROCm eager baseline of the same config (hipBLASLt GEMMs,
    MIOpen/ATen elementwise, RCCL DDP, torch.optim.SGD foreach), bf16 autocast."""
    import torch.nn as nn

    torch.manual_seed(1234)
    model = nn.Sequential(nn.Linear(args.in_features, args.hidden), nn.ReLU(), nn.Linear(args.hidden, args.hidden),
                          nn.ReLU(), nn.Linear(args.hidden, args.classes)).to(ctx.device)
    xavier_init(model)
    if ctx.distributed:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[ctx.device.index])
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9)
    crit = nn.CrossEntropyLoss()
    xs, ys = make_batches(args.nbatches, args.batch, args.in_features, args.classes, ctx.device, 17 + ctx.rank)

    def step(i):
        j = i % len(xs)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(xs[j])
            loss = crit(out.float(), ys[j])
        loss.backward()
        opt.step()

    return timed(ctx, step, args.steps, args.warmup)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16384, help="per-GPU batch")
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--in-features", type=int, default=784)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--nbatches", type=int, default=4)
    ap.add_argument("--bucket-elems", type=int, default=8 << 20)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-shard", action="store_true",
                    help="all-reduce + replicated optimizer instead of reduce-scatter / sharded optimizer / all-gather")
    ap.add_argument("--gemms", choices=["ldnn", "library"], default="ldnn",
                    help="ldnn: every GEMM on ldnn's own MFMA kernels (default); library: the plain GEMMs "
                         "(fp32 wgrads, bias+ReLU forwards, hidden dgrad) on hipBLASLt, as an A/B baseline")
    ap.add_argument("--pad-input", action="store_true",
                    help="with --gemms library: pad the 784-wide first layer to K = 832 (measured slightly slower)")
    ap.add_argument("--overlap-opt", action="store_true",
                    help="1 GPU: optimizer update of all weights but W_0 on a side stream beside wgrad(0)")
    ap.add_argument("--concurrent-wgrad", action="store_true",
                    help="1 GPU: wgrad(1) on a side stream beside dgrad(1) + wgrad(0)")
    ap.add_argument("--no-fuse-head-dgrad", action="store_true",
                    help="separate head dgrad GEMM instead of the head kernel's fused dgrad (dReLU + dbias)")
    ap.add_argument("--head-dgrad-mode", type=int, default=-1,
                    help="-1 auto (streaming dh kernel for <= 16 classes), 1 fused (h re-read), 2 fused (h in LDS)")
    ap.add_argument("--early-opt", choices=["auto", "on", "off"], default="auto",
                    help="1 GPU: update W_{L-1}..W_1 on a side stream beside the last dgrad GEMM")
    ap.add_argument("--compare-stock", action="store_true")
    ap.add_argument("--backend", default="auto", help="auto (nccl = RCCL on GPUs) | gloo (testing only)")
    args = ap.parse_args()

    ctx = D.setup(None if args.backend == "auto" else args.backend)
    n = ctx.world_size
    el, extra = run_ldnn(ctx, args)
    comm = "RCCL" if ctx.backend == "nccl" else ctx.backend
    ms = el / args.steps * 1e3
    value = args.batch * n * args.steps / el
    rec = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (device-generated N(0,1) inputs, uniform labels; random-init Xavier weights)",
        "config": {
            "model": f"mlp3 {args.in_features}-{args.hidden}-{args.hidden}-{args.classes} relu",
            "global_batch": args.batch * n,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "parallelism": f"dp{n}",
            "optimizer": "sgd momentum 0.9, fp32 master",
            "gemms": ("ldnn MFMA kernels only: bias+ReLU fwd (ReLU bit masks), dReLU dgrad on a transposed W, "
                      "fp32 wgrads (split-K slabs + slab_sum for the 784-wide one), classifier head (Linear + softmax-xent + argmax + "
                      "head dgrad), SGD" if args.gemms == "ldnn" else
                      "hipBLASLt: fp32 wgrads, bias/ReLU fwd, hidden dgrad; ldnn: fused dReLU+dbias pass, "
                      "classifier head (Linear + softmax-xent + argmax + head dgrad), SGD"),
            "grad_sync": ("none (1 GPU)" if n == 1 else
                          f"fp32 {comm} all-reduce, bucketed, overlapped" if args.no_shard else
                          f"fp32 {comm} reduce-scatter (bucketed, overlapped) + sharded SGD + bf16 weight all-gather"),
        },
    }
    rec.update(extra)
    if args.compare_stock:
        el_s = run_stock(ctx, args)
        stock = args.batch * n * args.steps / el_s
        rec["stock_pytorch_samples_per_s"] = round(stock, 1)
        rec["stock_pytorch_ms_per_step"] = round(el_s / args.steps * 1e3, 4)
        rec["speedup_vs_stock_pytorch"] = round(value / stock, 3)
    if ctx.is_main:
        print(json.dumps(rec), flush=True)
    D.teardown(ctx)


if __name__ == "__main__":
    main()
