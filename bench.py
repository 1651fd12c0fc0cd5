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
  comm       bf16 gradient reduce-scatter on RCCL every step (--grad-comm fp32: fp32),
             bucketed and overlapped with the backward pass, widened into the fp32
             shard of a sharded SGD (fp32 master), bf16 weight all-gather
  data       synthetic (device-generated Gaussian inputs, uniform labels),
             random-init (Xavier) weights; no dataset download exists here

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python bench.py --gpus N            (spawns `torch.distributed.run` itself, as a
                                                  child process, before any GPU call)
         or  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
                 --master-port P bench.py --gpus N
Under a launcher the world size must equal --gpus (checked); with RCCL every rank
must own a distinct GPU (checked: RCCL refuses two ranks on one device).

Rank 0 prints ONE JSON line; `value` is the whole-job samples/sec (max step time
over ranks).  Besides the headline it reports, per rank and maxed over ranks:
  per_gpu_local_ms     the same engine's comm-free step (world 1, no collectives)
  scaling_efficiency   per_gpu_local_ms / ms_per_step  (1.0 at N = 1)
  comm_us              standalone per-bucket reduce-scatter / all-gather times (N > 1)
  configs              BASELINE configs #4/#5 and the reference's own workload at this N:
                       LeNet-5 28x28 b256, ResNet-18 224x224 b64 / b256 (SGD momentum) and
                       EnhancedCNNModel 32x32 b64 with Adam lr 1e-3 per GPU, each a
                       graph-replayed step (N > 1: GraphedDPStep over the sharded DP --
                       bucket reduce-scatters issued between the links of the backward
                       graph chain, sharded optimizer, bf16 weight all-gathers) with its own
                       comm-free local time and scaling efficiency (--no-configs skips)
`--compare-stock` also times a stock PyTorch-ROCm eager implementation
(nn.Linear + DDP + torch.optim.SGD) of the headline config.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
GRAD_COMM = {"dtype": "bf16"}   # gradient collective dtype at N > 1 (--grad-comm)


def _grad_dtype():
    return torch.bfloat16 if GRAD_COMM["dtype"] == "bf16" else None


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


def fill_slots(eng, args, seed):
    """args.nbatches synthetic batches (device-generated N(0,1) inputs, uniform labels),
    each written into one input slot of the engine."""
    xs, ys = make_batches(args.nbatches, args.batch, args.in_features, args.classes, eng.device, seed)
    slots = eng.add_input_slots(len(xs))
    for (sx, sy), x, y in zip(slots, xs, ys):
        sx.copy_(x)
        sy.copy_(y)
    del xs, ys
    # prime every slot's segments (eager warm-up calls + the graph capture) before any
    # timing: untimed steps, so no capture can fall inside the timed region
    for _ in range(3):
        for i in range(len(slots)):
            eng.step(slot=1 + i)
    eng.reset_stats()   # the statistics then cover exactly the warmup + timed steps
    return slots


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


def timed_windows(ctx, step_fn, steps, warmup, windows=3):
    """The secondary configs' timing: `windows` back-to-back timed windows of `steps` steps each
    (each bracketed like `timed`, max over ranks), the median window reported -- one host or
    device hiccup inside a ~0.1 s window otherwise moves a config's number by tens of percent
    (seen once: EnhancedCNN Adam 2.20 ms in one run, 1.63-1.65 ms in every other).  Returns
    (median seconds, every window's ms per step)."""
    els, done = [], 0
    for w in range(windows):
        el = timed(ctx, lambda i: step_fn(done + i), steps, warmup if w == 0 else 0)
        done += steps + (warmup if w == 0 else 0)
        els.append(el)
    return sorted(els)[len(els) // 2], [round(e / steps * 1e3, 4) for e in els]


def run_ldnn(ctx, args):
    torch.manual_seed(1234)
    model = mlp3(args.in_features, args.hidden, args.classes)
    xavier_init(model)
    eng = StaticMLPEngine(model, args.batch, OptimConfig("sgd", lr=args.lr, momentum=0.9),
                          device=ctx.device, world_size=ctx.world_size, use_graphs=not args.no_graphs,
                          bucket_cap_elems=args.bucket_elems, shard_optimizer=False if args.no_shard else None,
                          library_gemms=args.gemms == "library",
                          fuse_head_dgrad=False if args.no_fuse_head_dgrad else None,
                          head_dgrad_mode=args.head_dgrad_mode, fuse_head_fwd=not args.no_fuse_head_fwd,
                          fuse_head_bwd=not args.no_fuse_head_bwd,
                          comm_dtype=_grad_dtype() if not args.no_shard else None)
    if ctx.distributed:
        dist.broadcast(eng.flat.master, src=0)
        eng.flat.refresh_shadow()
    # synthetic batches generated once, each straight into its own input slot of the
    # engine (a prefetching loader's layout): the step reads it in place, no copy
    slots = fill_slots(eng, args, 17 + ctx.rank)

    def step(i):
        eng.step(slot=1 + i % len(slots))

    el = timed(ctx, step, args.steps, args.warmup)
    loss, acc = eng.read_stats(args.batch * (args.steps + args.warmup))
    extra = dict(train_loss=round(loss, 4), n_params=sum(p.numel() for p in model.parameters()),
                 buckets=len(eng.buckets), gemm_kernels=eng.describe())
    if ctx.world_size > 1:
        extra["comm_us"] = comm_micro(ctx, eng)
        # the same engine without any collective: this rank's comm-free step time
        torch.manual_seed(1234)
        m1 = mlp3(args.in_features, args.hidden, args.classes)
        xavier_init(m1)
        loc = StaticMLPEngine(m1, args.batch, OptimConfig("sgd", lr=args.lr, momentum=0.9), device=ctx.device,
                              world_size=1, use_graphs=not args.no_graphs)

        lslots = fill_slots(loc, args, 17 + ctx.rank)

        def lstep(i):
            loc.step(slot=1 + i % len(lslots))

        extra["local_s"] = timed(ctx, lstep, args.steps, args.warmup)
        del loc
    return el, extra


def comm_micro(ctx, eng, iters: int = 10) -> dict:
    """Standalone RCCL time of each bucket's gradient reduce-scatter (in the engine's comm
    dtype) and bf16 all-gather (the sharded engine's two collectives), max over ranks, in
    microseconds."""
    out = {}
    gdt = torch.bfloat16 if getattr(eng, "comm_bf16", False) else torch.float32
    for i, (b, e, _) in enumerate(eng.buckets):
        g = torch.empty(e - b, dtype=gdt, device=ctx.device)
        gs = torch.empty((e - b) // ctx.world_size, dtype=gdt, device=ctx.device)
        w = torch.empty(e - b, dtype=torch.bfloat16, device=ctx.device)
        ws = torch.empty((e - b) // ctx.world_size, dtype=torch.bfloat16, device=ctx.device)
        res = []
        if ctx.backend != "nccl":   # gloo rehearsal: no device reduce-scatter / in-place gather
            fns = (lambda: dist.all_reduce(g), lambda: dist.all_reduce(w.float()))
        else:
            fns = (lambda: dist.reduce_scatter_tensor(gs, g), lambda: dist.all_gather_into_tensor(w, ws))
        for fn in fns:
            fn()
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize()
            t = torch.tensor([(time.perf_counter() - t0) / iters * 1e6], device=ctx.device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res.append(round(t.item(), 1))
        out[f"bucket{i}"] = {"mb_fp32": round((e - b) * 4 / 2**20, 2),
                             f"reduce_scatter_{'bf16' if gdt == torch.bfloat16 else 'fp32'}_us": res[0],
                             "all_gather_bf16_us": res[1]}
    return out


# (model, per-GPU batch, timed steps, optimizer): BASELINE configs #4 / #5 and the
# reference's own workload (EnhancedCNNModel, batch 64, Adam lr 1e-3: BAR/main.py:52-54)
CNN_CONFIGS = (("lenet5", 256, 50, "sgd"), ("resnet18", 64, 20, "sgd"), ("resnet18", 256, 8, "sgd"),
               ("enhanced_cnn", 64, 30, "adam"))


def run_cnn(ctx, name: str, batch: int, steps: int, optimizer: str = "sgd", warmup: int = 3) -> dict:
    """One CNN config at this world size: bf16 native kernels, synthetic data,
    random-init weights; SGD momentum 0.9 (lr 0.01) or Adam (lr 1e-3).  N = 1: the
    single-process graphed step.  N > 1: GraphedDPStep over DataParallel(shard_optimizer=
    True) -- each gradient bucket's fp32 RCCL reduce-scatter issued between the links of
    the backward graph chain, the fused optimizer on this rank's 1/N shard, the bf16
    weights all-gathered in place -- with the one-shot IPC path for buckets <= 4 MiB."""
    import ldnn
    from ldnn.data.datasets import SHAPES
    from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init as xinit
    from ldnn.optim import SGD, Adam
    from ldnn.parallel.comm import ONESHOT_DEFAULT_BYTES, default_comm
    from ldnn.parallel.ddp import DataParallel
    from ldnn.train.graphed import GraphedDPStep, GraphedStep

    shape = SHAPES[dataset_for(name)]
    nc = 1000 if name == "resnet18" else 10
    g = torch.Generator(device=ctx.device).manual_seed(100 + ctx.rank)
    xs = [torch.randn(batch, *shape, device=ctx.device, generator=g).bfloat16() for _ in range(2)]
    ys = [torch.randint(0, nc, (batch,), device=ctx.device, generator=g) for _ in range(2)]
    crit = CrossEntropyLoss()
    comm = default_comm(ONESHOT_DEFAULT_BYTES) if ctx.world_size > 1 else None

    def make(dp_on: bool):
        torch.manual_seed(0)
        m = build_model(name)
        xinit(m)
        ldnn.prepare(m, ctx.device)
        dp = (DataParallel(m, comm, bucket_cap_mb=32.0, shard_optimizer=True, comm_dtype=_grad_dtype())
              if dp_on else None)
        # (the optimizer after the wrapper: sharding re-lays the flat buffers out)
        opt = SGD(m.parameters(), lr=0.01, momentum=0.9) if optimizer == "sgd" else Adam(m.parameters(), lr=1e-3)
        net = dp if dp is not None else m
        opt.zero_grad()
        crit(net(xs[0]), ys[0]).backward()
        if dp is not None:
            dp.finish_gradient_sync()
        opt.step()
        if dp is not None:
            dp.wait_gathers()
            return GraphedDPStep(dp, crit, opt, xs[0], ys[0]), m
        return GraphedStep(m, crit, opt, xs[0], ys[0], warmup=0), m

    gs, m = make(ctx.world_size > 1)
    el, wins = timed_windows(ctx, lambda i: gs(xs[i % 2], ys[i % 2]), steps, warmup)
    ms = el / steps * 1e3
    rec = {"model": name, "per_gpu_batch": batch, "global_batch": batch * ctx.world_size, "steps": steps,
           "timing": "median of 3 timed windows of `steps` steps", "window_ms": wins,
           "optimizer": "sgd momentum 0.9 lr 0.01" if optimizer == "sgd" else "adam lr 1e-3",
           "ms_per_step": round(ms, 4), "samples_per_s": round(batch * ctx.world_size / el * steps, 1),
           "n_params": sum(p.numel() for p in m.parameters())}
    if ctx.world_size > 1:
        bk = gs.bk
        rec["grad_sync"] = (f"{GRAD_COMM['dtype']} reduce-scatter per bucket (between backward graph links) + "
                            f"sharded {optimizer} + bf16 weight all-gather; 1-D params all-reduced")
        rec["comm_dtype"] = f"{GRAD_COMM['dtype']} gradients / bf16 weights"
        rec["oneshot_ipc"] = bool(getattr(comm, "oneshot", None) is not None)
        rec["buckets"] = len(bk.buckets)
        rec["sharded_buckets"] = sum(1 for b in bk.buckets if b["sharded"])
        rec["graph_segments"] = gs.n_segments
        del gs
        gl, _ = make(False)
        ell, _ = timed_windows(ctx, lambda i: gl(xs[i % 2], ys[i % 2]), steps, warmup)
        rec["per_gpu_local_ms"] = round(ell / steps * 1e3, 4)
        rec["scaling_efficiency"] = round(ell / el, 4)
        del gl
    else:
        rec["per_gpu_local_ms"] = rec["ms_per_step"]
        rec["scaling_efficiency"] = 1.0
    torch.cuda.empty_cache()
    return rec


def run_configs(ctx, configs, run_fn) -> dict:
    """The secondary CNN configs, each guarded: a failing config records its error instead of
    costing the headline record.  After each config every rank learns whether any rank failed
    (0 ok, 1 failed, 2 device fault) with one small all_reduce(MAX), so a rank that failed alone
    never leaves its peers inside collectives it does not join; a device fault (or, with peers,
    any failure) ends the loop.
    The flag travels on a side gloo group, so it can never pair up with a collective of the
    config itself: peers still waiting inside the failed config's collectives leave them at the
    process group's timeout (an error of their own) and then meet the failed rank there."""
    out = {}
    side = dist.new_group(backend="gloo") if ctx.world_size > 1 else None
    for name, b, st, o in configs:
        key = f"{name}_b{b}" + ("_adam" if o == "adam" else "")
        err = None
        try:
            out[key] = run_fn(ctx, name, b, st, o)
        except Exception as e:  # noqa: BLE001 -- a secondary config must not cost the headline record
            err = e
            out[key] = {"error": f"{type(e).__name__}: {e}"[:500]}
        fault = err is not None and any(t in str(err) for t in ("HIP error", "hipError", "illegal", "fault"))
        code = 2 if fault else (1 if err is not None else 0)
        if ctx.world_size > 1:
            try:
                flag = torch.tensor([code], dtype=torch.int32)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=side)
                code = int(flag.item())
            except Exception:  # noqa: BLE001
                code = 2
        if code and err is None:
            out[key] = {"error": "failed on another rank"}
        # a device fault, or any failure with peers (their process group may be left broken or
        # mid-collective): no further configs
        if code == 2 or (code and ctx.world_size > 1):
            for n2, b2, _, o2 in configs[len(out):]:
                out[f"{n2}_b{b2}" + ("_adam" if o2 == "adam" else "")] = {"skipped": "an earlier config failed"}
            break
        if torch.cuda.is_available():
            torch.cuda.empty_cache()
    return out


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


def _free_port() -> int:
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: run `torch.distributed.run` as a CHILD process
    (never exec: nothing here has touched the GPU yet) and return its exit code.
    Rank 0's JSON line reaches our stdout through the inherited file descriptor."""
    if args.backend in ("auto", "nccl"):
        ndev = torch.cuda.device_count()   # does not initialise the GPU runtime
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} with RCCL needs {args.gpus} GPUs, this node has {ndev} "
                  f"(RCCL refuses two ranks on one GPU; use --backend gloo to rehearse)", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


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
    ap.add_argument("--no-fuse-head-fwd", action="store_true",
                    help="A/B: separate head kernel instead of the logits in the last hidden forward's epilogue")
    ap.add_argument("--no-fuse-head-bwd", action="store_true",
                    help="A/B: head dgrad stream + separate head wgrad instead of the fused MFMA head backward")
    ap.add_argument("--no-fuse-head-dgrad", action="store_true",
                    help="separate head dgrad GEMM instead of the head kernel's fused dgrad (dReLU + dbias)")
    ap.add_argument("--head-dgrad-mode", type=int, default=-1,
                    help="-1 auto (streaming dh kernel for <= 16 classes), 1 fused (h re-read), 2 fused (h in LDS)")
    ap.add_argument("--compare-stock", action="store_true")
    ap.add_argument("--backend", default="auto", help="auto (nccl = RCCL on GPUs) | gloo (testing only)")
    ap.add_argument("--grad-comm", choices=["bf16", "fp32"], default="bf16",
                    help="gradient reduce-scatter dtype at N > 1 (bf16: half the xGMI bytes, widened into the "
                         "fp32 shard of the sharded optimizer)")
    ap.add_argument("--no-configs", action="store_true", help="skip the LeNet-5 / ResNet-18 config timings")
    args = ap.parse_args()
    GRAD_COMM["dtype"] = args.grad_comm

    if args.gpus > 1 and D.launch_env()[1] == 1:
        sys.exit(self_launch(args))
    if D.launch_env()[1] != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {D.launch_env()[1]} ranks", file=sys.stderr)
        sys.exit(2)
    if args.backend in ("auto", "nccl") and args.gpus > torch.cuda.device_count():
        print(f"bench.py: --gpus {args.gpus} with RCCL needs one GPU per rank, this node has "
              f"{torch.cuda.device_count()}", file=sys.stderr)
        sys.exit(2)
    ctx = D.setup(None if args.backend == "auto" else args.backend)
    n = ctx.world_size
    assert n == args.gpus, (n, args.gpus)
    comm_info = {"backend": "RCCL" if ctx.backend == "nccl" else ctx.backend, "ranks": n}
    if n > 1:
        devs = [torch.zeros(1, dtype=torch.int64, device=ctx.device) for _ in range(n)]
        dist.all_gather(devs, torch.tensor([ctx.device.index or 0], device=ctx.device))
        comm_info["devices"] = [int(d.item()) for d in devs]
        if ctx.backend == "nccl" and len(set(comm_info["devices"])) != n:
            raise SystemExit(f"bench.py: RCCL ranks share a GPU: {comm_info['devices']}")
    el, extra = run_ldnn(ctx, args)
    local_s = extra.pop("local_s", el)
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
                      "fp32 wgrads (the 784-wide one split-K into slabs + one summing pass that also emits the bias "
                      "gradient from a ones column), classifier head (logits in the last hidden forward's epilogue, "
                      "softmax-xent + argmax, fused MFMA head backward), fused SGD"
                      if args.gemms == "ldnn" else
                      "hipBLASLt: fp32 wgrads, bias/ReLU fwd, hidden dgrad; ldnn: fused dReLU+dbias pass, "
                      "classifier head (Linear + softmax-xent + argmax + head dgrad), SGD"),
            "comm": comm_info,
            "grad_sync": ("none (1 GPU)" if n == 1 else
                          f"fp32 {comm} all-reduce, bucketed, overlapped" if args.no_shard else
                          f"{args.grad_comm} {comm} reduce-scatter (bucketed, overlapped) + sharded SGD (fp32 master) "
                          "+ bf16 weight all-gather"),
            "grad_comm_dtype": None if n == 1 else ("fp32" if args.no_shard else args.grad_comm),
        },
    }
    rec["per_gpu_local_ms"] = round(local_s / args.steps * 1e3, 4)
    rec["scaling_efficiency"] = round(local_s / el, 4)
    rec["rccl_ranks"] = n if ctx.backend == "nccl" else 0
    from ldnn.ops import _ext
    rec["native_build"] = _ext.build_info()   # which _C.so ran, and whether it matches this tree's sources
    rec.update(extra)
    if not args.no_configs:
        rec["configs"] = run_configs(ctx, CNN_CONFIGS, run_cnn)
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
