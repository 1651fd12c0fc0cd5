"""Graph-captured per-step DP on one GPU: the single-process graphed step
(GraphedStep) vs the graphed DP step with its bucket all-reduces captured into
the graph on a real RCCL communicator of world 1 (GraphedDPStep in_graph) and
the eager bucketed DP step, interleaved rounds in one process.

    python scripts/bench_cnn_dp.py --model resnet18 --batch 64
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402
from ldnn.data.datasets import SHAPES  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init  # noqa: E402
from ldnn.optim import SGD  # noqa: E402
from ldnn.parallel.comm import TorchComm  # noqa: E402
from ldnn.parallel.ddp import DataParallel  # noqa: E402
from ldnn.train.graphed import GraphedDPStep, GraphedStep  # noqa: E402


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args()
    store = dist.FileStore(os.path.join(tempfile.mkdtemp(), "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda:0"))
    shape = SHAPES[dataset_for(a.model)]
    nc = 1000 if a.model == "resnet18" else 10
    x = torch.randn(a.batch, *shape, device="cuda").bfloat16()
    y = torch.randint(0, nc, (a.batch,), device="cuda")
    crit = CrossEntropyLoss()
    ms = []
    for _ in range(3):
        torch.manual_seed(0)
        m = build_model(a.model)
        xavier_init(m)
        ldnn.prepare(m, "cuda")
        ms.append(m)
    opts = [SGD(m.parameters(), lr=0.01, momentum=0.9) for m in ms]
    for m, o in zip(ms, opts):  # eager first step: optimizer state exists before capture
        o.zero_grad()
        crit(m(x), y).backward()
        o.step()
    gs = GraphedStep(ms[0], crit, opts[0], x, y, warmup=0)
    dp = DataParallel(ms[1], TorchComm(), bucket_cap_mb=a.bucket_mb, broadcast_init=False,
                      comm_dtype=torch.bfloat16 if a.comm_dtype == "bf16" else None)
    gd = GraphedDPStep(dp, crit, opts[1], x, y)
    dpe = DataParallel(ms[2], TorchComm(), bucket_cap_mb=a.bucket_mb, broadcast_init=False,
                       comm_dtype=torch.bfloat16 if a.comm_dtype == "bf16" else None)

    def eager_dp():
        opts[2].zero_grad()
        crit(dpe(x), y).backward()
        dpe.finish_gradient_sync()
        opts[2].step()

    fns = {"graphed_single_ms": lambda: gs(x, y), "graphed_dp_rccl_in_graph_ms": lambda: gd(x, y),
           "eager_dp_rccl_ms": eager_dp}
    for fn in fns.values():
        for _ in range(3):
            fn()
    best = {k: 1e9 for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            best[k] = min(best[k], timed(fn, a.steps))
    rec = {"model": a.model, "batch": a.batch, "buckets": len(dp.bucketer.buckets), "comm_dtype": a.comm_dtype,
           "mode": gd.mode, **{k: round(v, 3) for k, v in best.items()}}
    rec["dp_over_single"] = round(best["graphed_dp_rccl_in_graph_ms"] / best["graphed_single_ms"], 3)
    print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
