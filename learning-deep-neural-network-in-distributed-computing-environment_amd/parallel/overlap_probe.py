"""Overlap probe for the segmented graphed DP step (train/graphed.py GraphedDPStep).

On one GPU there is no second rank to all-reduce with, so the bucket collectives
are replaced by a STAND-IN with the same stream behaviour as RCCL's: issued from
the host between two graphs of the backward chain, on its own HIP stream that
waits for the compute stream, joined (stream wait, no host sync) before the
optimizer graph.  The stand-in has RCCL's footprint: ``reps`` copies of the bucket
on ``blocks`` workgroups (an RCCL ring all-reduce runs one workgroup per channel,
a few dozen at most, paced by the xGMI links -- not a chip-wide HBM copy), sized
so its standalone time is of the order of that bucket's all-reduce on 8 x MI355X.
If the chain overlaps communication with the backward, the step with the stand-in
costs much less than the step without it plus the stand-in's standalone time.

    python scripts/overlap_probe.py --model resnet18 --batch 64   (prints one JSON line)
"""
from __future__ import annotations

import argparse
import json
import time

import torch


class _Join:
    def __init__(self, side):
        self.side = side

    def wait(self):
        torch.cuda.current_stream().wait_stream(self.side)


class StandInComm:
    """``comm_fn`` for GraphedDPStep: ``reps`` copies of bucket i on ``blocks``
    workgroups (native standin_copy kernel), on a side stream."""

    def __init__(self, device, reps: int = 4, blocks: int = 16):
        from ..ops import _ext

        self.C = _ext.C()
        self.side = torch.cuda.Stream(device=device)
        self.reps, self.blocks = int(reps), int(blocks)
        self.scratch: dict = {}

    def __call__(self, i, buf):
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            sc = self.scratch.get(i)
            if sc is None:
                sc = self.scratch[i] = torch.empty_like(buf)
            self.C.standin_copy(buf, sc, self.blocks, self.reps)
        return _Join(self.side)


def _timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def measure_overlap(model_name: str, batch: int, bucket_mb: float = 32.0, reps: int = 4, steps: int = 20,
                    rounds: int = 3, blocks: int = 16) -> dict:
    import ldnn
    from ldnn.data.datasets import SHAPES
    from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init
    from ldnn.optim import SGD
    from ldnn.parallel.comm import LocalComm
    from ldnn.parallel.ddp import DataParallel
    from ldnn.train.graphed import GraphedDPStep

    dev = torch.device("cuda", torch.cuda.current_device())
    shape = SHAPES[dataset_for(model_name)]
    nc = 1000 if model_name == "resnet18" else 10
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(batch, *shape, device=dev, generator=g).bfloat16()
    y = torch.randint(0, nc, (batch,), device=dev, generator=g)
    crit = CrossEntropyLoss()
    standin = StandInComm(dev, reps, blocks)
    steps_fn = {}
    for name, fn in (("single", lambda i, buf: None), ("with_standin", standin)):
        torch.manual_seed(0)
        m = build_model(model_name)
        xavier_init(m)
        ldnn.prepare(m, dev)
        opt = SGD(m.parameters(), lr=0.01, momentum=0.9)
        opt.zero_grad()
        crit(m(x), y).backward()
        opt.step()
        dp = DataParallel(m, LocalComm(), bucket_cap_mb=bucket_mb, broadcast_init=False)
        gd = GraphedDPStep(dp, crit, opt, x, y, mode="segmented", comm_fn=fn)
        steps_fn[name] = (gd, dp)
    gd, dp = steps_fn["with_standin"]
    bufs = [dp.bucketer.comm_buffer(i) for i in range(len(dp.bucketer.buckets))]

    def standin_alone():
        for i, b in enumerate(bufs):
            standin(i, b).wait()

    fns = {"single_ms": lambda: steps_fn["single"][0](x, y),
           "with_standin_ms": lambda: steps_fn["with_standin"][0](x, y),
           "standin_alone_ms": standin_alone}
    for f in fns.values():
        for _ in range(3):
            f()
    best = {k: 1e9 for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            best[k] = min(best[k], _timed(f, steps))
    hidden = best["single_ms"] + best["standin_alone_ms"] - best["with_standin_ms"]
    return {"model": model_name, "batch": batch, "bucket_mb": bucket_mb, "buckets": len(bufs),
            "bucket_mb_each": [round(b.numel() * b.element_size() / 2**20, 2) for b in bufs],
            "segments": gd.n_segments, "standin_reps": reps, "standin_blocks": blocks, **{k: round(v, 4) for k, v in best.items()},
            "hidden_ms": round(hidden, 4),
            "hidden_fraction": round(hidden / max(best["standin_alone_ms"], 1e-9), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=16)
    a = ap.parse_args()
    print(json.dumps(measure_overlap(a.model, a.batch, a.bucket_mb, a.reps, a.steps, blocks=a.blocks)), flush=True)


if __name__ == "__main__":
    main()
