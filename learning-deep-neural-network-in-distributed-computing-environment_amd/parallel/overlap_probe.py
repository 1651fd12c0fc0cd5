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
    """The stand-in's work handle: like an RCCL work, ``wait()`` orders the current stream
    after THIS collective (an event recorded when it was issued) -- not after everything
    queued on the side stream since (a weight all-gather waited by the forward must not
    also wait for the all-gathers issued after it)."""

    def __init__(self, side):
        self.ev = torch.cuda.Event()
        self.ev.record(side)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class StandInComm:
    """``comm_fn`` for GraphedDPStep: ``reps`` copies of bucket i on ``blocks``
    workgroups (native standin_copy kernel), on a side stream.  ``blocks`` = 0:
    calibrate -- the fewest workgroups whose single copy moves bytes at least at
    ``gbps`` (the xGMI bus bandwidth the stand-in impersonates, see calibrate())."""

    def __init__(self, device, reps: int = 4, blocks: int = 16, gbps: float = 300.0):
        from ..ops import _ext

        import os

        self.C = _ext.C()
        # (a high-priority stream, as RCCL's with utils.distributed.setup: LDNN_RCCL_HIGH_PRIO)
        self.priority = -1 if os.environ.get("LDNN_RCCL_HIGH_PRIO", "1") != "0" else 0
        self.side = torch.cuda.Stream(device=device, priority=self.priority)
        self.reps, self.blocks = int(reps), int(blocks)
        self.scratch: dict = {}
        self.calibration = None
        if self.blocks <= 0:
            self.calibrate(device, gbps)

    def calibrate(self, device, gbps: float, mb: int = 32):
        """Pick ``blocks`` (reps = 1) so the stand-in moves a buffer at >= ``gbps`` GB/s: an
        8-GPU RCCL reduce-scatter / all-gather of S bytes moves (N-1)/N S per rank, at
        roughly 300 GB/s bus bandwidth over MI355X xGMI (7 links x ~150 GB/s, ring
        channels); the stand-in is handed exactly those moved bytes."""
        src = torch.empty(mb << 18, dtype=torch.float32, device=device)
        dst = torch.empty_like(src)
        rates = {}
        for b in (4, 8, 12, 16, 24, 32, 48, 64, 96, 128):
            self.C.standin_copy(src, dst, b, 1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                self.C.standin_copy(src, dst, b, 1)
            torch.cuda.synchronize()
            rates[b] = src.numel() * 4 * 5 / (time.perf_counter() - t0) / 1e9
            if rates[b] >= gbps:
                break
        self.blocks = next((b for b, r in rates.items() if r >= gbps), max(rates))
        self.reps = 1
        self.calibration = {"target_gbps": gbps, "blocks": self.blocks,
                            "gbps": round(rates[self.blocks], 1), "stream_priority": self.priority}

    def __call__(self, i, buf):
        self.side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            sc = self.scratch.get(i)
            if sc is None:
                sc = self.scratch[i] = torch.empty_like(buf)
            self.C.standin_copy(buf, sc, self.blocks, self.reps)
        return _Join(self.side)


class ShardProbeComm:
    """A world-of-``world`` stand-in communicator on ONE GPU for the sharded step
    (DataParallel(shard_optimizer=True)): the bucket layout, shard ranges and every
    collective call site are the real ones, but each reduce-scatter / all-gather is
    the stand-in copy (RCCL's stream behaviour and footprint) of the bytes that
    collective moves over xGMI, (N-1)/N of its full buffer.  Numerics are not
    meaningful (nothing is summed); the timing is."""

    device_collectives = True

    def __init__(self, device, world: int = 8, reps: int = 4, blocks: int = 16, gbps: float = 300.0):
        from .comm import Comm

        self._rec = Comm()
        self.rank, self.world_size = 0, int(world)
        self.standin = StandInComm(device, reps, blocks, gbps)
        self._k = 0
        self.enabled = True   # False: every collective is a no-op (the chain's own cost)

    def record(self, *a, **k):
        return self._rec.record(*a, **k)

    def schedule_digest(self):
        return self._rec.schedule_digest()

    def _moved(self, t):
        n = t.numel() * (self.world_size - 1) // self.world_size // 8 * 8
        v = t.view(-1)[:max(n, 8)]
        return v if v.dtype == torch.float32 else v.view(torch.float32)   # (bf16 weights: same bytes)

    def reduce_scatter(self, out, inp, async_op=False):
        self._k += 1
        return self.standin(("rs", inp.data_ptr()), self._moved(inp)) if self.enabled else None

    def all_gather_into(self, out, inp, async_op=False):
        return self.standin(("ag", out.data_ptr()), self._moved(out)) if self.enabled else None

    def all_reduce(self, t, op="sum", async_op=False):
        if not self.enabled:
            return None
        return self.standin(("ar", t.data_ptr()), t if t.dtype == torch.float32 else t.view(torch.float32))

    def broadcast(self, t, src=0):
        return None

    def barrier(self):
        return None


class _JoinAll:
    def __init__(self, joins):
        self.joins = [j for j in joins if j is not None]

    def wait(self):
        for j in self.joins:
            j.wait()


def _as_f32(t):
    """The bytes of a received buffer as fp32 words (a bf16 exchange moves half the bytes)."""
    v = t.view(-1)
    if v.dtype == torch.float32:
        return v
    return v[:v.numel() // 2 * 2].view(torch.float32)


class P2PProbeComm:
    """A world-of-``world`` stand-in for per-step data parallelism on ONE GPU without sharding:
    ``gossip`` 1 / 2 (DataParallel(gossip=...), BR/communication.py:5-62, BDR/communication.py:5-77)
    or 0 (the equal all-reduce).  Every collective is replaced by stand-in copies with RCCL's
    stream behaviour: a gossip exchange of a bucket is, per neighbour, a copy of the bucket at
    ~one xGMI link's bandwidth (``link_gbps``) on that neighbour's own stream -- the ring and the
    double ring use one resp. two links side by side -- and an 8-rank ring all-reduce moves
    2 (N-1)/N of the bucket at ~``bus_gbps``.  The post-collective work (the fused neighbour mix of
    gossip) runs for real on the received buffers."""

    device_collectives = True

    def __init__(self, device, world: int = 8, link_gbps: float = 150.0, bus_gbps: float = 300.0):
        from .comm import Comm

        self._rec = Comm()
        self.rank, self.world_size = 0, int(world)
        self.links = [StandInComm(device, 1, 0, link_gbps), StandInComm(device, 1, 0, link_gbps)]
        self.bus = StandInComm(device, 1, 0, bus_gbps)
        self.bus.reps = 2
        self.enabled = True

    def record(self, *a, **k):
        return self._rec.record(*a, **k)

    def schedule_digest(self):
        return self._rec.schedule_digest()

    def sendrecv(self, sends, recvs, async_op=False):
        if not self.enabled:
            return None
        return _JoinAll([self.links[k](("p2p", k, rt.data_ptr()), _as_f32(rt)) for k, (rt, _) in enumerate(recvs)])

    def all_reduce(self, t, op="sum", async_op=False):
        if not self.enabled:
            return None
        n = t.numel() * (self.world_size - 1) // self.world_size // 8 * 8
        v = t.view(-1)[:max(n, 8)]
        return self.bus(("ar", t.data_ptr()), v if v.dtype == torch.float32 else v.view(torch.float32))

    def broadcast(self, t, src=0):
        return None

    def barrier(self):
        return None


def measure_gossip(model_name: str = "enhanced_cnn", batch: int = 64, world: int = 8, bucket_mb: float = 32.0,
                   optimizer: str = "adam", steps: int = 20, rounds: int = 3, link_gbps: float = 150.0,
                   bus_gbps: float = 300.0, comm_dtype: str = "fp32") -> list:
    """The graphed per-step DP step (GraphedDPStep, segmented: each bucket's exchange issued between
    the backward's graph links) with the all-reduce (gossip 0), the ring (1) and the double ring (2)
    on a P2PProbeComm world: one row per topology -- the chain with every collective a no-op, the
    step with the stand-ins, the stand-ins alone back to back, and the exposed part."""
    import ldnn
    from ldnn.data.datasets import SHAPES
    from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init
    from ldnn.optim import SGD, Adam
    from ldnn.parallel.ddp import DataParallel
    from ldnn.train.graphed import GraphedDPStep

    dev = torch.device("cuda", torch.cuda.current_device())
    shape = SHAPES[dataset_for(model_name)]
    nc = 1000 if model_name == "resnet18" else 10
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(batch, *shape, device=dev, generator=g).bfloat16()
    y = torch.randint(0, nc, (batch,), device=dev, generator=g)
    crit = CrossEntropyLoss()
    rows = []
    for gossip in (0, 1, 2):
        torch.manual_seed(0)
        m = build_model(model_name)
        xavier_init(m)
        ldnn.prepare(m, dev)
        comm = P2PProbeComm(dev, world, link_gbps, bus_gbps)
        dp = DataParallel(m, comm, bucket_cap_mb=bucket_mb, broadcast_init=False, gossip=gossip,
                          comm_dtype=torch.bfloat16 if comm_dtype == "bf16" else None)
        o = SGD(m.parameters(), lr=0.01, momentum=0.9) if optimizer == "sgd" else Adam(m.parameters(), lr=1e-3)
        o.zero_grad()
        crit(dp(x), y).backward()
        dp.finish_gradient_sync()
        o.step()
        gd = GraphedDPStep(dp, crit, o, x, y)
        bk = dp.bucketer

        def chain_only():
            comm.enabled = False
            try:
                gd(x, y)
            finally:
                comm.enabled = True

        def standin_alone():
            js = [bk.collective(i) for i in range(len(bk.buckets))]
            for j in js:
                if j is not None:
                    j.wait()

        fns = {"chain_ms": chain_only, "with_standin_ms": lambda: gd(x, y), "standin_alone_ms": standin_alone}
        for f in fns.values():
            for _ in range(3):
                f()
        best = {k: 1e9 for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                best[k] = min(best[k], _timed(f, steps))
        exposed = best["with_standin_ms"] - best["chain_ms"]
        rows.append({"model": model_name, "batch": batch, "optimizer": optimizer,
                     "topology": {0: "allreduce", 1: "ring", 2: "double_ring"}[gossip], "grad_comm_dtype": comm_dtype,
                     "mode": f"graphed per-step DP, world {world} stand-in (links {link_gbps:.0f} GB/s, "
                             f"all-reduce bus {bus_gbps:.0f} GB/s)", "buckets": len(bk.buckets),
                     "segments": gd.n_segments, **{k: round(v, 4) for k, v in best.items()},
                     "exposed_ms": round(exposed, 4),
                     "hidden_fraction": round(1.0 - exposed / max(best["standin_alone_ms"], 1e-9), 3),
                     "link_calibration": comm.links[0].calibration, "bus_calibration": comm.bus.calibration})
        del gd, dp, o, m
        torch.cuda.empty_cache()
    base = rows[0]["with_standin_ms"]
    for r in rows:
        r["vs_allreduce_step"] = round(r["with_standin_ms"] / base, 4)
    return rows


def _timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def measure_overlap(model_name: str, batch: int, bucket_mb: float = 32.0, reps: int = 4, steps: int = 20,
                    rounds: int = 3, blocks: int = 16, shard_world: int = 0, optimizer: str = "sgd",
                    tail_steps: int = 0, gbps: float = 300.0, comm_dtype: str = "fp32") -> dict:
    """shard_world > 0: the sharded step (reduce-scatter between backward links, sharded
    optimizer, bf16 weight all-gathers waited by the forward links) on a
    ShardProbeComm of that world size; the stand-ins then cover the reduce-scatter
    AND the all-gather bytes of each bucket."""
    if shard_world:
        return _measure_sharded(model_name, batch, bucket_mb, reps, steps, rounds, blocks, shard_world, optimizer,
                                tail_steps, gbps, comm_dtype)
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
    standin = StandInComm(dev, reps, blocks, gbps)
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
    _tail(fns["with_standin_ms"], tail_steps)
    return {"model": model_name, "batch": batch, "bucket_mb": bucket_mb, "buckets": len(bufs),
            "bucket_mb_each": [round(b.numel() * b.element_size() / 2**20, 2) for b in bufs],
            "segments": gd.n_segments, "standin_reps": standin.reps, "standin_blocks": standin.blocks,
            "standin_calibration": standin.calibration, **{k: round(v, 4) for k, v in best.items()},
            "hidden_ms": round(hidden, 4),
            "hidden_fraction": round(hidden / max(best["standin_alone_ms"], 1e-9), 3)}


def _tail(fn, n):
    """n more steps of the overlapped step after a 20 ms idle gap: the last stretch of a
    kernel trace is then that phase alone (scripts/probe_timeline.py)."""
    if n <= 0:
        return
    torch.cuda.synchronize()
    time.sleep(0.02)
    for _ in range(n):
        fn()
    torch.cuda.synchronize()


def _measure_sharded(model_name, batch, bucket_mb, reps, steps, rounds, blocks, world, optimizer, tail_steps=0,
                     gbps=300.0, comm_dtype="fp32"):
    import ldnn
    from ldnn.data.datasets import SHAPES
    from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init
    from ldnn.optim import SGD, Adam
    from ldnn.parallel.ddp import DataParallel
    from ldnn.train.graphed import GraphedDPStep, GraphedStep

    dev = torch.device("cuda", torch.cuda.current_device())
    shape = SHAPES[dataset_for(model_name)]
    nc = 1000 if model_name == "resnet18" else 10
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(batch, *shape, device=dev, generator=g).bfloat16()
    y = torch.randint(0, nc, (batch,), device=dev, generator=g)
    crit = CrossEntropyLoss()

    def opt_for(m):
        return SGD(m.parameters(), lr=0.01, momentum=0.9) if optimizer == "sgd" else Adam(m.parameters(), lr=1e-3)

    # the comm-free single-process step
    torch.manual_seed(0)
    m1 = build_model(model_name)
    xavier_init(m1)
    ldnn.prepare(m1, dev)
    o1 = opt_for(m1)
    o1.zero_grad()
    crit(m1(x), y).backward()
    o1.step()
    single = GraphedStep(m1, crit, o1, x, y, warmup=0)
    # the sharded step with stand-in collectives
    torch.manual_seed(0)
    m = build_model(model_name)
    xavier_init(m)
    ldnn.prepare(m, dev)
    comm = ShardProbeComm(dev, world, reps, blocks, gbps)
    dp = DataParallel(m, comm, bucket_cap_mb=bucket_mb, broadcast_init=False, shard_optimizer=True,
                      comm_dtype=torch.bfloat16 if comm_dtype == "bf16" else None)
    o = opt_for(m)
    o.zero_grad()
    crit(dp(x), y).backward()
    dp.finish_gradient_sync()
    o.step()
    dp.wait_gathers()
    gd = GraphedDPStep(dp, crit, o, x, y)
    bk = dp.bucketer

    def chain_only():   # the same graph chain with every collective a no-op
        comm.enabled = False
        try:
            gd(x, y)
        finally:
            comm.enabled = True

    def standin_alone():   # every collective of one step, back to back on the side stream
        joins = []
        for i, b in enumerate(bk.buckets):
            joins.append(bk.collective(i))
        bk.issue_gathers()
        for j in joins:
            if j is not None:
                j.wait()
        bk.wait_gathers()

    fns = {"single_graph_ms": lambda: single(x, y), "single_ms": chain_only, "with_standin_ms": lambda: gd(x, y),
           "standin_alone_ms": standin_alone}
    for f in fns.values():
        for _ in range(3):
            f()
    best = {k: 1e9 for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            best[k] = min(best[k], _timed(f, steps))
    # single_ms: the sharded chain with no-op collectives (its cut points included);
    # single_graph_ms: the one-graph step without data parallelism (the chain's own cost)
    hidden = best["single_ms"] + best["standin_alone_ms"] - best["with_standin_ms"]
    _tail(lambda: gd(x, y), tail_steps)
    return {"model": model_name, "batch": batch, "mode": f"sharded (world {world} stand-in)", "optimizer": optimizer,
            "grad_comm_dtype": comm_dtype,
            "bucket_mb": bucket_mb, "buckets": len(bk.buckets),
            "sharded_buckets": sum(1 for b in bk.buckets if b["sharded"]),
            "bucket_mb_each": [round((b["end"] - b["begin"]) * 4 / 2**20, 2) for b in bk.buckets],
            "segments": gd.n_segments, "forward_waits": sum(1 for w in gd.waits if w),
            "standin_reps": comm.standin.reps, "standin_blocks": comm.standin.blocks,
            "standin_calibration": comm.standin.calibration,
            **{k: round(v, 4) for k, v in best.items()}, "hidden_ms": round(hidden, 4),
            "exposed_ms": round(best["with_standin_ms"] - best["single_ms"], 4),
            "hidden_fraction": round(hidden / max(best["standin_alone_ms"], 1e-9), 3)}


def measure_mlp_sharded(world: int = 8, batch: int = 16384, hidden: int = 4096, in_features: int = 784,
                        classes: int = 10, bucket_elems: int = 8 << 20, reps: int = 1, blocks: int = 0,
                        steps: int = 20, rounds: int = 3, tail_steps: int = 0, gbps: float = 300.0,
                        comm_dtype: str = "bf16") -> dict:
    """The headline engine's sharded data-parallel step (train/static_mlp.py
    StaticMLPEngine at world ``world``, rank 0: bench.py's mlp3 784-4096-4096-10 at
    16384 samples per GPU, SGD momentum) on ONE GPU, every reduce-scatter / all-gather
    replaced by the stand-in copy of the bytes it moves over xGMI ((N-1)/N of the
    gradient bucket in ``comm_dtype``, resp. of the bf16 weight bucket).  The engine's own schedule runs:
    reduce-scatters issued between the backward's graph segments, shard updates and
    weight all-gathers in forward order, the next step's forward waiting for each
    bucket's gather right before its first GEMM.  Needs a (world-1) RCCL group for the
    engine's rank bookkeeping; nothing goes over it in the timed steps."""
    import os

    import torch.distributed as dist

    from ldnn.models.mlp import mlp3
    from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine

    dev = torch.device("cuda", torch.cuda.current_device())
    if not dist.is_initialized():
        import socket

        s_ = socket.socket()
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
        s_.close()
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev)

    def engine(w):
        torch.manual_seed(1234)
        m = mlp3(in_features, hidden, classes)
        for mod in m.modules():
            if isinstance(mod, torch.nn.Linear):
                torch.nn.init.xavier_uniform_(mod.weight)
                torch.nn.init.zeros_(mod.bias)
        e = StaticMLPEngine(m, batch, OptimConfig("sgd", lr=0.01, momentum=0.9), device=dev, world_size=w,
                            bucket_cap_elems=bucket_elems, shard_optimizer=True if w > 1 else None,
                            comm_dtype=torch.bfloat16 if (w > 1 and comm_dtype == "bf16") else None)
        g = torch.Generator(device=dev).manual_seed(3)
        e.load_batch(torch.randn(batch, in_features, device=dev, generator=g).bfloat16(),
                     torch.randint(0, classes, (batch,), device=dev, generator=g))
        return e

    single = engine(1)
    eng = engine(world)
    standin = StandInComm(dev, reps, blocks, gbps)
    state = {"on": True}

    def moved(t):
        n = t.numel() * (world - 1) // world // 8 * 8
        v = t.view(-1)[:max(n, 8)]
        return v if v.dtype == torch.float32 else v.view(torch.float32)

    def rs(i):   # (the buffer the reduce-scatter reads: the bf16 stage or the fp32 gradient)
        return standin(("rs", i), moved(eng._rs_buffers(i)[0])) if state["on"] else None

    def ag(i):
        b, e_, _ = eng.buckets[i]
        return standin(("ag", i), moved(eng.flat.shadow[b:e_])) if state["on"] else None

    eng._reduce_scatter, eng._all_gather = rs, ag
    eng._broadcast_biases = lambda bi, capturing: None   # (a few KB: not a bandwidth term)

    def chain_only():
        state["on"] = False
        try:
            eng.step()
        finally:
            state["on"] = True

    def standin_alone():
        js = [rs(i) for i in range(len(eng.buckets))] + [ag(i) for i in reversed(range(len(eng.buckets)))]
        for j in js:
            j.wait()

    def overlapped():
        eng.step()

    # prime (eager warm-up calls + the graph captures) before any timing
    for _ in range(4):
        single.step()
        chain_only()
        overlapped()
    eng.sync()
    fns = {"single_ms": single.step, "chain_ms": chain_only, "with_standin_ms": overlapped,
           "standin_alone_ms": standin_alone}
    best = {k: 1e9 for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            best[k] = min(best[k], _timed(f, steps))   # (device-wide sync at both ends)
    exposed = best["with_standin_ms"] - best["chain_ms"]
    hid = best["standin_alone_ms"] - exposed
    _tail(overlapped, tail_steps)
    eng.sync()
    return {"model": f"mlp3 {in_features}-{hidden}-{hidden}-{classes}", "batch": batch,
            "mode": f"static engine, sharded (world {world} stand-in)", "optimizer": "sgd momentum 0.9",
            "grad_comm_dtype": comm_dtype,
            "buckets": len(eng.buckets), "bucket_mb_fp32": [round((e_ - b) * 4 / 2**20, 2) for b, e_, _ in eng.buckets],
            "segments": len(eng.segments), "standin_reps": standin.reps, "standin_blocks": standin.blocks,
            "standin_calibration": standin.calibration,
            **{k: round(v, 4) for k, v in best.items()}, "exposed_ms": round(exposed, 4),
            "exposed_fraction_of_step": round(exposed / max(best["chain_ms"], 1e-9), 4),
            "hidden_ms": round(hid, 4), "hidden_fraction": round(hid / max(best["standin_alone_ms"], 1e-9), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=0,
                    help="stand-in workgroups; 0 = calibrate to --gbps (reps 1)")
    ap.add_argument("--gbps", type=float, default=300.0,
                    help="xGMI bus bandwidth the calibrated stand-in moves a collective's bytes at")
    ap.add_argument("--shard", type=int, default=0, help="world size of the sharded-step probe (0 = all-reduce step)")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    ap.add_argument("--grad-comm", choices=["fp32", "bf16"], default="bf16",
                    help="gradient collective dtype of the sharded step and of the --gossip rows")
    ap.add_argument("--gossip", action="store_true",
                    help="per-step all-reduce vs ring vs double-ring gossip rows (P2PProbeComm, world --shard or 8)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tail-steps", type=int, default=0, help="then this many overlapped steps after an idle gap "
                    "(kernel-trace timelines: scripts/probe_timeline.py)")
    a = ap.parse_args()
    if a.gossip:
        for row in measure_gossip(a.model, a.batch, a.shard or 8, a.bucket_mb, a.optimizer, a.steps, a.rounds,
                                  comm_dtype=a.grad_comm):
            print(json.dumps(row), flush=True)
        return
    if a.model == "mlp3":   # the headline engine (StaticMLPEngine), sharded at world --shard (default 8)
        print(json.dumps(measure_mlp_sharded(a.shard or 8, a.batch if a.batch != 64 else 16384, reps=a.reps,
                                             blocks=a.blocks, steps=a.steps, rounds=a.rounds,
                                             tail_steps=a.tail_steps, gbps=a.gbps, comm_dtype=a.grad_comm)),
              flush=True)
        return
    print(json.dumps(measure_overlap(a.model, a.batch, a.bucket_mb, a.reps, a.steps, rounds=a.rounds, blocks=a.blocks,
                                     shard_world=a.shard, optimizer=a.optimizer, tail_steps=a.tail_steps,
                                     gbps=a.gbps, comm_dtype=a.grad_comm)), flush=True)


if __name__ == "__main__":
    main()
