"""Per-step gossip / weighted all-reduce on the static MLP engine (StaticMLPEngine
grad_mix) == the reference formulas evaluated by FakeWorld on the ranks' own gradients.

Each rank trains its OWN replica (decentralised SGD).  Per step t, every rank also
computes its plain local gradient g_r at its current weights with a world-1 engine
(SGD, lr 1, no momentum: g = W - W'), the ranks all-gather those, and FakeWorld runs
parallel.aggregation's gossip_mix / allreduce_mix on them in fp32 -- the expected
mixed gradient.  The distributed engine's update (SGD lr, no momentum) must equal
lr x that.  Reference: Balanced Ring/communication.py:5-62, Balanced
Double-Ring/communication.py:5-77, Balanced All-Reduce/communication.py:4-18.

Run:  python -m torch.distributed.run --nproc-per-node 3 --master-addr 127.0.0.1 \
          scripts/check_engine_gossip.py --hops 1 [--weight 0.7]
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402,F401
from ldnn.models.mlp import mlp3  # noqa: E402
from ldnn.parallel import aggregation as A  # noqa: E402
from ldnn.parallel.comm import FakeWorld  # noqa: E402
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine  # noqa: E402
from ldnn.utils import distributed as D  # noqa: E402


def flat_params(m):
    return torch.cat([p.detach().float().flatten() for p in m.parameters()])


def load_params(m, v):
    o = 0
    with torch.no_grad():
        for p in m.parameters():
            n = p.numel()
            p.copy_(v[o:o + n].view_as(p))
            o += n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hops", type=int, default=1, help="0 = all-reduce (weighted), 1 ring, 2 double ring")
    ap.add_argument("--weight", type=float, default=None, help="local_weight (None = equal)")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--lr", type=float, default=0.05)
    a = ap.parse_args()
    ctx = D.setup("gloo")
    N, r, dev = ctx.world_size, ctx.rank, ctx.device
    B, H = a.batch, a.hidden
    torch.manual_seed(0)
    model = mlp3(784, H, 10)
    eng = StaticMLPEngine(model, B, OptimConfig("sgd", lr=a.lr, momentum=0.0), device=dev, world_size=N,
                          bucket_cap_elems=1 << 17, use_graphs=True, grad_mix=(a.hops, a.weight))
    assert len(eng.buckets) >= 2, eng.buckets
    assert not eng.shard or (a.hops == 0 and a.weight is None)
    torch.manual_seed(0)
    rm = mlp3(784, H, 10)
    ref = StaticMLPEngine(rm, B, OptimConfig("sgd", lr=1.0, momentum=0.0), device=dev, world_size=1,
                          use_graphs=False)
    g = torch.Generator(device="cpu").manual_seed(11 + r)
    worst = 0.0
    for t in range(a.steps):
        x = torch.randn(B, 784, generator=g).to(dev).bfloat16()
        y = torch.randint(0, 10, (B,), generator=g).to(dev)
        w0 = flat_params(model)
        # this rank's own gradient at its current weights
        load_params(rm, w0)
        ref.flat.refresh_shadow()
        ref.load_batch(x, y)
        ref.step()
        torch.cuda.synchronize()
        gl = (w0 - flat_params(rm)).cpu()
        allg = [torch.zeros_like(gl) for _ in range(N)]
        dist.all_gather(allg, gl)
        # the reference formulas on every rank's gradient (FakeWorld, fp32)
        if a.hops == 0:
            exp = FakeWorld(N).run(lambda c: (lambda v: (A.allreduce_mix(v, c, a.weight is not None,
                                                                         a.weight or 0.0), v)[1])(allg[c.rank].clone()))
        else:
            exp = FakeWorld(N).run(lambda c: (lambda v: (A.gossip_mix(v, c, a.hops, a.weight is not None,
                                                                      a.weight or 0.5), v)[1])(allg[c.rank].clone()))
        eng.load_batch(x, y)
        eng.step()
        torch.cuda.synchronize()
        got = ((w0 - flat_params(model)) / a.lr).cpu()
        e = exp[r]
        err = ((got - e).norm() / e.norm().clamp_min(1e-12)).item()
        worst = max(worst, err)
        print(f"rank {r} step {t}: rel err {err:.3e}", flush=True)
    t = torch.tensor([worst])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if r == 0:
        print(f"worst {t.item():.3e}", flush=True)
        if t.item() < 2e-3:
            print("ENGINE_GOSSIP_OK", flush=True)
    D.teardown(ctx)


if __name__ == "__main__":
    main()
