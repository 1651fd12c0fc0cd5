"""Graph-captured per-step DP (GraphedDPStep through train_local_epoch) on N ranks
== ONE graphed rank on the concatenated batches.

Run:  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
          scripts/check_graphed_dp.py        (gloo; the ranks may share one GPU)
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402
from ldnn.optim import SGD, Adam  # noqa: E402
from ldnn.parallel.comm import TorchComm  # noqa: E402
from ldnn.parallel.ddp import DataParallel  # noqa: E402
from ldnn.train.trainer import train_local_epoch  # noqa: E402
from ldnn.utils import distributed as D  # noqa: E402


class ListLoader:
    def __init__(self, batches):
        self.batches = batches

    def __len__(self):
        return len(self.batches)

    def __iter__(self):
        return iter(self.batches)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--model", default="lenet5")
    ap.add_argument("--batch", type=int, default=128, help="per rank")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--oneshot", action="store_true",
                    help="also train with the one-shot IPC all-reduce on (buckets <= 4 MiB) and require "
                         "the same parameters as with it off")
    ap.add_argument("--shard", action="store_true",
                    help="DataParallel(shard_optimizer=True): reduce-scatter + sharded optimizer + weight all-gather")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32")
    ap.add_argument("--gossip", type=int, default=0,
                    help="1 / 2: per-step ring / double-ring gossip (DataParallel(gossip=...)): the graphed chain "
                         "must give the parameters of the eager bucketed gossip step (replicas differ by design)")
    a = ap.parse_args()
    ctx = D.setup(a.backend)
    N, r, dev = ctx.world_size, ctx.rank, ctx.device
    B = a.batch
    shape = {"lenet5": (1, 28, 28)}.get(a.model, (3, 32, 32))
    g = torch.Generator(device="cpu").manual_seed(5)
    xs = [torch.randn(N * B, *shape, generator=g) for _ in range(a.steps)]
    ys = [torch.randint(0, 10, (N * B,), generator=g) for _ in range(a.steps)]
    # the last batch is odd-shaped: the eager bucketed fallback runs too
    xs.append(xs[0][: N * (B // 2)])
    ys.append(ys[0][: N * (B // 2)])

    def run(world, rank, comm, graphs=True):
        torch.manual_seed(0)
        m = build_model(a.model)
        xavier_init(m)
        ldnn.prepare(m, dev)
        cd = torch.bfloat16 if a.comm_dtype == "bf16" else None
        dp = (DataParallel(m, comm, bucket_cap_mb=0.05, shard_optimizer=a.shard, comm_dtype=cd, gossip=a.gossip,
                           local_weight=0.7 if a.gossip == 2 else None)
              if comm is not None else None)
        # (built after the wrapper: sharding re-lays the flat buffers out)
        opt = SGD(m.parameters(), lr=0.02, momentum=0.9) if a.optimizer == "sgd" else Adam(m.parameters(), lr=1e-3)
        batches = []
        for x, y in zip(xs, ys):
            b = x.shape[0] // world
            batches.append((x[rank * b:(rank + 1) * b].to(dev).bfloat16(), y[rank * b:(rank + 1) * b].to(dev)))
        net = dp if dp is not None else m
        loss, acc, bl = train_local_epoch(net, ListLoader(batches), CrossEntropyLoss(), opt, dev, graphs=graphs,
                                          dp=dp)
        if dp is not None:
            if a.shard:
                assert dp.sharded and any(b["sharded"] for b in dp.bucketer.buckets)
            dp.gather_master(opt)   # collective: whole fp32 master on every rank
        torch.cuda.synchronize()
        return m, bl

    m, bl = run(N, r, TorchComm())
    got = torch.cat([p.detach().flatten().cpu() for p in m.parameters()])
    print(f"rank {r}: batch losses {[round(v, 4) for v in bl]}", flush=True)
    ok = True
    if a.gossip:
        me, _ = run(N, r, TorchComm(), graphs=False)
        ref = torch.cat([p.detach().flatten().cpu() for p in me.parameters()])
        torch.manual_seed(0)
        m0 = build_model(a.model)
        xavier_init(m0)
        p0 = torch.cat([p.detach().flatten() for p in m0.parameters()])
        du, dr = (got - p0).double(), (ref - p0).double()
        err = (du - dr).norm().item() / max(dr.norm().item(), 1e-12)
        print(f"rank {r}: gossip graphed vs eager relative update difference {err:.3e}", flush=True)
        t = torch.tensor([1.0 if err < 1e-2 else 0.0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        if r == 0 and t.item() == 1.0:
            print("GRAPHED_DP_OK", flush=True)
        D.teardown(ctx)
        return
    if a.oneshot:
        c1 = TorchComm()
        os_ = c1.enable_oneshot(4 << 20, device=dev)
        assert os_ is not None, "one-shot self-test failed"
        calls0 = os_._c.calls
        m1, _ = run(N, r, c1)
        c1.check_errors()
        used = os_._c.calls - calls0
        got1 = torch.cat([p.detach().flatten().cpu() for p in m1.parameters()])
        diff = (got1 - got).abs().max().item()
        scale = got.abs().max().item()
        print(f"rank {r}: one-shot calls {used}, max |params(one-shot) - params(gloo)| {diff:.3e}", flush=True)
        ok = ok and used > 0 and diff <= 1e-6 * max(scale, 1.0)
    if r == 0:
        ref_m, ref_bl = run(1, 0, None)
        ref = torch.cat([p.detach().flatten().cpu() for p in ref_m.parameters()])
        torch.manual_seed(0)
        m0 = build_model(a.model)
        xavier_init(m0)
        p0 = torch.cat([p.detach().flatten() for p in m0.parameters()])
        du, dr = (got - p0).double(), (ref - p0).double()
        err = (du - dr).norm().item() / max(dr.norm().item(), 1e-12)
        print(f"relative update difference vs single rank: {err:.3e}", flush=True)
        ok = ok and err < (2e-2 if a.comm_dtype == "fp32" else 5e-2)
    t = torch.tensor([1.0 if ok else 0.0])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    others = [torch.zeros_like(got) for _ in range(N)]
    dist.all_gather(others, got)
    same = all(torch.equal(others[0], o) for o in others)
    if r == 0:
        print("REPLICAS_IDENTICAL" if same else "REPLICAS_DIFFER", flush=True)
        if t.item() == 1.0 and same:
            print("GRAPHED_DP_OK", flush=True)
    D.teardown(ctx)


if __name__ == "__main__":
    main()
