"""Correctness of the static engine's multi-rank path (bucketed async all-reduce
between graph segments, per-bucket optimizer segments): N ranks with per-rank
batches must end with the same parameters as ONE rank on the concatenated batch.

Run:  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
          scripts/check_static_dp.py --backend gloo      (2 ranks may share one GPU)
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402
from ldnn.models.mlp import mlp3  # noqa: E402
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine  # noqa: E402
from ldnn.utils import distributed as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--graphs", type=int, default=1)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--cap", type=int, default=1 << 17)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--shard", type=int, default=-1, help="-1 auto (on for N > 1), 0 off, 1 on")
    ap.add_argument("--tail", type=str, default="",
                    help="comma-separated per-rank sample counts of one final dp_tail_step (e.g. '2,0': rank 0's "
                         "partial batch of 2, rank 1 without data); the reference then trains the concatenated "
                         "tail with eager_step")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    ap.add_argument("--comm-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="gradient reduce-scatter dtype of the sharded step (bf16: widened into the fp32 shard)")
    ap.add_argument("--tol", type=float, default=2e-2,
                    help="max |param - reference| allowed, relative to the tensor's max |param| (+ 1e-3 absolute)")
    a = ap.parse_args()
    ctx = D.setup(a.backend)
    N, r = ctx.world_size, ctx.rank
    B, H = a.batch, a.hidden
    torch.manual_seed(0)
    model = mlp3(784, H, 10)
    # small bucket cap -> several buckets / segments on the multi-rank path
    cfg = OptimConfig("sgd", lr=0.05, momentum=0.9) if a.optimizer == "sgd" else OptimConfig("adam", lr=1e-3)
    eng = StaticMLPEngine(model, B, cfg, device=ctx.device, world_size=N,
                          bucket_cap_elems=a.cap, use_graphs=bool(a.graphs),
                          shard_optimizer=None if a.shard < 0 else bool(a.shard),
                          comm_dtype=torch.bfloat16 if a.comm_dtype == "bf16" else None)
    print(f"rank {r}: shard={eng.shard} comm_bf16={eng.comm_bf16 if eng.shard else False}", flush=True)
    print(f"rank {r}: buckets {eng.buckets}", flush=True)
    g = torch.Generator(device="cpu").manual_seed(5)
    S = a.steps
    xs = [torch.randn(N * B, 784, generator=g) for _ in range(S)]
    ys = [torch.randint(0, 10, (N * B,), generator=g) for _ in range(S)]
    for i in range(S):
        eng.reset_stats()
        eng.load_batch(xs[i][r * B:(r + 1) * B].to(ctx.device).bfloat16(), ys[i][r * B:(r + 1) * B].to(ctx.device))
        eng.step()
        torch.cuda.synchronize()
        print(f"rank {r} step {i} loss {eng.read_stats(B)[0]:.5f} finite={bool(torch.isfinite(eng.flat.shadow).all())}",
              flush=True)
    tails = [int(v) for v in a.tail.split(",")] if a.tail else []
    if tails:
        assert len(tails) == N
        gt = torch.Generator(device="cpu").manual_seed(6)
        xt = torch.randn(sum(tails), 784, generator=gt)
        yt = torch.randint(0, 10, (sum(tails),), generator=gt)
        o = sum(tails[:r])
        n = tails[r]
        eng.dp_tail_step(xt[o:o + n].to(ctx.device).bfloat16() if n else None, yt[o:o + n].to(ctx.device) if n else None)
        torch.cuda.synchronize()
    # the forward reads the fp32 master biases: they must agree on every rank after
    # sharded updates too (each rank updates only its shard of the master)
    eng.sync()
    bm = torch.cat([eng.bias[l].detach().float().flatten() for l in range(len(eng.bias))])
    bmx, bmn = bm.clone(), bm.clone()
    if N > 1:
        dist.all_reduce(bmx, op=dist.ReduceOp.MAX)
        dist.all_reduce(bmn, op=dist.ReduceOp.MIN)
    bias_ok = bool(torch.equal(bmx, bmn))
    if r == 0:
        print("BIASES_CONSISTENT" if bias_ok else
              f"BIASES_STALE max spread {(bmx - bmn).abs().max().item():.3e}", flush=True)
    eng.gather_master()   # sharded optimizer: make the fp32 master whole on every rank
    torch.cuda.synchronize()
    got = eng.flat.master.detach().cpu().clone()
    sh = eng.flat.shadow.detach().float().cpu()
    print(f"rank {r}: shadow == bf16(master): "
          f"{bool(torch.equal(sh, eng.flat.master.detach().bfloat16().float().cpu()))}", flush=True)
    if r == 0:
        # single-rank reference on the concatenated batch (same kernels, no graphs)
        torch.manual_seed(0)
        ref = StaticMLPEngine(mlp3(784, H, 10), N * B, cfg, device=ctx.device, world_size=1, use_graphs=False)
        for i in range(S):
            ref.load_batch(xs[i].to(ctx.device).bfloat16(), ys[i].to(ctx.device))
            ref.step()
        if tails and sum(tails):
            ref.eager_step(xt.to(ctx.device).bfloat16(), yt.to(ctx.device))
        torch.cuda.synchronize()
        # map the two flat layouts through the named parameters
        ok = True
        for (n1, p1), (n2, p2) in zip(eng.model.named_parameters(), ref.model.named_parameters()):
            d = (p1.detach().cpu() - p2.detach().cpu()).abs().max().item()
            scale = p2.detach().abs().max().item() + 1e-6
            print(f"{n1}: max|diff| = {d:.3e} (scale {scale:.3e})")
            ok &= d <= a.tol * scale + 1e-3
        ok &= bias_ok
        print("STATIC_DP_OK" if ok else "STATIC_DP_MISMATCH", flush=True)
    # every rank holds identical parameters
    t = got.to(ctx.device)
    mx, mn = t.clone(), t.clone()
    if N > 1:
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    if r == 0:
        print("REPLICAS_IDENTICAL" if torch.equal(mx, mn) else "REPLICAS_DIVERGED", flush=True)
    D.teardown(ctx)


if __name__ == "__main__":
    main()
