"""Probe: can two RCCL ranks share one GPU on this box?  Runs one all-reduce and one
grouped send/recv ring exchange; prints a JSON line per rank.  Launch with
torch.distributed.run --nproc-per-node 2 (both ranks wrap onto cuda:0)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

import ldnn
from ldnn.utils import distributed as D


def main():
    ctx = D.setup("nccl")
    r, n = ctx.rank, ctx.world_size
    x = torch.full((1 << 20,), float(r + 1), device=ctx.device)
    dist.all_reduce(x)
    ok_ar = bool((x == n * (n + 1) / 2).all().item())
    send = torch.full((4096,), float(r), device=ctx.device)
    recv = torch.empty_like(send)
    ops = [dist.P2POp(dist.isend, send, (r + 1) % n), dist.P2POp(dist.irecv, recv, (r - 1) % n)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    ok_p2p = bool((recv == float((r - 1) % n)).all().item())
    print(json.dumps({"rank": r, "world": n, "device": str(ctx.device), "backend": ctx.backend,
                      "allreduce_ok": ok_ar, "sendrecv_ok": ok_p2p}), flush=True)
    D.teardown(ctx)


if __name__ == "__main__":
    main()
