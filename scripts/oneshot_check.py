"""Two-or-more-rank check of the one-shot IPC all-reduce (parallel/ipc.py), every rank
on cuda:0 of the one-GPU box (RCCL refuses duplicate devices, so the process group is
gloo; the one-shot kernels themselves only use HIP IPC).  Checks fp32 and bf16 sums
against the expected values over many back-to-back calls (staging halves alternate),
the kernel captured into a hipGraph and replayed 20 times (device-side epochs), the
self-test, and times it; prints one JSON line per rank.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/oneshot_check.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

import ldnn  # noqa: F401
from ldnn.parallel.ipc import OneShotAllReduce
from ldnn.utils import distributed as D


def main():
    ctx = D.setup("gloo")
    r, n = ctx.rank, ctx.world_size
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os_ = OneShotAllReduce(1 << 20, device=dev, blocks=32)
    if os_.connect_error is not None:
        raise os_.connect_error
    ok = True
    for it in range(50):
        for dt, numel in ((torch.float32, 1 << 16), (torch.bfloat16, 4096 + 8), (torch.float32, 8)):
            base = torch.arange(numel, device=dev, dtype=torch.float32) % 97
            t = (base * (r + 1) + it).to(dt)
            os_.all_reduce(t)
            want = (base * (n * (n + 1) / 2) + n * it).to(dt).float()
            tol = 0 if dt == torch.float32 else 2e-2 * want.abs().max().item()
            if not torch.allclose(t.float(), want, rtol=0, atol=tol):
                ok = False
    torch.cuda.synchronize()
    os_.check()
    # captured into a hipGraph and replayed: every replay is a new call (device-side
    # epochs): the sum must follow the input each time
    buf = torch.zeros(4096, device=dev)
    src = torch.zeros(4096, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        buf.copy_(src)
        os_.all_reduce(buf)
    torch.cuda.current_stream().wait_stream(side)
    for it in range(20):
        src.fill_(float(r + 1) * (it + 1))
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        want = (it + 1) * n * (n + 1) / 2
        if not torch.all(buf == want):
            ok = False
    os_.check()
    ok = ok and os_.self_test()
    x = torch.ones(1 << 18, device=dev)
    for _ in range(5):
        os_.all_reduce(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        os_.all_reduce(x)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 100 * 1e6
    dist.barrier()
    print(json.dumps({"rank": r, "world": n, "ok": ok, "calls": os_._c.calls,
                      "oneshot_1MB_fp32_us": round(us, 1)}), flush=True)
    D.teardown(ctx)
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
