"""Do independent branches of a captured hipGraph run concurrently on MI355X?
A chain of K small kernels on one stream vs the same kernels split over two / four
forked streams inside one capture; prints replay time per graph."""
import json
import sys

import torch


def build(nstreams, K, numel):
    xs = [torch.zeros(numel, device="cuda") for _ in range(nstreams)]
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    g = torch.cuda.CUDAGraph()
    main = torch.cuda.current_stream()
    with torch.cuda.graph(g):
        cap = torch.cuda.current_stream()
        for s in streams:
            s.wait_stream(cap)
        for i in range(K):
            s = streams[i % nstreams]
            with torch.cuda.stream(s):
                xs[i % nstreams].add_(1.0)
        for s in streams:
            cap.wait_stream(s)
    return g


def bench(g, it=50):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


for numel in (1024, 1 << 20, 8 << 20):
    r = {"numel": numel, "K": 64}
    for ns in (1, 2, 4):
        r[f"us_{ns}streams"] = round(bench(build(ns, 64, numel)), 1)
    print(json.dumps(r), flush=True)
