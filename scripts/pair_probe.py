"""Probe: would running a layer's dgrad and wgrad side by side pay?  For EnhancedCNN / ResNet
backward conv shapes, time dgrad alone, wgrad alone, both back to back on one stream, and both on
two streams at once (eager launches, events, median of repeats).  One JSON line per shape."""
import argparse
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

SHAPES = {
    "enhanced_cnn": [(64, 128, 16, 128, 1), (64, 256, 8, 256, 1), (64, 512, 4, 512, 1), (64, 1024, 2, 1024, 1),
                     (64, 64, 32, 128, 2), (64, 128, 16, 256, 2), (64, 256, 8, 512, 2), (64, 512, 4, 1024, 2)],
    "resnet18": [(64, 64, 56, 64, 1), (64, 128, 28, 128, 1), (64, 256, 14, 256, 1), (64, 512, 7, 512, 1),
                 (64, 64, 56, 128, 2), (64, 128, 28, 256, 2), (64, 256, 14, 512, 2)],
}


def timed(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        ev[0].record()
        for _ in range(iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1000.0 / iters)
    ts.sort()
    return round(ts[2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="enhanced_cnn")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    C_ = _ext.C()
    s1 = torch.cuda.current_stream()
    s2 = torch.cuda.Stream()
    for (N, C, H, K, st) in SHAPES[a.model]:
        P = (H + 2 - 3) // st + 1
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, 3, 3, C, device="cuda") * 0.05).bfloat16()
        gy = torch.randn(N, P, P, K, device="cuda").bfloat16()
        dx = torch.empty_like(x)
        dw = torch.zeros(K, 3, 3, C, device="cuda")

        def dg():
            C_.conv_dgrad(gy, w, dx, st, 1)

        def wg():
            C_.conv_wgrad(gy, x, dw, st, 1, 0.0)

        def seq():
            dg()
            wg()

        def par():   # one fork / join around all the iterations' pairs: the concurrency alone
            s2.wait_stream(s1)
            for _ in range(a.iters):
                dg()
                with torch.cuda.stream(s2):
                    wg()
            s1.wait_stream(s2)

        def seq_all():
            for _ in range(a.iters):
                seq()

        with torch.cuda.stream(s2):   # the side stream's own workspaces exist before timing
            wg()
        torch.cuda.synchronize()
        r = {"model": a.model, "shape": [N, C, H, K, st], "dgrad_us": timed(dg, a.iters),
             "wgrad_us": timed(wg, a.iters), "seq_us": round(timed(seq_all, 1) / a.iters, 2), "par_us": round(timed(par, 1) / a.iters, 2)}
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
