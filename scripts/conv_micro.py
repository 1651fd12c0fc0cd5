"""Per-shape conv microbenchmark: ldnn LDS-DMA conv kernels (fwd / dgrad / wgrad)
vs MIOpen via torch (channels_last bf16), TFLOP/s per pass.

    python scripts/conv_micro.py [--batch 64] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

# ResNet-18 @224 conv shapes (C, H, K, R, stride, pad); batch from --batch
SHAPES = [(64, 56, 64, 3, 1, 1), (64, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 1), (128, 28, 256, 3, 2, 1),
          (256, 14, 256, 3, 1, 1), (256, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 1), (64, 56, 128, 1, 2, 0)]
# EnhancedCNN @32 stride-1 3x3 convs (--model enhanced_cnn)
SHAPES_ECNN = [(128, 16, 128, 3, 1, 1), (256, 8, 256, 3, 1, 1), (512, 4, 512, 3, 1, 1), (1024, 2, 1024, 3, 1, 1)]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--no-stock", action="store_true")
    ap.add_argument("--model", choices=["resnet18", "enhanced_cnn"], default="resnet18")
    a = ap.parse_args()
    C_ = _ext._C
    assert C_ is not None, "ldnn extension not loaded"
    N = a.batch
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (C, H, K, R, st, pad) in (SHAPES if a.model == "resnet18" else SHAPES_ECNN):
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
        dx = torch.empty_like(x)
        dw = torch.empty(K, R, R, C, device="cuda", dtype=torch.float32)
        flops = 2.0 * N * P * P * K * C * R * R
        t = {
            "fwd": timeit(lambda: C_.conv_fwd(x, w, y, st, pad), a.iters),
            "dgrad": timeit(lambda: C_.conv_dgrad(dy, w, dx, st, pad), a.iters),
            "wgrad": timeit(lambda: C_.conv_wgrad(dy, x, dw, st, pad), a.iters),
        }
        rec = {"shape": f"N{N} C{C} H{H} K{K} R{R} s{st}"}
        for k, v in t.items():
            tot[k] += v
            rec[k + "_us"] = round(v, 2)
            rec[k + "_tf"] = round(flops / v / 1e6, 1)
        if not a.no_stock:
            xt = x.permute(0, 3, 1, 2).requires_grad_(True)  # NHWC memory = channels_last
            wt = w.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            dyt = dy.permute(0, 3, 1, 2)
            f = lambda: torch.nn.functional.conv2d(xt, wt, stride=st, padding=pad)  # noqa: E731
            out = f()
            rec["miopen_fwd_us"] = round(timeit(f, a.iters), 2)
            rec["miopen_bwd_us"] = round(timeit(lambda: torch.autograd.grad(out, (xt, wt), dyt, retain_graph=True),
                                                a.iters), 2)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
