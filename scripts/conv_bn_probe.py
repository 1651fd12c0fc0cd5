"""Cost of the fused BatchNorm-statistics conv epilogue: ldnn conv_fwd per ResNet-18 @224
shape with and without the next BN's statistics accumulated + finalized in the epilogue,
on ReLU-like inputs (half zeros).

    python scripts/conv_bn_probe.py [--batch 64] [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

SHAPES = [(64, 56, 64, 3, 1, 1), (64, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 1), (128, 28, 256, 3, 2, 1),
          (256, 14, 256, 3, 1, 1), (256, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 1), (64, 56, 128, 1, 2, 0)]


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
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    C_ = _ext.C()
    N = a.batch
    for (C, H, K, R, st, pad) in SHAPES:
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, C, device="cuda").clamp_min(0).bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        ws = torch.zeros(C_.bn_workspace_floats(K), device="cuda")
        g = torch.ones(K, device="cuda")
        b = torch.zeros(K, device="cuda")
        rm = torch.zeros(K, device="cuda")
        rv = torch.ones(K, device="cuda")
        sm = torch.empty(K, device="cuda")
        si = torch.empty(K, device="cuda")
        flops = 2.0 * N * P * P * K * C * R * R
        t0 = timeit(lambda: C_.conv_fwd(x, w, y, st, pad), a.iters)
        t1 = timeit(lambda: C_.conv_fwd(x, w, y, st, pad, None, 0, bn_ws=ws, bn_gamma=g, bn_beta=b,
                                        bn_running_mean=rm, bn_running_var=rv, bn_save_mean=sm,
                                        bn_save_invstd=si, bn_eps=1e-5, bn_momentum=0.1), a.iters)
        print(json.dumps({"shape": f"N{N} C{C} H{H} K{K} R{R} s{st}", "plain_us": round(t0, 2),
                          "bn_stats_us": round(t1, 2), "plain_tf": round(flops / t0 / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
