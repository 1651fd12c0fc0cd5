"""ResNet-18 layer-1 conv passes (64 -> 64 channels, 3x3 stride 1, 56 x 56): the weight-
stationary persistent kernel (set_conv_ws 1), and the ResNet 7x7 / 2 stem (conv_patch_ws_kernel vs
conv_patch_kernel, with the fused BN statistics)
against the halo kernel (set_conv_ws 0).  One JSON line per (batch, mode): median us of 20
event-timed launches for fwd (with the fused BN statistics when --bn) and dgrad.

    python scripts/bench_ws64.py [--batches 64,256]
    (the LDNN_CONV_XF=1|2|4|7 knockout builds of the ws64 forward were removed in round 6;
    profiles/r4/conv_ws64_micro.jsonl holds their results)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="64,256")
    ap.add_argument("--modes", default="0,1")
    ap.add_argument("--fwd-only", action="store_true", help="time the forward pass only")
    ap.add_argument("--no-stem", action="store_true")
    a = ap.parse_args()
    for N in (int(b) for b in a.batches.split(",")):
        x = torch.randn(N, 56, 56, 64, device="cuda").bfloat16()
        w = (torch.randn(64, 3, 3, 64, device="cuda") * 0.04).bfloat16()
        y = torch.empty_like(x)
        gy = torch.randn_like(x)
        dx = torch.empty_like(x)
        fl = 2.0 * N * 56 * 56 * 64 * 576
        for m in (int(t) for t in a.modes.split(",")):
            C.set_conv_ws(m)
            f = timeit(lambda: C.conv_fwd(x, w, y, 1, 1))
            d = None if a.fwd_only else timeit(lambda: C.conv_dgrad(gy, w, dx, 1, 1))
            print(json.dumps({"batch": N, "ws_mode": m, "fwd_us": f, "dgrad_us": d, "fwd_tf": round(fl / f / 1e6, 1),
                              "dgrad_tf": round(fl / d / 1e6, 1) if d else None,
                              "xf": os.environ.get("LDNN_CONV_XF", "0")}), flush=True)
        C.set_conv_ws(1)
        if a.no_stem:
            continue
        # the 7x7 / 2 stem (conv_patch_ws_kernel vs conv_patch_kernel), with the fused BN statistics
        xs = torch.zeros(N, 224, 224, 8, device="cuda", dtype=torch.bfloat16)
        xs[..., :3] = torch.randn(N, 224, 224, 3, device="cuda").bfloat16()
        ws_ = (torch.randn(64, 7, 7, 8, device="cuda") * 0.05).bfloat16()
        ys = torch.empty(N, 112, 112, 64, device="cuda", dtype=torch.bfloat16)
        bw = torch.zeros(C.bn_workspace_floats(64), device="cuda")
        sm, si = torch.zeros(64, device="cuda"), torch.zeros(64, device="cuda")
        fls = 2.0 * N * 112 * 112 * 64 * 49 * 3
        for m in (int(t) for t in a.modes.split(",")):
            C.set_conv_ws(m)
            f = timeit(lambda: C.conv_fwd(xs, ws_, ys, 2, 3, bn_ws=bw, bn_save_mean=sm, bn_save_invstd=si))
            print(json.dumps({"batch": N, "ws_mode": m, "stem_fwd_bn_us": f, "stem_tf_real": round(fls / f / 1e6, 1),
                              "xf": os.environ.get("LDNN_CONV_XF", "0")}), flush=True)
        C.set_conv_ws(1)


if __name__ == "__main__":
    main()
