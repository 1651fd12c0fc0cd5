"""Forward-conv prototypes of round 6 (conv_lds.hip XF bits 64 / 128), one JSON line per shape.

Run once per LDNN_CONV_XF value (the knob is read once per process) and compare:
  * XF=128: B (weight) fragments loaded straight to VGPRs, only A through LDS-DMA -- the output
    must be bit-identical to XF=0 (`crc` equal), the time says whether it pays;
  * XF=64: a BatchNorm + ReLU applied to every A fragment after its LDS read (the per-fragment cost
    of folding the mid-block BN into its consumer conv; its output is not the plain conv's) --
    compare the fwd time with XF=0 plus the bn_apply pass it would remove (`bn_apply_us`).

    LDNN_CONV_XF=128 python scripts/conv_proto_ab.py --batch 256
"""
import argparse
import json
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

# (C, H, K, R, stride, pad): the 128x128 gather-kernel forward shapes of ResNet-18 @224 and EnhancedCNN @32
SHAPES = {"resnet18": [(64, 56, 128, 3, 2, 1), (128, 28, 128, 3, 1, 1), (128, 28, 256, 3, 2, 1),
                       (256, 14, 256, 3, 1, 1), (256, 14, 512, 3, 2, 1), (512, 7, 512, 3, 1, 1)],
          "enhanced_cnn": [(64, 32, 128, 3, 2, 1), (128, 16, 128, 3, 1, 1), (256, 8, 256, 3, 1, 1),
                           (512, 4, 512, 3, 1, 1)]}


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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--model", choices=list(SHAPES), default="resnet18")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    C_ = _ext._C
    assert C_ is not None, "ldnn extension not loaded"
    xf = int(os.environ.get("LDNN_CONV_XF", "0"))
    N = a.batch
    tot = 0.0
    for (C, H, K, R, st, pad) in SHAPES[a.model]:
        P = (H + 2 * pad - R) // st + 1
        g = torch.Generator(device="cuda").manual_seed(C * 1000 + H)
        x = torch.randn(N, H, H, C, device="cuda", generator=g).bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda", generator=g) * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: C_.conv_fwd(x, w, y, st, pad), a.iters)
        torch.cuda.synchronize()
        crc = zlib.crc32(y.view(torch.int16).cpu().numpy().tobytes())
        # the pass a fold would remove: BN apply + ReLU over the conv's input
        M = N * H * H
        xb, yb = x.view(M, C), torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        sm, si = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        ws = torch.zeros(C_.bn_workspace_floats(C), device="cuda")
        C_.bn_fwd(xb, yb, None, gamma, beta, rm, rv, sm, si, ws, 1e-5, 0.1, False, True, None)
        t_bn = timeit(lambda: C_.bn_fwd(xb, yb, None, gamma, beta, rm, rv, sm, si, ws, 1e-5, 0.1, False, True, None),
                      a.iters)
        tot += t
        print(json.dumps({"xf": xf, "shape": f"N{N} C{C} H{H} K{K} R{R} s{st}", "fwd_us": round(t, 2),
                          "tflops": round(2.0 * N * P * P * K * C * R * R / t / 1e6, 1), "crc": crc,
                          "bn_apply_us": round(t_bn, 2)}), flush=True)
    print(json.dumps({"xf": xf, "model": a.model, "batch": N, "fwd_total_us": round(tot, 1)}), flush=True)


if __name__ == "__main__":
    main()
