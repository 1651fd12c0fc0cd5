"""Micro bench of the ResNet-18 classifier head's GEMMs (64 x 512 -> 1000) and the
global average pool: the current dispatch vs split-K / other tilings.

    python scripts/bench_fc_head.py --batch 64
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--k", type=int, default=512)
    ap.add_argument("--n", type=int, default=1000)
    a = ap.parse_args()
    C = _ext.C()
    dev = torch.device("cuda:0")
    B, K, N = a.batch, a.k, a.n
    x = torch.randn(B, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16() * 0.05
    b = torch.randn(N, device=dev)
    y = torch.empty(B, N, dtype=torch.bfloat16, device=dev)
    gz = torch.randn(B, N, device=dev).bfloat16()
    dw = torch.zeros(N, K, device=dev)
    dx = torch.empty(B, K, dtype=torch.bfloat16, device=dev)
    ref_y = (x.float() @ w.float().t() + b)
    ref_dw = gz.float().t() @ x.float()
    ref_dx = gz.float() @ w.float()
    out = []

    def rec(name, us, err):
        out.append({"batch": B, "op": name, "us": round(us, 2), "maxerr": err})
        print(json.dumps(out[-1]), flush=True)

    # forward: bias epilogue, bf16 out
    f = lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS, bias=b)
    rec("fwd_default", timed(f), (y.float() - ref_y).abs().max().item())
    for sk in (2, 4, 8):
        if K // sk < 64:
            continue
        ne, nc = C.gemm_splitk_ws(B, N, sk)
        ws = torch.empty(ne, device=dev)
        cnt = torch.zeros(nc, dtype=torch.int32, device=dev)
        f = lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS, bias=b, tile=128, splitk=sk, ws=ws, cnt=cnt)
        y.zero_()
        rec(f"fwd_sk{sk}", timed(f), (y.float() - ref_y).abs().max().item())
    # wgrad: dW[N][K] = gz^T x, fp32 out
    f = lambda: C.gemm(gz, x, dw, False, False, beta=0.0)
    rec("wgrad_default", timed(f), (dw - ref_dw).abs().max().item())
    for tile in (128, 256):
        f = lambda: C.gemm(gz, x, dw, False, False, beta=0.0, tile=tile, splitk=1)
        rec(f"wgrad_tile{tile}", timed(f), (dw - ref_dw).abs().max().item())
    # dgrad: dx = gz W, bf16 out
    f = lambda: C.gemm(gz, w, dx, True, False)
    rec("dgrad_default", timed(f), (dx.float() - ref_dx).abs().max().item())
    for sk in (2, 4, 8):
        ne, nc = C.gemm_splitk_ws(B, K, sk)
        ws = torch.empty(ne, device=dev)
        cnt = torch.zeros(nc, dtype=torch.int32, device=dev)
        f = lambda: C.gemm(gz, w, dx, True, False, tile=128, splitk=sk, ws=ws, cnt=cnt)
        rec(f"dgrad_sk{sk}", timed(f), (dx.float() - ref_dx).abs().max().item())
    # global average pool of the last stage (B x 7 x 7 x 512, channels-last)
    h = torch.randn(B, 49, K, device=dev).bfloat16()
    g = torch.empty(B, K, dtype=torch.bfloat16, device=dev)
    f = lambda: C.gap_fwd(h, g)
    rec("gap_fwd", timed(f), (g.float() - h.float().mean(1)).abs().max().item())

if __name__ == "__main__":
    main()
