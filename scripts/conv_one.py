"""Run one conv shape's fwd + stride-1 dgrad N times (for PMC / trace runs).

    python scripts/conv_one.py --C 128 --H 28 --K 128 [--R 3 --stride 1 --batch 64 --iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--C", type=int, default=128)
    ap.add_argument("--H", type=int, default=28)
    ap.add_argument("--K", type=int, default=128)
    ap.add_argument("--R", type=int, default=3)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C_ = _ext._C
    N, C, H, K, R, st = a.batch, a.C, a.H, a.K, a.R, a.stride
    pad = R // 2
    P = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
    y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    dx = torch.empty_like(x)
    for _ in range(a.iters):
        C_.conv_fwd(x, w, y, st, pad)
        C_.conv_dgrad(dy, w, dx, st, pad)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
