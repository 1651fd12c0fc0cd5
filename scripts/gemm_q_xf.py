"""gemm_q pipeline experiments on a bias+ReLU forward shape (default the headline
M 16384, N 4096, K 4096; --K 784 = the first layer): variant 32 = production, 33 = no
in-loop LDS-DMA (operands stale after tile 1), 34 = no DMA wait, 36 = no in-loop
fragment reads, 37 = neither DMA nor reads, 96 = no epilogue, 160 = epilogue without
its global stores.  Results are wrong for the knockouts by construction: only the time
is of interest -- which part of the kernel sets its time.

    python scripts/gemm_q_xf.py [--M 16384] [--N 4096] [--K 4096] [--variants 32,33,96,160]
"""
import argparse
import json
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
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=16384)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--variants", default="32,33,64,36,37,40,48")
    a = ap.parse_args()
    M, N, K = a.M, a.N, a.K
    x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    for rep in range(2):
        for v in (int(t) for t in a.variants.split(",")):
            t = min(timeit(lambda: C.gemm(x, w, c, True, True, C.EPI_BIAS_RELU, bias=bias, tile=256, variant=v))
                    for _ in range(3))
            print(json.dumps({"M": M, "N": N, "K": K, "rep": rep, "variant": v, "us": round(t, 1),
                              "tflops": round(fl / t / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
