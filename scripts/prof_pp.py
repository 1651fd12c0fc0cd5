"""Run the fwd1 MLP GEMM (16384 x 4096 x 4096, bias+ReLU) through several ldnn
variants and hipBLASLt, N times each, for rocprofv3 kernel-trace / PMC passes.
usage: python scripts/prof_pp.py [--variants 4,6,0] [--iters 20] [--shape fwd1]"""
import argparse
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from bench_gemm_pp import cases  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="4,6,0")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shape", default="fwd1")
ap.add_argument("--batch", type=int, default=16384)
a = ap.parse_args()
for name, flops, out, ref, lib, mk in cases(a.batch):
    if name != a.shape:
        continue
    fns = [lib] + [mk(int(v)) for v in a.variants.split(",")]
    for fn in fns:
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
print("done")
