"""Run one GEMM configuration repeatedly (for rocprofv3 counter collection)."""
import argparse
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402
from ldnn.ops import _ext  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=4096)
ap.add_argument("--N", type=int, default=4096)
ap.add_argument("--K", type=int, default=4096)
ap.add_argument("--akc", type=int, default=1)
ap.add_argument("--bkc", type=int, default=1)
ap.add_argument("--tile", type=int, default=256)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--torch", action="store_true")
a = ap.parse_args()
C = _ext.C()
A = (torch.rand(a.M, a.K, device="cuda") * 2 - 1 if a.akc else torch.rand(a.K, a.M, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(a.N, a.K, device="cuda") * 2 - 1 if a.bkc else torch.rand(a.K, a.N, device="cuda") * 2 - 1).bfloat16()
Cm = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
for _ in range(a.iters):
    if a.torch:
        torch.matmul(A if a.akc else A.t(), B.t() if a.bkc else B)
    else:
        C.gemm(A, B, Cm, bool(a.akc), bool(a.bkc), tile=a.tile)
torch.cuda.synchronize()
