"""gemm_q pipeline experiments on the headline forward shape (M 16384, N 4096, K 4096,
bias+ReLU): variant 32 = production, 33 = no in-loop LDS-DMA (operands stale after
tile 1), 34 = no DMA wait, 36 = no in-loop fragment reads, 37 = neither DMA nor reads.
Results are wrong for 33-37 by construction: only the time is of interest -- which
part of the loop sets the K-tile time."""
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


M, N, K = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, 4096, 4096
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
bias = torch.randn(N, device="cuda")
fl = 2.0 * M * N * K
for rep in range(2):
    for v in (32, 33, 64, 36, 37, 40, 48):
        t = min(timeit(lambda: C.gemm(a, b, c, True, True, C.EPI_BIAS_RELU, bias=bias, tile=256, variant=v))
                for _ in range(3))
        print(json.dumps({"rep": rep, "variant": v, "us": round(t, 1), "tflops": round(fl / t / 1e6, 1)}), flush=True)
