"""Fixed-vs-per-K cost of the MLP forward GEMM: time(K) at M=16384, N=4096 for K in a
sweep; a linear fit separates the per-tile prologue/epilogue from the K loop."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()
M, N = 16384, 4096
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "32,0").split(",")]
for K in (512, 1024, 2048, 4096, 8192):
    h = ((torch.rand(M, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    W = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).bfloat16()
    bias = torch.rand(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = {"K": K}
    fns = {f"v{v}": (lambda v=v: C.gemm(h, W, y, True, True, C.EPI_BIAS_RELU, bias=bias, tile=256, variant=v))
           for v in variants}
    fns["lib"] = lambda: torch._addmm_activation(bias.bfloat16(), h, W.t(), out=y)
    best = {k: 1e9 for k in fns}
    for fn in fns.values():
        fn()
    for _ in range(5):
        for k, fn in fns.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            best[k] = min(best[k], e0.elapsed_time(e1) * 100)
    row.update({k: round(v, 1) for k, v in best.items()})
    print(json.dumps(row), flush=True)
