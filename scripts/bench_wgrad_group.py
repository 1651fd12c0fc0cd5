"""wgrad-shape sweep of the four-wave GEMM's tile grouping (variant bits 8..11: G =
2^(gsel-1) tile-rows per group, 0 = default 4) at the mlp3 wgrad shapes, plus
hipBLASLt for reference.  Prints one JSON line per shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def t(fn, it=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


B = 16384
for M, N in ((4096, 4096),):
    dy = torch.randn(B, M, device="cuda").bfloat16()
    x = torch.randn(B, N, device="cuda").bfloat16()
    dw = torch.empty(M, N, device="cuda")
    fns = {f"g{gs}": (lambda gs=gs: C.gemm(dy, x, dw, False, False, tile=256, variant=32 | (gs << 8)))
           for gs in (0, 1, 2, 4, 5, 6)}
    fns["hipblaslt"] = lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=dw)
    best = {k: 1e9 for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            best[k] = min(best[k], t(f))
    print(json.dumps({"M": M, "N": N, "K": B, **{k + "_us": round(v, 1) for k, v in best.items()}}), flush=True)
