"""wgrad GEMM (dW = dz^T h, both operands batch-major) tile / split-K sweep for the
MLP engine's layers.  python scripts/bench_wgrad.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402


def timeit(fn, iters=30):
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
    C = _ext._C
    assert C is not None
    B = 4096
    ref = None  # noqa: F841
    for (M, N) in [(4096, 784), (4096, 4096)]:
        dz = torch.randn(B, M, device="cuda").bfloat16()
        h = torch.randn(B, N, device="cuda").bfloat16()
        dW = torch.empty(M, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * B
        ref = (dz.float().t() @ h.float())
        for tile, sk in [(0, 0), (256, 1), (128, 1), (128, 2), (128, 3), (128, 4), (128, 6), (128, 8)]:
            ws = cnt = None
            if tile == 128 and sk > 1:
                ne, nc = C.gemm_splitk_ws(M, N, sk)
                ws = torch.empty(ne, dtype=torch.float32, device="cuda")
                cnt = torch.zeros(nc, dtype=torch.int32, device="cuda")
            fn = lambda: C.gemm(dz, h, dW, False, False, tile=tile, splitk=sk, ws=ws, cnt=cnt)  # noqa: E731
            try:
                us = timeit(fn)
            except Exception as ex:  # noqa: BLE001
                print(json.dumps({"M": M, "N": N, "tile": tile, "splitk": sk, "error": str(ex)[:120]}), flush=True)
                continue
            fn()
            torch.cuda.synchronize()
            err = ((dW - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"M": M, "N": N, "tile": tile, "splitk": sk, "us": round(us, 2),
                              "tflops": round(fl / us / 1e6, 1), "rel_err": float(f"{err:.2e}")}), flush=True)


if __name__ == "__main__":
    main()
