"""Weight-gradient GEMM options at the bench's batch (dW = dz^T h, fp32 out):
hipBLASLt plain mm, hipBLASLt batched split-K (bmm over batch slices + slice sum),
and ldnn's 128-tile in-launch split-K combine.  One JSON line per (shape, variant)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    C = _ext.C()
    B = int(os.environ.get("B", 16384))
    for M, N in ((4096, 784), (4096, 4096)):
        dz = torch.randn(B, M, device="cuda").bfloat16()
        h = torch.randn(B, N, device="cuda").bfloat16()
        ref = dz.float().t() @ h.float()
        dW = torch.empty(M, N, device="cuda")
        fl = 2.0 * B * M * N
        res = {}
        res["mm"] = bench(lambda: torch.mm(dz.t(), h, out_dtype=torch.float32, out=dW))
        err = (dW - ref).abs().max().item()
        dWt = torch.empty(N, M, device="cuda")

        def ft():
            torch.mm(h.t(), dz, out_dtype=torch.float32, out=dWt)
            dW.copy_(dWt.t())
        res["mmT_transpose"] = bench(ft)
        ft()
        assert (dW - ref).abs().max().item() <= 2 * err + 1e-3
        for s in (4,):
            ws = torch.empty(s, M, N, device="cuda")
            a, b = dz.view(s, B // s, M).transpose(1, 2), h.view(s, B // s, N)

            def f(a=a, b=b, ws=ws):
                torch.bmm(a, b, out_dtype=torch.float32, out=ws)
                torch.sum(ws, 0, out=dW)
            res[f"bmm_split{s}"] = bench(f)
        for sk in (4,):
            ne, nc = C.gemm_splitk_ws(M, N, sk)
            wsp = torch.empty(ne, dtype=torch.float32, device="cuda")
            cnt = torch.zeros(nc, dtype=torch.int32, device="cuda")
            res[f"ldnn128_sk{sk}"] = bench(lambda: C.gemm(dz, h, dW, False, False, tile=128, splitk=sk, ws=wsp, cnt=cnt))
        res["ldnn_default"] = bench(lambda: C.gemm(dz, h, dW, False, False))
        for k, us in res.items():
            print(json.dumps({"B": B, "M": M, "N": N, "variant": k, "us": round(us, 2),
                              "tflops": round(fl / us / 1e6, 1), "mm_maxerr": err}), flush=True)


if __name__ == "__main__":
    main()
