"""MLP wgrad shapes through the conv LDS-DMA wgrad kernel (1x1 conv over a 1x1 image)
vs the GEMM path.  python scripts/bench_wgrad_conv.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402
from scripts.bench_wgrad import timeit  # noqa: E402


def main():
    C = _ext._C
    B = 4096
    for (M, N) in [(4096, 784), (4096, 4096)]:
        dz = torch.randn(B, M, device="cuda").bfloat16()
        h = torch.randn(B, N, device="cuda").bfloat16()
        ref = dz.float().t() @ h.float()
        dW = torch.empty(M, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * B
        us = timeit(lambda: C.conv_wgrad(dz.view(B, 1, 1, M), h.view(B, 1, 1, N), dW.view(M, 1, 1, N), 1, 0))
        err = ((dW - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"path": "conv_wgrad", "M": M, "N": N, "us": round(us, 2), "tflops": round(fl / us / 1e6, 1),
                          "rel_err": float(f"{err:.2e}")}), flush=True)
        us = timeit(lambda: C.gemm(dz, h, dW, False, False))
        print(json.dumps({"path": "gemm", "M": M, "N": N, "us": round(us, 2), "tflops": round(fl / us / 1e6, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
