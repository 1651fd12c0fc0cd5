"""Library GEMM (hipBLASLt via torch) vs ldnn kernels on the MLP's plain GEMMs:
fp32-output wgrads (torch.mm out_dtype) and the fused bias+ReLU forward
(torch._addmm_activation).  python scripts/bench_blaslt.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402
from scripts.bench_wgrad import timeit  # noqa: E402


def rec(**k):
    print(json.dumps(k), flush=True)


def main():
    C = _ext._C
    B = 4096
    for (M, N) in [(4096, 784), (4096, 4096)]:
        dz = torch.randn(B, M, device="cuda").bfloat16()
        h = torch.randn(B, N, device="cuda").bfloat16()
        dW = torch.empty(M, N, device="cuda", dtype=torch.float32)
        fl = 2.0 * M * N * B
        ref = dz.float().t() @ h.float()
        try:
            f = lambda: torch.mm(dz.t(), h, out_dtype=torch.float32, out=dW)  # noqa: E731
            f()
            torch.cuda.synchronize()
            err = ((dW - ref).abs().max() / ref.abs().max()).item()
            us = timeit(f)
            rec(op="wgrad", path="torch.mm out_dtype f32 (out=)", M=M, N=N, us=round(us, 2),
                tflops=round(fl / us / 1e6, 1), rel_err=float(f"{err:.2e}"))
        except Exception as ex:  # noqa: BLE001
            rec(op="wgrad", path="torch.mm out_dtype", error=str(ex)[:200])
        try:
            f = lambda: torch.mm(dz.t(), h, out_dtype=torch.float32)  # noqa: E731
            us = timeit(f)
            rec(op="wgrad", path="torch.mm out_dtype f32", M=M, N=N, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
        except Exception as ex:  # noqa: BLE001
            rec(op="wgrad", path="torch.mm out_dtype (no out)", error=str(ex)[:200])
        us = timeit(lambda: torch.mm(dz.t(), h))
        rec(op="wgrad", path="torch.mm bf16 out", M=M, N=N, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
        us = timeit(lambda: C.gemm(dz, h, dW, False, False))
        rec(op="wgrad", path="ldnn", M=M, N=N, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
    # forward Linear + bias + ReLU
    for (K, N) in [(784, 4096), (4096, 4096)]:
        x = torch.randn(B, K, device="cuda").bfloat16()
        W = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        b = torch.randn(N, device="cuda").bfloat16()
        bf = b.float()
        y = torch.empty(B, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * B * N * K
        try:
            us = timeit(lambda: torch._addmm_activation(b, x, W.t(), use_gelu=False))
            rec(op="fwd", path="torch._addmm_activation relu", K=K, N=N, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
        except Exception as ex:  # noqa: BLE001
            rec(op="fwd", path="_addmm_activation", error=str(ex)[:200])
        us = timeit(lambda: C.gemm(x, W, y, True, True, C.EPI_BIAS_RELU, bias=bf))
        rec(op="fwd", path="ldnn", K=K, N=N, us=round(us, 2), tflops=round(fl / us / 1e6, 1))
    # dgrad: dX = dY W (bf16 out, no epilogue) for reference
    dY = torch.randn(B, 4096, device="cuda").bfloat16()
    W = (torch.randn(4096, 4096, device="cuda") * 0.02).bfloat16()
    fl = 2.0 * B * 4096 * 4096
    us = timeit(lambda: torch.mm(dY, W))
    rec(op="dgrad", path="torch.mm", us=round(us, 2), tflops=round(fl / us / 1e6, 1))


if __name__ == "__main__":
    main()
