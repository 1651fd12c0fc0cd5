"""The MLP's first-layer forward (16384 x 784 @ 784 x 4096, bias + ReLU, bf16 out) on each GEMM
kernel ldnn has, one JSON line each: the four-wave 256x256 gemm_q (with and without the ReLU
bit-mask output the engine uses), the 8-wave 256x256 k256 and the 2-workgroups-per-CU 128x128
kernel.  Question behind it: does a kernel whose workgroups overlap one tile's epilogue with
another's K loop beat the one-workgroup-per-CU 256^2 tile at K = 784?

    python scripts/gemm_fwd0_micro.py
"""
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
    C_ = _ext._C
    assert C_ is not None, "ldnn extension not loaded"
    M, N, K = 16384, 4096, 784
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.05).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    ref = torch.relu(x.float() @ w.float().t() + b)
    mask = torch.empty(M, N // 8, device="cuda", dtype=torch.uint8)
    rows = []
    cases = [("gemm_q 256x256 4-wave, bias+relu", dict(tile=256, variant=32), 2, None),
             ("gemm_q 256x256 4-wave, bias+relu+mask (engine)", dict(tile=256, variant=32), 2, mask),
             ("k256 256x256 8-wave, bias+relu", dict(tile=256, variant=1), 2, None),
             ("k128 128x128 4-wave x2/CU, bias+relu", dict(tile=128), 2, None)]
    for rep in range(2):
        for name, kw, epi, mo in cases:
            y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

            def run():
                C_.gemm(x, w, y, True, True, epi=epi, bias=b, mask_out=mo, **kw)
            t = timeit(run)
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            rows.append({"rep": rep, "kernel": name, "us": round(t, 2),
                         "tflops": round(2.0 * M * N * K / t / 1e6, 1), "rel_err": round(err, 5)})
            print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
