"""GEMM micro-benchmark: ldnn MFMA kernel vs torch.matmul (hipBLASLt) on the
MLP shapes, random bf16 operands, interleaved rounds in one process."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters


def main():
    shapes = [
        ("fwd L2", 4096, 4096, 4096, True, True),
        ("dgrad L2", 4096, 4096, 4096, True, False),
        ("wgrad L2", 4096, 4096, 4096, False, False),
        ("fwd L1", 4096, 4096, 784, True, True),
        ("wgrad L1", 4096, 784, 4096, False, False),
        ("sq8k", 8192, 8192, 8192, True, True),
    ]
    out = []
    for name, M, N, K, akc, bkc in shapes:
        a = (torch.rand(M, K, device="cuda") * 2 - 1 if akc else torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device="cuda") * 2 - 1 if bkc else torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16 if akc else torch.float32)
        A = a if akc else a.t()
        B = b.t() if bkc else b
        fl = 2.0 * M * N * K
        row = dict(shape=name, M=M, N=N, K=K, auto_tile=C.gemm.__doc__ and None)
        for tile in (128, 256):
            t = min(timeit(lambda: C.gemm(a, b, c, akc, bkc, tile=tile)) for _ in range(3))
            row[f"t{tile}_tflops"] = round(fl / t / 1e9, 1)
        for v in (1, 2, 3):
            t = min(timeit(lambda: C.gemm(a, b, c, akc, bkc, tile=256, variant=v)) for _ in range(3))
            row[f"t256_v{v}_tflops"] = round(fl / t / 1e9, 1)
        t_ref = min(timeit(lambda: torch.matmul(A, B)) for _ in range(3))
        row["torch_tflops"] = round(fl / t_ref / 1e9, 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


if __name__ == "__main__":
    main()
