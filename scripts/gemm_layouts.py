"""hipBLASLt time of C[M,N] = A[M,K] B[K,N] for the four operand storage layouts
(A k-contiguous or m-contiguous, B k-contiguous or n-contiguous), bf16 in, fp32/bf16 out.
Used to decide which layout each MLP GEMM should be fed in (profiles/gemm_layouts_r1.jsonl)."""
import json
import sys

import torch


def bench(fn, it=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / it


def main():
    out = []
    for M, N, K in [(4096, 784, 4096), (4096, 4096, 4096), (784, 4096, 4096)]:
        for a_k in (True, False):
            for b_k in (True, False):
                A = torch.randn(M, K, device="cuda").bfloat16() if a_k else torch.randn(K, M, device="cuda").bfloat16()
                B = torch.randn(N, K, device="cuda").bfloat16() if b_k else torch.randn(K, N, device="cuda").bfloat16()
                a = A if a_k else A.t()
                b = B.t() if b_k else B
                for od in (torch.float32, torch.bfloat16):
                    C = torch.empty(M, N, device="cuda", dtype=od)
                    if od == torch.float32:
                        f = lambda: torch.mm(a, b, out_dtype=torch.float32, out=C)  # noqa: E731
                    else:
                        f = lambda: torch.mm(a, b, out=C)  # noqa: E731
                    us = bench(f)
                    r = {"M": M, "N": N, "K": K, "A": "k-contig" if a_k else "m-contig",
                         "B": "k-contig" if b_k else "n-contig", "out": str(od).split(".")[-1], "us": round(us, 2),
                         "tflops": round(2 * M * N * K / us / 1e6, 1)}
                    out.append(r)
                    print(json.dumps(r), flush=True)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as fh:
            for r in out:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
