"""The MLP first layer's weight gradient, dW0 [4096][784] (+ the ones-column bias gradient)
= dz1^T [4096 x 16384] . x [16384 x 792], both operands k-strided: today one gemm_q
split-K launch over 4 column tiles of 256 (792 of 1024 columns real) + slab_sum_cols.
Candidates: the 3 full column tiles (768) on gemm_q split-K, and the 24-column tail
(16 features + the ones column + pad) on the 128-tile kernel with the in-launch
combine.  Prints one JSON line per variant (median us of 20 launches).

    python scripts/bench_wgrad0.py
"""
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
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    B, M, N, Np = 16384, 4096, 784, 832
    dz = (torch.randn(B, M, device="cuda") * 0.1).bfloat16()
    xp = torch.zeros(B, Np, device="cuda", dtype=torch.bfloat16)
    xp[:, :N] = torch.randn(B, N, device="cuda").bfloat16()
    xp[:, N] = 1.0
    dW = torch.empty(M, N, device="cuda")
    db = torch.empty(M, device="cuda")
    out = []
    for sk in (4,):
        slab = torch.empty(sk, M, 792, device="cuda")
        g = lambda: C.gemm(dz, xp[:, :792], slab, False, False, tile=256, splitk=sk)  # noqa: E731
        s = lambda: C.slab_sum_cols(slab, dW, db)  # noqa: E731
        out.append({"variant": f"current 792 cols sk{sk}", "gemm_us": timeit(g), "sum_us": timeit(s)})
    for sk in (4, 5, 6, 8):
        slab = torch.empty(sk, M, 768, device="cuda")
        g = lambda: C.gemm(dz, xp[:, :768], slab, False, False, tile=256, splitk=sk)  # noqa: E731
        out.append({"variant": f"main 768 cols sk{sk}", "gemm_us": timeit(g)})
    tail = torch.empty(M, 24, device="cuda")
    for sk in (8, 16, 32):
        ne, nc = C.gemm_splitk_ws(M, 24, sk)
        ws = torch.empty(ne, device="cuda")
        cnt = torch.zeros(nc, dtype=torch.int32, device="cuda")
        g = lambda: C.gemm(dz, xp[:, 768:792], tail, False, False, tile=128, splitk=sk, ws=ws, cnt=cnt)  # noqa: E731
        out.append({"variant": f"tail 24 cols k128 combine sk{sk}", "gemm_us": timeit(g)})
        ref = dz.float().t() @ xp[:, 768:792].float()
        out[-1]["rel_err"] = float(((tail - ref).norm() / ref.norm()).item())
    for r in out:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
