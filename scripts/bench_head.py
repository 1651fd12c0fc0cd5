"""Microbenchmark of the fused MLP head backward (head.hip head_bwd) at the headline shape
(h = 16384 x 4096 bf16, 10 classes), against a plain device copy of the same bytes (read h,
write dh: the HBM roof of this kernel).  One JSON line; the grid knob LDNN_HEAD_BWD_WGS is read
once per process, so sweep it from the shell.

    LDNN_HEAD_BWD_WGS=1024 python scripts/bench_head.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldnn.ops import _ext  # noqa: E402


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    B, K, ncls = 16384, 4096, 10
    C = _ext.C()
    h = torch.relu(torch.randn(B, K, device="cuda")).bfloat16()
    W = torch.zeros(16, K, device="cuda", dtype=torch.bfloat16)
    W[:ncls] = (torch.randn(ncls, K, device="cuda") / K ** 0.5).bfloat16()
    dl = torch.zeros(B, 16, device="cuda", dtype=torch.bfloat16)
    dl[:, :ncls] = (torch.randn(B, ncls, device="cuda") / B).bfloat16()
    dh = torch.empty_like(h)
    dbias, dW, db = torch.zeros(K, device="cuda"), torch.zeros(16, K, device="cuda"), torch.zeros(16, device="cuda")
    t_head = timeit(lambda: C.head_bwd(h, W, dl, dh, dW, dbias, C.EPI_DRELU, db))
    t_copy = timeit(lambda: dh.copy_(h))
    gb = 2 * h.numel() * 2 / 1e9
    print(json.dumps({"wgs": os.environ.get("LDNN_HEAD_BWD_WGS", "default"), "head_bwd_us": round(t_head, 1),
                      "copy_us": round(t_copy, 1), "head_TBps": round(gb * 1e3 / t_head, 2),
                      "copy_TBps": round(gb * 1e3 / t_copy, 2)}), flush=True)


if __name__ == "__main__":
    main()
