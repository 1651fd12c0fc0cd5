"""Head backward at the headline shape (B 16384, K 4096, 10 classes): the fused MFMA
head_bwd vs head_dgrad_stream + head_wgrad (us per call).

    python scripts/bench_head_bwd.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
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
    C = _ext.C()
    B, K = 16384, 4096
    h = torch.relu(torch.randn(B, K, device="cuda")).bfloat16()
    W = torch.zeros(16, K, device="cuda", dtype=torch.bfloat16)
    W[:10] = (torch.randn(10, K, device="cuda") / 64).bfloat16()
    dl = torch.zeros(B, 16, device="cuda", dtype=torch.bfloat16)
    dl[:, :10] = (torch.randn(B, 10, device="cuda") / B).bfloat16()
    dh = torch.empty(B, K, device="cuda", dtype=torch.bfloat16)
    dbias, dW, db = torch.zeros(K, device="cuda"), torch.zeros(16, K, device="cuda"), torch.zeros(16, device="cuda")
    t_f = timeit(lambda: C.head_bwd(h, W, dl, dh, dW, dbias, C.EPI_DRELU, db))
    t_s = timeit(lambda: C.head_dgrad_stream(h, W, dl, dh, dbias, C.EPI_DRELU))
    t_w = timeit(lambda: C.head_wgrad(dl, h, dW, db, 4))
    t_c = timeit(lambda: dh.copy_(h))   # the same bytes moved by a plain copy (read h, write dh)
    print(json.dumps({"B": B, "K": K, "head_bwd_us": round(t_f, 2), "head_dgrad_stream_us": round(t_s, 2),
                      "head_wgrad_us": round(t_w, 2), "copy_us": round(t_c, 2), "gbps_fused": round(2 * B * K * 2 / t_f / 1e3, 1)}))


if __name__ == "__main__":
    main()
