"""A/B of the four-wave GEMM's forward epilogues (gemm_q.hip): bias+ReLU vs bias+ReLU
with the classifier head's partial logits (EPI_BIAS_RELU_HEAD), at the mlp3 forward
shape (K = 4096) and an epilogue-bound one (K = 64).  Prints one JSON line per shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


M, N = 16384, 4096
for K in (4096, 64):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    hw = torch.zeros(16, N, device="cuda", dtype=torch.bfloat16)
    hw[:10] = torch.randn(10, N, device="cuda").bfloat16()
    parts = torch.empty((N + 255) // 256, M, 16, device="cuda")
    dl = torch.empty(M, 16, device="cuda", dtype=torch.bfloat16)
    lg = torch.empty(M, 16, device="cuda", dtype=torch.bfloat16)
    st = torch.zeros((M + 15) // 16, 2, device="cuda")
    lab = torch.randint(0, 10, (M,), device="cuda")
    hb = torch.zeros(16, device="cuda")
    mask = torch.empty(M, N // 8, device="cuda", dtype=torch.uint8)
    fns = {
        "bias_relu": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=32),
        "bias_relu_mask": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, mask_out=mask),
        "bias_relu_head": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, head_w=hw, head_part=parts),
        "head_fwd_xent": lambda: C.head_fwd_xent(y, hw, hb, lab, lg, dl, st, 10, 1.0 / M),
        "head_xent_parts": lambda: C.head_xent_parts(parts, hb, lab, lg, dl, st, 10, 1.0 / M),
    }
    best = {k: 1e9 for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            best[k] = min(best[k], t(f))
    print(json.dumps({"M": M, "N": N, "K": K, **{k + "_us": round(v, 1) for k, v in best.items()}}), flush=True)
