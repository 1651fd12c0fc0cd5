"""How much of a four-wave GEMM is its epilogue?  bias+ReLU forward (variant 32) vs the
same kernel without an epilogue (XF bit 6, variant 96), with the epilogue but no global
stores (XF bit 7, variant 160) and with non-temporal stores, at the mlp3 forward shapes."""
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
for K in (4096, 784, 64):
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    mask = torch.randint(0, 256, (M, N // 8), device="cuda", dtype=torch.uint8)
    fns = {"epilogue": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=32),
           "no_epilogue": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=96),
           "epilogue_no_stores": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=160),
           "nontemporal_stores": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256,
                                                variant=32 | 4096),
           # variant bit 13: the fp32-staged row epilogue (epilogue_q) instead of the register-side one
           "fp32_staged_epilogue": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, tile=256,
                                                  variant=32 | 8192),
           "mask_out": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, mask_out=mask),
           "mask_out_fp32_staged": lambda: C.gemm(x, w, y, True, True, C.EPI_BIAS_RELU, bias=b, mask_out=mask,
                                                  variant=8192),
           "dgrad_mask_in": lambda: C.gemm(x, w, y, True, True, C.EPI_DRELU, mask_in=mask),
           "dgrad_mask_in_fp32_staged": lambda: C.gemm(x, w, y, True, True, C.EPI_DRELU, mask_in=mask,
                                                       variant=8192)}
    best = {k: 1e9 for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            best[k] = min(best[k], t(f))
    print(json.dumps({"M": M, "N": N, "K": K, **{k + "_us": round(v, 1) for k, v in best.items()}}), flush=True)
