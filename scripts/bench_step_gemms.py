"""Time the GEMMs of the headline MLP step (784-4096-4096-10, batch 16384) under ldnn
kernel variants and hipBLASLt, one JSON line per shape.

    python scripts/bench_step_gemms.py [--batch 16384] [--only wgrad0,dgrad1]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def t(fn, it=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / it * 1e3)
    return round(best, 1)


def ws_q(M, N, sk):
    ne, nc = C.gemm_pp_ws(M, N, sk)
    return torch.empty(ne, device="cuda"), torch.zeros(nc, device="cuda", dtype=torch.int32)


def ws_128(M, N, sk):
    ne, nc = C.gemm_splitk_ws(M, N, sk)
    return torch.empty(ne, device="cuda"), torch.zeros(nc, device="cuda", dtype=torch.int32)


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--in-features", type=int, default=784)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    B, H, K0 = a.batch, a.hidden, a.in_features
    only = set(a.only.split(",")) if a.only else None
    x, h1, h2 = rnd(B, K0), rnd(B, H), rnd(B, H)
    dz1, dz2 = rnd(B, H), rnd(B, H)
    W0, W1 = rnd(H, K0), rnd(H, H)
    b = torch.zeros(H, device="cuda")
    out = torch.empty(B, H, device="cuda", dtype=torch.bfloat16)
    dW0, dW1 = torch.empty(H, K0, device="cuda"), torch.empty(H, H, device="cuda")
    db = torch.zeros(H, device="cuda")
    mask = torch.zeros(B, H // 8, dtype=torch.uint8, device="cuda")
    fl = lambda M, N, K: 2.0 * M * N * K  # noqa: E731

    def rec(name, flops, d):
        r = {"shape": name, "batch": B}
        for k, v in d.items():
            us = t(v)
            r[k + "_us"] = us
            r[k + "_tf"] = round(flops / us / 1e6, 1)
        print(json.dumps(r), flush=True)

    if not only or "fwd0" in only:
        rec("fwd0", fl(B, H, K0), {
            "auto": lambda: C.gemm(x, W0, out, True, True, C.EPI_BIAS_RELU, bias=b),
            "q": lambda: C.gemm(x, W0, out, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=32),
            "k128": lambda: C.gemm(x, W0, out, True, True, C.EPI_BIAS_RELU, bias=b, tile=128),
            "k256": lambda: C.gemm(x, W0, out, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=1),
            "q_mask": lambda: C.gemm(x, W0, out, True, True, C.EPI_BIAS_RELU, bias=b, mask_out=mask),
            "lib": lambda: torch._addmm_activation(b.bfloat16(), x, W0.t(), out=out)})
    if not only or "fwd1" in only:
        rec("fwd1", fl(B, H, H), {
            "q": lambda: C.gemm(h1, W1, out, True, True, C.EPI_BIAS_RELU, bias=b, tile=256, variant=32),
            "lib": lambda: torch._addmm_activation(b.bfloat16(), h1, W1.t(), out=out)})
    if not only or "dgrad1" in only:
        W1t = W1.t().contiguous()
        rec("dgrad1", fl(B, H, H), {
            "q_drelu": lambda: C.gemm(dz2, W1, out, True, False, C.EPI_DRELU, aux=h1, dbias=db, tile=256, variant=32),
            "q_none": lambda: C.gemm(dz2, W1, out, True, False, C.EPI_NONE, tile=256, variant=32),
            "q_drelu_nodb": lambda: C.gemm(dz2, W1, out, True, False, C.EPI_DRELU, aux=h1, tile=256, variant=32),
            "q_mask": lambda: C.gemm(dz2, W1, out, True, False, C.EPI_DRELU, dbias=db, mask_in=mask),
            "q_mask_nodb": lambda: C.gemm(dz2, W1, out, True, False, C.EPI_DRELU, mask_in=mask),
            "qT_drelu": lambda: C.gemm(dz2, W1t, out, True, True, C.EPI_DRELU, aux=h1, dbias=db, tile=256,
                                       variant=32),
            "qT_none": lambda: C.gemm(dz2, W1t, out, True, True, C.EPI_NONE, tile=256, variant=32),
            "lib": lambda: torch.mm(dz2, W1, out=out)})
    if not only or "wgrad1" in only:
        rec("wgrad1", fl(H, H, B), {
            "q": lambda: C.gemm(dz2, h1, dW1, False, False, tile=256, variant=32),
            "lib": lambda: torch.mm(dz2.t(), h1, out_dtype=torch.float32, out=dW1)})
        dz2t, h1t = dz2.t().contiguous(), h1.t().contiguous()
        rec("wgrad1_kc", fl(H, H, B), {
            "q": lambda: C.gemm(dz2t, h1t, dW1, True, True, tile=256, variant=32)})
    if not only or "wgrad0" in only:
        d = {}
        for sk in (1, 2, 4, 8):
            wq = ws_q(H, K0, sk)
            d[f"q_sk{sk}"] = (lambda sk=sk, wq=wq: C.gemm(dz1, x, dW0, False, False, tile=256, variant=32, splitk=sk,
                                                         ws=wq[0], cnt=wq[1]) if sk > 1 else
                              C.gemm(dz1, x, dW0, False, False, tile=256, variant=32))
        for sk in (2, 4):
            w8 = ws_128(H, K0, sk)
            d[f"k128_sk{sk}"] = (lambda sk=sk, w8=w8: C.gemm(dz1, x, dW0, False, False, tile=128, splitk=sk, ws=w8[0],
                                                            cnt=w8[1]))
            d[f"k128_atom{sk}"] = (lambda sk=sk: C.gemm(dz1, x, dW0, False, False, beta=1.0, tile=128, splitk=sk))
        d["k128_sk1"] = lambda: C.gemm(dz1, x, dW0, False, False, tile=128)
        d["lib"] = lambda: torch.mm(dz1.t(), x, out_dtype=torch.float32, out=dW0)
        rec("wgrad0", fl(H, K0, B), d)
        dz1t, xt = dz1.t().contiguous(), x.t().contiguous()
        d = {}
        for sk in (1, 4):
            wq = ws_q(H, K0, sk)
            d[f"q_sk{sk}"] = (lambda sk=sk, wq=wq: C.gemm(dz1t, xt, dW0, True, True, tile=256, variant=32, splitk=sk,
                                                         ws=wq[0], cnt=wq[1]) if sk > 1 else
                              C.gemm(dz1t, xt, dW0, True, True, tile=256, variant=32))
        rec("wgrad0_kc", fl(H, K0, B), d)


if __name__ == "__main__":
    main()
