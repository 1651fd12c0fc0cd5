"""MLP-step GEMMs at the headline shapes (mlp3 784-4096-4096-10, batch 16384):
ldnn ping-pong kernel (variant 4) vs ldnn 2-stage k256 (variant 0) vs hipBLASLt
(torch), random bf16 operands, interleaved rounds in one process, each checked
against an fp32 torch reference first.  One JSON line per shape.

usage: python scripts/bench_gemm_pp.py [--batch 16384] [--rounds 5] [--only fwd1,...]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

C = _ext.C()


def timeit(fn, iters=10):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(iters):
        fn()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / iters * 1e3  # us


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).bfloat16()


def cases(B):
    out = []
    for K0, name in ((4096, "1"), (784, "0")):
        h = rnd(B, K0)
        W = rnd(4096, K0) * (1.0 / K0 ** 0.5)
        W = W.bfloat16()
        bias = torch.rand(4096, device="cuda") * 0.1
        y = torch.empty(B, 4096, device="cuda", dtype=torch.bfloat16)
        ref = lambda h=h, W=W, bias=bias: torch.relu(h.float() @ W.float().t() + bias)  # noqa: E731
        bb = bias.bfloat16()
        lib = lambda h=h, W=W, bb=bb, y=y: torch._addmm_activation(bb, h, W.t(), out=y)  # noqa: E731
        mk = lambda v, h=h, W=W, bias=bias, y=y: (lambda: C.gemm(h, W, y, True, True, C.EPI_BIAS_RELU, bias=bias,  # noqa: E731
                                                                  tile=256, variant=v))
        out.append((f"fwd{name}", 2.0 * B * 4096 * K0, y, ref, lib, mk))
    # dgrad L1: dz1 = (dz2 @ W1) * relu'(h1), dbias0 += colsum
    dz2 = rnd(B, 4096) * 0.01
    dz2 = dz2.bfloat16()
    W1 = rnd(4096, 4096) * (1.0 / 64)
    W1 = W1.bfloat16()
    h1 = torch.relu(rnd(B, 4096))
    dz1 = torch.empty(B, 4096, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(4096, device="cuda")
    ref = lambda: (dz2.float() @ W1.float()) * (h1.float() > 0)  # noqa: E731
    lib = lambda: torch.mm(dz2, W1, out=dz1)  # noqa: E731
    mk = lambda v: (lambda: C.gemm(dz2, W1, dz1, True, False, C.EPI_DRELU, aux=h1, dbias=db, tile=256,  # noqa: E731
                                   variant=v))
    out.append(("dgrad1", 2.0 * B * 4096 * 4096, dz1, ref, lib, mk))
    ref_n = lambda: dz2.float() @ W1.float()  # noqa: E731
    mk_n = lambda v: (lambda: C.gemm(dz2, W1, dz1, True, False, tile=256, variant=v))  # noqa: E731
    out.append(("dgrad1n", 2.0 * B * 4096 * 4096, dz1, ref_n, lib, mk_n))
    # wgrads (fp32 out): dW = dz^T h
    import os
    for K0, name, sk in ((4096, "1", 1), (784, "0", int(os.environ.get("WG0_SPLITK", "4")))):
        dz = rnd(B, 4096) * 0.01
        dz = dz.bfloat16()
        h = rnd(B, K0)
        dW = torch.empty(4096, K0, device="cuda")
        ref = lambda dz=dz, h=h: dz.float().t() @ h.float()  # noqa: E731
        lib = lambda dz=dz, h=h, dW=dW: torch.mm(dz.t(), h, out_dtype=torch.float32, out=dW)  # noqa: E731
        ws = cnt = None
        if sk > 1:
            ne, nc = C.gemm_pp_ws(4096, K0, sk)
            ws = torch.empty(ne, device="cuda")
            cnt = torch.zeros(nc, device="cuda", dtype=torch.int32)

        def mk(v, dz=dz, h=h, dW=dW, sk=sk, ws=ws, cnt=cnt):
            if v in (4, 32) and sk > 1:
                return lambda: C.gemm(dz, h, dW, False, False, tile=256, variant=v, splitk=sk, ws=ws, cnt=cnt)
            return lambda: C.gemm(dz, h, dW, False, False, tile=256, variant=v)
        out.append((f"wgrad{name}", 2.0 * B * 4096 * K0, dW, ref, lib, mk))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="4,0")
    a = ap.parse_args()
    variants = [int(v) for v in a.variants.split(",")]
    for name, flops, out, ref, lib, mk in cases(a.batch):
        if a.only and name not in a.only.split(","):
            continue
        r = ref()
        row = {"shape": name, "batch": a.batch}
        fns = {"lib": lib}
        for v in variants:
            fns[f"v{v}"] = mk(v)
        for k, fn in fns.items():
            fn()
            torch.cuda.synchronize()
            err = ((out.float() - r).abs().max() / r.abs().max().clamp_min(1e-6)).item()
            row[f"{k}_err"] = float(f"{err:.2e}")
        for fn in fns.values():
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        best = {k: 1e30 for k in fns}
        for _ in range(a.rounds):
            for k, fn in fns.items():
                best[k] = min(best[k], timeit(fn))
        for k in fns:
            row[f"{k}_us"] = round(best[k], 1)
            row[f"{k}_tf"] = round(flops / best[k] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
