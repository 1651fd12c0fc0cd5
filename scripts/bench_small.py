"""Per-kernel timings of the small / odd-shaped launches in one mlp3 training step."""
import sys
import torch
sys.path.insert(0, ".")
import ldnn  # noqa
from ldnn.ops import _ext
C = _ext.C()


def t(fn, it=50):
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


B, D0, H, NC = 4096, 784, 4096, 16
dev, bf = "cuda", torch.bfloat16
x = torch.randn(B, D0, device=dev).to(bf)
h2 = torch.randn(B, H, device=dev).to(bf)
dz1 = torch.randn(B, H, device=dev).to(bf)
dz3 = torch.randn(B, NC, device=dev).to(bf)
W3 = torch.randn(NC, H, device=dev).to(bf)
dW1 = torch.empty(H, D0, device=dev)
dW3 = torch.empty(NC, H, device=dev)
out = torch.empty(B, H, device=dev, dtype=bf)
h3 = torch.empty(B, NC, device=dev, dtype=bf)
db = torch.zeros(H, device=dev)
db3 = torch.zeros(NC, device=dev)
labels = torch.randint(0, 10, (B,), device=dev)
stats = torch.zeros(2, device=dev)
bias3 = torch.zeros(NC, device=dev)
res = {}
for sk in (1, 2, 3, 4):
    res[f"wgrad_L1_t128_sk{sk}"] = t(lambda: C.gemm(dz1, x, dW1, False, False, tile=128, splitk=sk))
res["wgrad_L1_t256"] = t(lambda: C.gemm(dz1, x, dW1, False, False, tile=256))
res["wgrad_L3_auto"] = t(lambda: C.gemm(dz3, h2, dW3, False, False))
for sk in (1, 4, 8, 16, 32):
    res[f"wgrad_L3_sk{sk}"] = t(lambda: C.gemm(dz3, h2, dW3, False, False, tile=128, splitk=sk))
for tile in (128, 256):
    res[f"dgrad_L3_t{tile}"] = t(lambda: C.gemm(dz3, W3, out, True, False, C.EPI_DRELU, aux=h2, dbias=db, tile=tile))
    res[f"dgrad_L3_t{tile}_nodb"] = t(lambda: C.gemm(dz3, W3, out, True, False, C.EPI_DRELU, aux=h2, tile=tile))
res["fwd_L3_skinny"] = t(lambda: C.gemm(h2, W3, h3, True, True, C.EPI_BIAS, bias=bias3))
res["fwd_L3_t128"] = t(lambda: C.gemm(h2, W3, h3, True, True, C.EPI_BIAS, bias=bias3, tile=128))
lg = torch.randn(B, NC, device=dev).to(bf)
dl = torch.empty_like(lg)
res["xent"] = t(lambda: C.softmax_xent(lg[:, :10], labels, dl[:, :10], stats, dbias=db3, num_classes=10,
                                       grad_scale=1.0 / B))
res["xent_nodb"] = t(lambda: C.softmax_xent(lg[:, :10], labels, dl[:, :10], stats, num_classes=10,
                                            grad_scale=1.0 / B))
res["fill_small"] = t(lambda: db.zero_())
for k, v in res.items():
    print(f"{k:28s} {v:8.1f} us")
hstats = torch.zeros(B // 16, 2, device=dev)
res2 = {}
res2["head_fwd_xent"] = t(lambda: C.head_fwd_xent(h2, W3, bias3, labels, h3, dz3, hstats, 10, 1.0 / B))
dW3z = torch.zeros(NC, H, device=dev)
for sp in (1, 4, 8, 16):
    res2[f"head_wgrad_s{sp}"] = t(lambda: C.head_wgrad(dz3, h2, dW3z, db3, sp))
for k, v in res2.items():
    print(f"{k:28s} {v:8.1f} us")
