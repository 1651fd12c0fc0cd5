"""First-layer GEMMs vs the input width: does padding K = 784 (MNIST) to a multiple
of 32/64/128 help hipBLASLt?  fwd = addmm+ReLU [B,K]x[K,4096], wgrad = [4096,B]x[B,K] fp32."""
import json

import torch


def bench(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


B, H = 16384, 4096
for K in (768, 784, 800, 832, 896):
    x = torch.randn(B, K, device="cuda").bfloat16()
    W = torch.randn(H, K, device="cuda").bfloat16()
    b = torch.randn(H, device="cuda").bfloat16()
    out = torch.empty(B, H, device="cuda", dtype=torch.bfloat16)
    dz = torch.randn(B, H, device="cuda").bfloat16()
    dW = torch.empty(H, K, device="cuda")
    f = bench(lambda: torch._addmm_activation(b, x, W.t(), out=out))
    w = bench(lambda: torch.mm(dz.t(), x, out_dtype=torch.float32, out=dW))
    print(json.dumps({"B": B, "K": K, "fwd_us": round(f, 2), "wgrad_us": round(w, 2),
                      "sum_us": round(f + w, 2)}), flush=True)
