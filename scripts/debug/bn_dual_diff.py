"""Debug: fused vs separate relu(bn_a(x) + bn_b(r)) -- which outputs differ."""
import torch

import ldnn
from ldnn.models.layers import BatchNorm2d
from ldnn.ops import functional as LF

N, C, H, W = 8, 64, 16, 16
torch.manual_seed(11)
x = torch.randn(N, C, H, W, device="cuda") * 1.5 + 0.2
r = torch.randn(N, C, H, W, device="cuda") * 0.7 - 0.1
g1 = torch.randn(N, C, H, W, device="cuda").bfloat16().float()
res = []
for fused in (True, False, True):
    LF.BN_DUAL_FUSED = fused
    torch.manual_seed(5)
    ba, bb = BatchNorm2d(C), BatchNorm2d(C)
    with torch.no_grad():
        for b in (ba, bb):
            b.weight.uniform_(-1.0, 1.5)
            b.bias.uniform_(-0.5, 0.5)
    holder = torch.nn.ModuleList([ba, bb])
    ldnn.prepare(holder, "cuda")
    xb = x.bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    rb = r.bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = LF.batch_norm_dual_act(xb, ba, rb, bb)
    (y.float() * g1).sum().backward()
    torch.cuda.synchronize()
    res.append([y.detach().float(), xb.grad.float(), rb.grad.float()] + [p.grad.clone() for p in (ba.weight, ba.bias, bb.weight, bb.bias)])
names = ["y", "dx", "dr", "dgamma_a", "dbeta_a", "dgamma_b", "dbeta_b"]
for n, a, b, c in zip(names, *res):
    d = (a - b).abs()
    d2 = (a - c).abs()
    bad = (d > 1e-2 * b.abs().max()).nonzero()
    print(n, "fused-vs-sep max", d.max().item(), "fused-vs-fused max", d2.max().item(), "n bad", bad.shape[0], bad[:8].flatten().tolist() if bad.numel() else "")
    if n.startswith("d") and a.dim() == 1:
        print("   fused", a[:8].tolist())
        print("   sep  ", b[:8].tolist())
