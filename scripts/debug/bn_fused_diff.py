"""Per-parameter gradient difference: conv-epilogue BN statistics (m1) vs the BN's own
reduce (m2, m3) on resnet18 (8,3,96,96) -- debugging aid for the fused-stats path."""
import sys

import torch

sys.path.insert(0, ".")
import ldnn  # noqa: E402
import ldnn.models.layers as layers_mod  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402
from ldnn.models.layers import Conv2d  # noqa: E402

layers_mod.FUSE_BN_STATS = True
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1
torch.manual_seed(0)
m1, m2, m3 = build_model("resnet18"), build_model("resnet18"), build_model("resnet18")
xavier_init(m1)
for mm in (m2, m3):
    mm.load_state_dict(m1.state_dict())
    for m in mm.modules():
        if isinstance(m, Conv2d):
            m.__dict__["_ldnn_stats_bn"] = None
for mm in (m1, m2, m3):
    ldnn.prepare(mm, "cuda")
x = torch.randn(8, 3, 96, 96, device="cuda").bfloat16()
y = torch.randint(0, 10, (8,), device="cuda")
crit = CrossEntropyLoss()
for m in (m1, m2, m3):
    m.train()
    for _ in range(iters):
        crit(m(x), y).backward()
torch.cuda.synchronize()
fused = {n for n, m in m1.named_modules() if isinstance(m, Conv2d) and m._ldnn_stats_bn is not None}
print("fused convs:", sorted(fused))
for (n, p1), (_, p2), (_, p3) in zip(m1.named_parameters(), m2.named_parameters(), m3.named_parameters()):
    g1, g2, g3 = (p.grad.flatten().double() for p in (p1, p2, p3))
    d12 = ((g1 - g2).norm() / g2.norm()).item()
    d32 = ((g3 - g2).norm() / g2.norm()).item()
    print(f"{n:40s} {d12:9.2e} {d32:9.2e} {'BAD' if d12 > 0.02 else ''}", flush=True)
