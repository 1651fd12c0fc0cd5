"""Diagnostic: ldnn-GEMM engine vs hipBLASLt engine after one step (B = 4096,
1024-wide mlp3): relative differences of every backward tensor, and each
engine's dW against an fp32 torch reference on its OWN inputs."""
import sys

import torch

sys.path.insert(0, ".")
from ldnn.models.mlp import mlp3  # noqa: E402
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine  # noqa: E402

torch.manual_seed(0)
B = 4096
m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
m2.load_state_dict(m1.state_dict())
cfg = OptimConfig("sgd", lr=0.05, momentum=0.0)
e1 = StaticMLPEngine(m1, B, cfg, use_graphs=False, library_gemms=False)
e2 = StaticMLPEngine(m2, B, cfg, use_graphs=False, library_gemms=True)
print("splitk", e1._wgrad_splitk, [None if w is None else w[2] for w in e1._wgrad_ws])
g = torch.Generator(device="cuda").manual_seed(11)
x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
y = torch.randint(0, 10, (B,), device="cuda", generator=g)
for e in (e1, e2):
    e.load_batch(x, y)
    e.step()
torch.cuda.synchronize()


def rel(a, b):
    return f"{((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item():.2e}"


for l in (1, 2):
    print(f"h[{l}]", rel(e1.h[l], e2.h[l]))
for l in (3, 2, 1):
    print(f"dz[{l}]", rel(e1.dz[l], e2.dz[l]))
for l in (2, 1, 0):
    print(f"dW[{l}]", rel(e1.dW[l], e2.dW[l]))
    for name, e in (("ldnn", e1), ("lib", e2)):
        ref = e.dz[l + 1].float().t() @ e.h[l].float()
        print(f"   {name} vs fp32 on own inputs", rel(e.dW[l][:, : ref.shape[1]], ref))
for name, e in (("ldnn", e1), ("lib", e2)):
    C = e.num_classes
    ref = (e.dz[3].float()[:, :C] @ e.W[2].float()[:C]) * (e.h[2].float() > 0)
    print(name, "dz[2] vs fp32 on own inputs", rel(e.dz[2], ref), "head_dgrad", e.head_dgrad,
          "W2 diff", rel(e1.W[2], e2.W[2]))
    ref1 = (e.dz[2].float() @ e.W[1].float()) * (e.h[1].float() > 0)
    print(name, "dz[1] vs fp32 on own inputs", rel(e.dz[1], ref1))
