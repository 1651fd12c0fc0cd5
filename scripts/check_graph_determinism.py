"""Diagnose graph-vs-eager differences: runs two eager copies and a graphed copy of
the same model on the same batches and prints per-parameter max |diff| per step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import ldnn
from ldnn.models import CrossEntropyLoss, build_model, xavier_init
from ldnn.optim import SGD
from ldnn.train.graphed import GraphedStep

name = sys.argv[1] if len(sys.argv) > 1 else "enhanced_cnn_small"
shape = (32, 3, 32, 32) if name != "lenet5" else (256, 1, 28, 28)
torch.manual_seed(0)
ms = [build_model(name) for _ in range(3)]
xavier_init(ms[0])
for m in ms[1:]:
    m.load_state_dict(ms[0].state_dict())
for m in ms:
    ldnn.prepare(m, "cuda")
os_ = [SGD(m.parameters(), lr=0.05, momentum=0.9) for m in ms]
crit = CrossEntropyLoss()
g = torch.Generator(device="cuda").manual_seed(1)
xs = [torch.randn(*shape, device="cuda", generator=g).bfloat16() for _ in range(5)]
ys = [torch.randint(0, 10, (shape[0],), device="cuda", generator=g) for _ in range(5)]
for m, o in zip(ms, os_):
    o.zero_grad(); crit(m(xs[0]), ys[0]).backward(); o.step()
def diff(a, b):
    return max((p.detach().float() - q.detach().float()).abs().max().item() for p, q in zip(a.parameters(), b.parameters()))
print("after eager step0: e0-e1", diff(ms[0], ms[1]), "e0-e2", diff(ms[0], ms[2]))
gs = GraphedStep(ms[2], crit, os_[2], xs[1], ys[1], warmup=0)
for i in range(1, 5):
    for m, o in zip(ms[:2], os_[:2]):
        o.zero_grad(); crit(m(xs[i]), ys[i]).backward(); o.step()
    gs(xs[i], ys[i])
    torch.cuda.synchronize()
    print(f"step {i}: eager-eager {diff(ms[0], ms[1]):.3e} eager-graph {diff(ms[0], ms[2]):.3e}")
    for (n, p), (_, q), (_, r) in zip(ms[0].named_parameters(), ms[1].named_parameters(), ms[2].named_parameters()):
        d01 = (p - q).abs().max().item(); d02 = (p - r).abs().max().item()
        if d02 > 0 or d01 > 0:
            print(f"   {n:30s} ee {d01:.3e} eg {d02:.3e}")
