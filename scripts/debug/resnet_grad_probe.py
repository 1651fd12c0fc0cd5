"""ResNet-18 one eager training step on a small input: per-parameter gradient norm next to an fp32
CPU reference's, and the cosine between them (localises a kernel path that drops a gradient).

    python scripts/debug/resnet_grad_probe.py --batch 16 --hw 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--model", default="resnet18")
    a = ap.parse_args()
    torch.manual_seed(0)
    m = build_model(a.model)
    xavier_init(m)
    ref = build_model(a.model)
    ref.load_state_dict(m.state_dict())
    ldnn.prepare(m, "cuda")
    x = torch.randn(a.batch, 3, a.hw, a.hw)
    y = torch.randint(0, 10, (a.batch,))
    crit = CrossEntropyLoss()
    crit(m(x.cuda()), y.cuda()).backward()
    torch.nn.functional.cross_entropy(ref(x), y).backward()
    torch.cuda.synchronize()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        g = p.grad.float().cpu().flatten() if p.grad is not None else torch.zeros(q.numel())
        h = q.grad.flatten()
        cos = torch.nn.functional.cosine_similarity(g.double(), h.double(), dim=0).item()
        print(json.dumps({"param": n, "norm": round(g.norm().item(), 6), "ref_norm": round(h.norm().item(), 6),
                          "cos": round(cos, 5), "env": {k: v for k, v in os.environ.items() if k.startswith("LDNN_")}}))


if __name__ == "__main__":
    main()
