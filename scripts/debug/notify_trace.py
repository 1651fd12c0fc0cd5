"""Print every FlatParams readiness notification of one native backward (debug)."""
import traceback

import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

import ldnn
from ldnn.models import CrossEntropyLoss, build_model

m = build_model("enhanced_cnn_small")
ldnn.prepare(m, "cuda")
flat = m.fc._ldnn_flat
names = {id(s.param): s.name for s in flat.segments}
seen = {}


def hook(params):
    for p in params:
        n = names[id(p)]
        seen[n] = seen.get(n, 0) + 1
        if seen[n] > 1 or n.startswith("fc"):
            print("notify", n, seen[n], "group", [names[id(q)] for q in params])
            traceback.print_stack(limit=6)


flat.add_ready_group_hook(hook)
x = torch.randn(32, 3, 32, 32, device="cuda").bfloat16()
y = torch.randint(0, 10, (32,), device="cuda")
CrossEntropyLoss()(m(x), y).backward()
torch.cuda.synchronize()
print("counts", sorted(set(seen.values())), len(seen), len(flat.segments))
