"""Graph-replayed training steps (train.graphed.GraphedStep) vs the same steps run eagerly, twice:
per parameter the cosine between the graphed and an eager run's updates next to the cosine between
the two eager runs' updates (the arrival-order noise floor); one JSON line per parameter whose graphed
cosine falls below the eager one by more than 0.1.

    python scripts/debug/graphed_vs_eager_probe.py --model resnet18 --batch 16 --hw 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402
from ldnn.optim import SGD  # noqa: E402
from ldnn.train.graphed import STAGE_S2D, GraphedStep  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--lr-drop-at", type=int, default=3, help="lr x 0.1 from this step on (0: never), as the test")
    a = ap.parse_args()
    torch.manual_seed(0)
    ms = [build_model(a.model) for _ in range(3)]
    xavier_init(ms[0])
    for m in ms[1:]:
        m.load_state_dict(ms[0].state_dict())
    for m in ms:
        ldnn.prepare(m, "cuda")
    os_ = [SGD(m.parameters(), lr=0.05, momentum=0.9) for m in ms]
    crit = CrossEntropyLoss()
    g = torch.Generator(device="cuda").manual_seed(1)
    shape = (a.batch, 3, a.hw, a.hw)
    xs = [torch.randn(*shape, device="cuda", generator=g).bfloat16() for _ in range(a.steps + 1)]
    ys = [torch.randint(0, 10, (a.batch,), device="cuda", generator=g) for _ in range(a.steps + 1)]
    for m, o in zip(ms, os_):
        o.zero_grad()
        crit(m(xs[0]), ys[0]).backward()
        o.step()
    p0 = [q.detach().clone() for q in ms[1].parameters()]
    gs = GraphedStep(ms[0], crit, os_[0], xs[1], ys[1], warmup=0)
    staged = getattr(gs.x, "_ldnn_s2d", None) is not None
    for i in range(1, a.steps + 1):
        if i == a.lr_drop_at:
            for o in os_:
                o.param_groups[0]["lr"] *= 0.1
        gs(xs[i], ys[i])
        for m, o in zip(ms[1:], os_[1:]):
            o.zero_grad()
            crit(m(xs[i]), ys[i]).backward()
            o.step()
    torch.cuda.synchronize()
    n_bad = 0
    for (n, p), q, s, r in zip(ms[0].named_parameters(), ms[1].parameters(), ms[2].parameters(), p0):
        d1, d2, d3 = ((t.detach() - r).flatten().double() for t in (p, q, s))
        cg = torch.nn.functional.cosine_similarity(d1, d2, dim=0).item()
        ce = torch.nn.functional.cosine_similarity(d3, d2, dim=0).item()
        if cg < ce - 0.1:
            n_bad += 1
            print(json.dumps({"param": n, "cos_graph": round(cg, 4), "cos_eager": round(ce, 4),
                              "stage_s2d": STAGE_S2D, "staged": staged}), flush=True)
    print(json.dumps({"summary": True, "n_bad": n_bad, "stage_s2d": STAGE_S2D, "staged": staged}), flush=True)


if __name__ == "__main__":
    main()
