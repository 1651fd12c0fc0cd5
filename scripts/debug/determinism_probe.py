"""Run-to-run reproducibility of one ResNet-18 / EnhancedCNN training step on ldnn's
kernels: the same weights and input, stepped R times; per module, the largest
relative difference of its forward output between runs, then of every parameter
gradient.  fp32-atomic arrival order may differ (|rel| ~1e-6); anything much larger
points at a race.  Prints one JSON line per module / parameter with a spread above
`--show`, plus a summary line."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402


def rel(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--hw", type=int, default=112)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--show", type=float, default=1e-4)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = build_model(a.model)
    xavier_init(m)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    ldnn.prepare(m, "cuda")
    m.train()
    f = m._ldnn_flat
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(a.batch, 3, a.hw, a.hw, device="cuda", generator=g).bfloat16()
    nc = 1000 if a.model == "resnet18" else 10
    y = torch.randint(0, nc, (a.batch,), device="cuda", generator=g)
    outs = []
    hooks = []
    cur = {}

    def hook(name):
        def fn(mod, inp, out):
            o = out[0] if isinstance(out, (tuple, list)) else out
            if torch.is_tensor(o):
                cur[name] = o.detach().float().clone()
        return fn

    for name, mod in m.named_modules():
        if name:
            hooks.append(mod.register_forward_hook(hook(name)))
    for r in range(a.runs):
        m.load_state_dict(sd)   # same weights and BN buffers every run
        f.refresh_shadow()
        f.reattach_grads()
        f.grad.zero_()
        f._stale.clear()
        cur = {}
        out = m(x)
        loss = CrossEntropyLoss()(out, y)
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}
        bufs = {n: b.detach().float().clone() for n, b in m.named_buffers()}
        outs.append((dict(cur), grads, bufs, out.detach().float().clone()))
    worst = {"fwd": 0.0, "grad": 0.0, "buf": 0.0}
    first = None
    base = outs[0]
    for r in range(1, a.runs):
        o = outs[r]
        for name in base[0]:
            d = rel(o[0][name], base[0][name])
            worst["fwd"] = max(worst["fwd"], d)
            if d > a.show:
                if first is None:
                    first = name
                print(json.dumps({"run": r, "kind": "fwd", "module": name, "rel": d}))
        for name in base[1]:
            d = rel(o[1][name], base[1][name])
            worst["grad"] = max(worst["grad"], d)
            if d > a.show:
                print(json.dumps({"run": r, "kind": "grad", "param": name, "rel": d}))
        for name in base[2]:
            if "num_batches" in name:
                continue
            d = rel(o[2][name], base[2][name])
            worst["buf"] = max(worst["buf"], d)
            if d > a.show:
                print(json.dumps({"run": r, "kind": "buf", "buffer": name, "rel": d}))
    print(json.dumps({"summary": True, "model": a.model, "batch": a.batch, "hw": a.hw, "worst": worst,
                      "first_fwd_module_over_show": first,
                      "logits_rel": max(rel(outs[r][3], base[3]) for r in range(1, a.runs))}), flush=True)


if __name__ == "__main__":
    main()
