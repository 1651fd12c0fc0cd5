"""Isolate the ResNet-18 stem BN+ReLU+max-pool gradient gap.

Three ways to compute the stem (conv1 7x7/2 -> bn1 -> relu -> maxpool 3x3/2) gradients:
  fused  -- ldnn, LF.BN_POOL_FUSED=True  (bn_maxpool_fwd/bwd, stats from conv epilogue)
  sep    -- ldnn, LF.BN_POOL_FUSED=False (BN apply + separate pool passes)
  fp32   -- plain torch.nn oracle (tests/ref_models.py) with the same weights

Part A injects the SAME upstream gradient G at the pool output into all three.
Part B splits the full model at the stem output: the trunk's gradient arriving at the
stem (G_fused, G_sep, G_fp32) is compared first, then fed into the stem.
Prints one JSON line per (config, quantity)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, xavier_init  # noqa: E402
from ldnn.ops import functional as LF  # noqa: E402
from ref_models import oracle_for, rel  # noqa: E402

DEV = os.environ.get("DEV", "cuda")


def ldnn_stem(m, x):
    return LF.bn_relu_maxpool(m.conv1(x), m.bn1, m.maxpool)


def ldnn_trunk(m, y):
    z = m.layer4(m.layer3(m.layer2(m.layer1(y))))
    return m.fc(m.avgpool(z).flatten(1))


def grads(m):
    return {"bn1.weight": m.bn1.weight.grad.detach().float().clone(),
            "bn1.bias": m.bn1.bias.grad.detach().float().clone(),
            "conv1.weight": m.conv1.weight.grad.detach().float().clone()}


def zero(m):
    f = getattr(m, "_ldnn_flat", None)
    if f is None:   # the torch.nn oracle
        for p in m.parameters():
            p.grad = None
        return
    f.reattach_grads()   # ldnn: gradients are views of the flat buffer
    f.grad.zero_()
    f._stale.clear()


def run(N, H, seed=0):
    torch.manual_seed(seed)
    m = build_model("resnet18")
    xavier_init(m)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    ldnn.prepare(m, DEV)
    m.train()
    ref = oracle_for("resnet18", sd, DEV)
    ref.train()
    g = torch.Generator(device=DEV).manual_seed(seed + 1)
    x = torch.randn(N, 3, H, H, device=DEV, generator=g).bfloat16()
    yl = torch.randint(0, 10, (N,), device=DEV, generator=g)
    P = ((H + 1) // 2 + 1) // 2
    G = torch.randn(N, 64, P, P, device=DEV, generator=g).bfloat16().float()
    tag = f"N{N}_H{H}"
    out = []

    # ---- part A: identical upstream gradient G at the pool output
    res = {}
    for name, fused in (("fused", True), ("sep", False), ("sep2", False)):
        LF.BN_POOL_FUSED = fused
        zero(m)
        y = ldnn_stem(m, x)
        (y.float() * G).sum().backward()
        res[name] = (y.detach().float(), grads(m))
    zero(ref)
    xf = x.float()
    yr = ref.stem(xf)
    (yr * G).sum().backward()
    gref = {"bn1.weight": ref.bn1.weight.grad, "bn1.bias": ref.bn1.bias.grad, "conv1.weight": ref.conv1.weight.grad}
    gref_a = {k: v.clone() for k, v in gref.items()}
    out.append({"cfg": tag, "part": "A_injected_G", "q": "stem_out",
                "fused_vs_sep_maxabs": (res["fused"][0] - res["sep"][0]).abs().max().item(),
                "fused_vs_fp32": rel(res["fused"][0], yr), "sep_vs_fp32": rel(res["sep"][0], yr)})
    for k in gref:
        out.append({"cfg": tag, "part": "A_injected_G", "q": k,
                    "fused_vs_fp32": rel(res["fused"][1][k], gref[k]), "sep_vs_fp32": rel(res["sep"][1][k], gref[k]),
                    "fused_vs_sep": rel(res["fused"][1][k], res["sep"][1][k]),
                    "sep_vs_sep2": rel(res["sep2"][1][k], res["sep"][1][k])})

    # ---- part B: the trunk's own gradient at the stem output
    crit = CrossEntropyLoss()
    gt = {}
    full = {}
    for name, fused in (("fused", True), ("sep", False), ("sep2", False)):
        LF.BN_POOL_FUSED = fused
        zero(m)
        y = ldnn_stem(m, x)
        yd = y.detach().float().bfloat16().requires_grad_(True)
        logits = ldnn_trunk(m, yd)
        crit(logits, yl).backward()
        gt[name] = yd.grad.detach().float().clone()
        y.float().mul(gt[name]).sum().backward()   # push that gradient through the stem
        full[name] = (logits.detach().float(), grads(m))
    zero(ref)
    yr = ref.stem(xf)
    yrd = yr.detach().requires_grad_(True)
    lr_ = ref.trunk(yrd)
    torch.nn.functional.cross_entropy(lr_, yl).backward()
    g_true = yrd.grad.detach().clone()
    (yr * g_true).sum().backward()
    gref = {"bn1.weight": ref.bn1.weight.grad, "bn1.bias": ref.bn1.bias.grad, "conv1.weight": ref.conv1.weight.grad}
    out.append({"cfg": tag, "part": "B_model", "q": "logits",
                "fused_vs_fp32": rel(full["fused"][0], lr_), "sep_vs_fp32": rel(full["sep"][0], lr_),
                "fused_vs_sep": rel(full["fused"][0], full["sep"][0])})
    out.append({"cfg": tag, "part": "B_model", "q": "grad_at_stem_out",
                "fused_vs_fp32": rel(gt["fused"], g_true), "sep_vs_fp32": rel(gt["sep"], g_true),
                "fused_vs_sep": rel(gt["fused"], gt["sep"]), "sep_vs_sep2": rel(gt["sep2"], gt["sep"])})
    for k in gref:
        out.append({"cfg": tag, "part": "B_model", "q": k,
                    "fused_vs_fp32": rel(full["fused"][1][k], gref[k]), "sep_vs_fp32": rel(full["sep"][1][k], gref[k]),
                    "fused_vs_sep": rel(full["fused"][1][k], full["sep"][1][k]),
                    "sep_vs_sep2": rel(full["sep2"][1][k], full["sep"][1][k])})
    # part C: fp32-true upstream gradient fed into both ldnn stems (isolates the stem backward at model scale)
    for name, fused in (("fused", True), ("sep", False)):
        LF.BN_POOL_FUSED = fused
        zero(m)
        y = ldnn_stem(m, x)
        (y.float() * g_true.bfloat16().float()).sum().backward()
        full[name] = grads(m)
    for k in gref:
        out.append({"cfg": tag, "part": "C_true_G", "q": k,
                    "fused_vs_fp32": rel(full["fused"][k], gref[k]), "sep_vs_fp32": rel(full["sep"][k], gref[k])})
    # part D: the fp32 oracle with ONLY the conv1-output gradient rounded to bf16 (what
    # ldnn's BN backward stores): how much of the stem wgrad gap that rounding explains
    zero(ref)
    c = ref.conv1(xf)
    c.register_hook(lambda gr: gr.bfloat16().float())
    yr2 = ref.maxpool(torch.relu(ref.bn1(c)))
    (yr2 * G).sum().backward()
    out.append({"cfg": tag, "part": "D_fp32_bf16_dx", "q": "conv1.weight",
                "vs_fp32": rel(ref.conv1.weight.grad, gref_a["conv1.weight"])})
    # D2: ... and the conv output itself stored in bf16 (what the BN reads in ldnn)
    zero(ref)
    c = ref.conv1(xf)
    c.register_hook(lambda gr: gr.bfloat16().float())
    cb = c + (c.detach().bfloat16().float() - c.detach())   # bf16 value, identity gradient
    yr3 = ref.maxpool(torch.relu(ref.bn1(cb)))
    (yr3 * G).sum().backward()
    out.append({"cfg": tag, "part": "D2_fp32_bf16_conv_out_and_dx", "q": "conv1.weight",
                "vs_fp32": rel(ref.conv1.weight.grad, gref_a["conv1.weight"]),
                "bn1.weight_vs_fp32": rel(ref.bn1.weight.grad, gref_a["bn1.weight"])})
    # part E: stock PyTorch bf16 autocast (MIOpen / hipBLASLt) on the same model: its
    # gradient at the stem output vs fp32, twice (its own run-to-run spread)
    if DEV == "cuda":
        gs = []
        for _ in range(2):
            zero(ref)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                yb = ref.stem(xf)
                ybd = yb.detach().requires_grad_(True)
                lb = ref.trunk(ybd)
            torch.nn.functional.cross_entropy(lb.float(), yl).backward()
            gs.append(ybd.grad.detach().float().clone())
        out.append({"cfg": tag, "part": "E_stock_autocast_bf16", "q": "grad_at_stem_out",
                    "vs_fp32": rel(gs[0], g_true), "run_to_run": rel(gs[1], gs[0])})
    LF.BN_POOL_FUSED = True
    return out


if __name__ == "__main__":
    for N, H in ((4, 64), (16, 112), (16, 224)):
        for rec in run(N, H):
            print(json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)
