"""ResNet-18 forward module by module on the native path (training mode), each stage's output
against an fp32 CPU copy of the same module fed the same input: relative error per stage, one
JSON line each.  Localises a stage whose fused kernels go wrong for an input size.

    python scripts/debug/resnet_block_probe.py --batch 16 --hw 64
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import ldnn  # noqa: E402
from ldnn.models import build_model, xavier_init  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--hw", type=int, default=64)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = build_model("resnet18")
    xavier_init(m)
    ref = build_model("resnet18")
    ref.load_state_dict(m.state_dict())
    ldnn.prepare(m, "cuda")
    x = torch.randn(a.batch, 3, a.hw, a.hw)
    stages = [("stem", lambda mm: (lambda t: mm.maxpool(mm.relu(mm.bn1(mm.conv1(t))))))]
    for ln in ("layer1", "layer2", "layer3", "layer4"):
        for bi in range(2):
            stages.append((f"{ln}.{bi}", lambda mm, ln=ln, bi=bi: getattr(mm, ln)[bi]))
    h = x.cuda()
    for name, get in stages:
        hin = h.float().cpu()
        h = get(m)(h)
        r = get(ref)(hin)
        hf = h.float().cpu()
        err = ((hf - r).norm() / r.norm().clamp_min(1e-12)).item()
        print(json.dumps({"stage": name, "shape": list(h.shape), "rel_err": round(err, 5),
                          "out_std": round(hf.std().item(), 5), "ref_std": round(r.std().item(), 5)}), flush=True)
        h = h.detach()


if __name__ == "__main__":
    main()
