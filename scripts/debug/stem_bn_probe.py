"""ResNet-18 stem (conv1 -> bn1 -> relu -> maxpool) in training mode on the native path: the
per-channel statistics of the BN output (mean ~ 0, var ~ 1 when the fused statistics are right)
and of the conv output, for one input size; one JSON line.

    python scripts/debug/stem_bn_probe.py --batch 16 --hw 64
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
    ldnn.prepare(m, "cuda")
    x = torch.randn(a.batch, 3, a.hw, a.hw, device="cuda")
    for rep in range(3):
        y = m.conv1(x)
        yf = y.float()
        z = m.bn1(y).float()
        bn = m.bn1
        row = {"rep": rep, "batch": a.batch, "hw": a.hw,
               "conv_mean": yf.mean((0, 2, 3))[:4].tolist(), "conv_std": yf.std((0, 2, 3))[:4].tolist(),
               "bn_out_mean": z.mean((0, 2, 3))[:4].tolist(), "bn_out_std": z.std((0, 2, 3))[:4].tolist(),
               "running_mean": bn.running_mean[:4].tolist(), "running_var": bn.running_var[:4].tolist(),
               "pre": str(type(bn.__dict__.get("_ldnn_pre")))}
        print(json.dumps(row))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
