"""CNN training throughput (samples/s, 1 GPU): ldnn native path (implicit-GEMM conv,
fused BN+add+ReLU, fused optimizer) vs stock PyTorch-ROCm (MIOpen convs, autocast bf16,
channels_last, torch.optim), same model / batch / synthetic data.

    python scripts/bench_cnn.py --model enhanced_cnn --batch 256
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402
from ldnn.models import CrossEntropyLoss, build_model, dataset_for, xavier_init  # noqa: E402
from ldnn.data.datasets import SHAPES  # noqa: E402
from ldnn.optim import SGD, Adam  # noqa: E402


def run(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="enhanced_cnn")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-stock", action="store_true")
    ap.add_argument("--conv-impl", type=int, default=0, help="0 = LDS-DMA fast path, 1 = generic conv kernel only")
    ap.add_argument("--graph", action="store_true", help="replay the ldnn step from one hipGraph (train.graphed)")
    ap.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd",
                    help="sgd = momentum 0.9; adam = the reference config (BAR/main.py:53, lr 1e-3)")
    a = ap.parse_args()
    from ldnn.ops import _ext as _e

    _e.C().set_conv_impl(a.conv_impl)
    shape = SHAPES[dataset_for(a.model)]
    nc = 1000 if a.model == "resnet18" else 10
    x = torch.randn(a.batch, *shape, device="cuda")
    y = torch.randint(0, nc, (a.batch,), device="cuda")

    torch.manual_seed(0)
    m = build_model(a.model)
    xavier_init(m)
    ldnn.prepare(m, "cuda")
    opt = (Adam(m.parameters(), lr=1e-3) if a.optimizer == "adam" else SGD(m.parameters(), lr=0.01, momentum=0.9))
    crit = CrossEntropyLoss()
    xb = x.bfloat16()

    def step_ldnn():
        opt.zero_grad()
        crit(m(xb), y).backward()
        opt.step()

    if a.graph:
        from ldnn.train.graphed import GraphedStep

        gs = GraphedStep(m, crit, opt, xb, y)

        def step_ldnn():  # noqa: F811
            gs(xb, y)

    t = run(step_ldnn, a.steps, a.warmup)
    rec = {"model": a.model, "batch": a.batch, "optimizer": a.optimizer, "conv_impl": a.conv_impl, "graph": a.graph, "ldnn_ms": round(t * 1e3, 3), "ldnn_samples_per_s": round(a.batch / t, 1)}
    if not a.no_stock:
        import torch.nn as nn

        torch.manual_seed(0)
        ref = build_model(a.model)
        # swap ldnn layers for stock torch behaviour: run the CPU/fp32 code path under autocast
        ref = ref.cuda().to(memory_format=torch.channels_last)
        os.environ["LDNN_DISABLE_NATIVE"] = "1"
        from ldnn.ops import _ext

        _ext._DISABLED = True
        ropt = (torch.optim.Adam(ref.parameters(), lr=1e-3) if a.optimizer == "adam" else
                torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9))
        ce = nn.CrossEntropyLoss()
        xc = x.contiguous(memory_format=torch.channels_last)

        def step_stock():
            ropt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = ce(ref(xc).float(), y)
            loss.backward()
            ropt.step()

        ts = run(step_stock, a.steps, a.warmup)
        _ext._DISABLED = False
        rec.update(stock_ms=round(ts * 1e3, 3), stock_samples_per_s=round(a.batch / ts, 1),
                   speedup=round(ts / t, 3))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
