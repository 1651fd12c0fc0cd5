"""Where a small conv pass spends its time: the LDNN_CONV_XF=32 diagnostic build of the
LDS-DMA conv kernel stamps s_memrealtime (100 MHz) per workgroup at entry, after its first
K-tile landed (prologue), after the main loop and at exit (split-K hand-off + epilogue).
Per pass: the dispatch ramp (last entry - first entry), the medians of the three phases,
and the span first entry -> last exit, beside the event-timed pass.

    LDNN_CONV_XF=32 python scripts/conv_phase_trace.py [--model enhanced_cnn] [--batch 64]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("LDNN_CONV_XF", "32")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ldnn  # noqa: E402,F401
from ldnn.ops import _ext  # noqa: E402

SHAPES = {"enhanced_cnn": [(128, 16, 128, 3, 1, 1), (256, 8, 256, 3, 1, 1), (512, 4, 512, 3, 1, 1)],
          "resnet18_l1": [(64, 56, 64, 3, 1, 1)],
          "resnet18": [(64, 56, 64, 3, 1, 1), (128, 28, 128, 3, 1, 1), (256, 14, 256, 3, 1, 1), (512, 7, 512, 3, 1, 1)]}


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else 0.0


def pct(v, q):
    v = sorted(v)
    return round(v[min(len(v) - 1, int(q * len(v)))], 2) if v else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="enhanced_cnn", choices=list(SHAPES))
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    C = _ext._C
    assert C is not None and os.environ.get("LDNN_CONV_XF") == "32"
    tr = torch.zeros(1 << 16, 8, dtype=torch.int64, device="cuda")
    C.set_conv_trace(tr)
    N = a.batch
    for (Ci, H, K, R, st, pad) in SHAPES[a.model]:
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(N, H, H, Ci, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, Ci, device="cuda") * 0.05).bfloat16()
        y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(N, P, P, K, device="cuda").bfloat16()
        dx = torch.empty_like(x)
        dw = torch.empty(K, R, R, Ci, device="cuda", dtype=torch.float32)
        passes = {"fwd": lambda: C.conv_fwd(x, w, y, st, pad), "dgrad": lambda: C.conv_dgrad(dy, w, dx, st, pad),
                  "wgrad": lambda: C.conv_wgrad(dy, x, dw, st, pad)}
        for name, fn in passes.items():
            for _ in range(3):
                fn()
            tr.zero_()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            t = tr.cpu()
            t = t[t[:, 0] > 0].double() * 0.01   # 100 MHz ticks -> us
            if len(t) == 0:
                print(json.dumps({"shape": f"C{Ci} H{H} K{K}", "pass": name, "traced": 0}), flush=True)
                continue
            t0 = t[:, 0].min()
            ok = t[:, 3] > 0
            rec = {"shape": f"N{N} C{Ci} H{H} K{K}", "pass": name, "workgroups": len(t),
                   "event_us": round(s.elapsed_time(e) * 1e3, 2),
                   "span_us": round((t[ok, 3].max() - t0).item(), 2),
                   "ramp_us": round((t[:, 0].max() - t0).item(), 2),
                   "prologue_us": round(med((t[ok, 1] - t[ok, 0]).tolist()), 2),
                   "loop_us": round(med((t[ok, 2] - t[ok, 1]).tolist()), 2),
                   "tail_us": round(med((t[ok, 3] - t[ok, 2]).tolist()), 2),
                   "wg_total_us": round(med((t[ok, 3] - t[ok, 0]).tolist()), 2),
                   "late_start_wgs": int(((t[:, 0] - t0) > 2.0).sum().item()),
                   # tail spread: a split-K hand-off's last-arriving workgroup also sums the slabs
                   "tail_p10_p90": [pct((t[ok, 3] - t[ok, 2]).tolist(), 0.1), pct((t[ok, 3] - t[ok, 2]).tolist(), 0.9)],
                   "loop_p10_p90": [pct((t[ok, 2] - t[ok, 1]).tolist(), 0.1), pct((t[ok, 2] - t[ok, 1]).tolist(), 0.9)]}
            # split-K combine phases (stamps 4..6): slab stores drained, ticket drawn, slabs summed (summer)
            cb = ok & (t[:, 4] > 0)
            if cb.any():
                sm = cb & (t[:, 6] > 0)
                rec["combine"] = {"store_drain_us": round(med((t[cb, 4] - t[cb, 2]).tolist()), 2),
                                  "ticket_us": round(med((t[cb, 5] - t[cb, 4]).tolist()), 2),
                                  "summers": int(sm.sum().item()),
                                  "sum_loads_us": round(med((t[sm, 6] - t[sm, 5]).tolist()), 2) if sm.any() else None,
                                  "epilogue_us": round(med((t[sm, 3] - t[sm, 6]).tolist()), 2) if sm.any() else None,
                                  "summer_tail_us": round(med((t[sm, 3] - t[sm, 2]).tolist()), 2) if sm.any() else None,
                                  "summer_wait_for_last_us": round(med((t[sm, 5] - t[sm, 4]).tolist()), 2) if sm.any() else None}
            print(json.dumps(rec), flush=True)
    C.set_conv_trace(None)


if __name__ == "__main__":
    main()
