"""Summarise scripts/experiment_matrix.sh runs: final metrics table (markdown) and one
figure with the six variants' validation-accuracy / loss curves per global epoch.
    python scripts/matrix_report.py gpurun_out/matrix profiles/experiment_matrix_r2"""
import json
import os
import sys

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

src, dst = sys.argv[1], sys.argv[2]
names = ["BAR", "BR", "BDR", "DAR", "DR", "DDR"]
rows, curves = [], {}
for n in names:
    p = os.path.join(src, n, "histories.json")
    if not os.path.exists(p):
        continue
    r = json.load(open(p))
    h = r["histories"]
    tl, ta, vl, va = h[4], h[5], h[6], h[7]
    curves[n] = (ta, va, tl, vl)
    rows.append((n, len(va), va[0], max(va), va[-1], ta[-1], vl[-1], tl[-1], r.get("test_acc"), r.get("f1_macro")))
with open(dst + ".md", "w") as f:
    f.write("| variant | global epochs | epoch-1 val acc % | best val acc % | final val acc % | final train acc % "
            "| final val loss | final train loss | test acc % | test macro F1 |\n|" + "---|" * 10 + "\n")
    for n, e, v1, vb, vf, tf, vlf, tlf, te, f1 in rows:
        f.write(f"| {n} | {e} | {v1:.2f} | {vb:.2f} | {vf:.2f} | {tf:.2f} | {vlf:.4f} | {tlf:.4f} | "
                f"{te if te is None else round(te, 2)} | {f1 if f1 is None else round(f1, 4)} |\n")
fig, ax = plt.subplots(1, 2, figsize=(16, 6))
for i, (n, (ta, va, tl, vl)) in enumerate(curves.items()):
    x = range(1, len(va) + 1)
    ax[0].plot(x, va, color=f"C{i}", label=f"{n} val")
    ax[0].plot(x, ta, "--", color=f"C{i}", alpha=0.5, label=f"{n} train")
    ax[1].plot(x, vl, color=f"C{i}", label=f"{n} val")
ax[0].set_xlabel("global epoch"); ax[0].set_ylabel("accuracy %"); ax[0].legend(ncol=2, fontsize=8)
ax[1].set_xlabel("global epoch"); ax[1].set_ylabel("validation loss"); ax[1].legend(fontsize=8)
fig.tight_layout()
fig.savefig(dst + ".png", dpi=80)
print(open(dst + ".md").read())
