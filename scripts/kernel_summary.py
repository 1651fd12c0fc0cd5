"""Summarise a rocprofv3 --kernel-trace csv directory: per-kernel total / per-step time."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
tot, cnt = defaultdict(float), defaultdict(int)
for fn in files:
    with open(fn) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or "?"
            dt = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            tot[name] += dt
            cnt[name] += 1
all_us = sum(tot.values())
print(f"{'us/step':>9} {'calls/step':>10} {'avg us':>8}  kernel   (total {all_us / steps:.1f} us/step over {steps} steps)")
for name, t in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{t / steps:9.1f} {cnt[name] / steps:10.2f} {t / cnt[name]:8.2f}  {name[:150]}")
