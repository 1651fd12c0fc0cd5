"""Summarise a rocprofv3 --kernel-trace output (csv directory or rocpd .db files under
it): per-kernel total / per-step time.

    python scripts/kernel_summary.py gpurun_out/prof 30
"""
import csv
import glob
import sqlite3
import sys
from collections import defaultdict

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
tot, cnt = defaultdict(float), defaultdict(int)
for fn in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    with open(fn) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name") or row.get("KernelName") or "?"
            dt = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            tot[name] += dt
            cnt[name] += 1
for fn in glob.glob(f"{d}/**/*.db", recursive=True) + glob.glob(f"{d}/*.db"):
    for name, dur in sqlite3.connect(fn).execute("select name, duration from kernels"):
        tot[name] += dur / 1e3
        cnt[name] += 1
all_us = sum(tot.values())
print(f"{'us/step':>9} {'calls/step':>10} {'avg us':>8}  kernel   (total {all_us / steps:.1f} us/step over {steps} steps)")
for name, t in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{t / steps:9.1f} {cnt[name] / steps:10.2f} {t / cnt[name]:8.2f}  {name[:150]}")
