"""Average PMC counters per kernel-name substring from rocprofv3 counter CSVs."""
import collections
import csv
import glob
import sys

d, sub = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
for k, v in out.items():
    print(f"{k:28s} {v:16.1f}")
if "SQ_WAVE_CYCLES" in out:
    wc = out["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in out:
            print(f"{k}/WAVE_CYCLES = {out[k] / wc:.3f}")
