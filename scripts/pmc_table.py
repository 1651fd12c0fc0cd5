"""Per-kernel table from a rocprofv3 output dir: mean duration (kernel-trace pass
under kt/) and mean PMC counters (every other pass), one row per kernel name.
Adds MHz = GRBM_GUI_ACTIVE / duration and MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE x 4 SIMD x 256 CU)... printed raw where the normalisation is unknown."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
dur = collections.defaultdict(list)
for f in glob.glob(f"{d}/kt/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))


def short(n):
    return n if len(n) < 90 else n[:87] + "..."


for name in sorted(set(dur) | set(cnt), key=lambda n: -sum(dur.get(n, [0]))):
    ds = sorted(dur.get(name, []))
    med = ds[len(ds) // 2] if ds else float("nan")
    print(f"== {short(name)}\n   calls {len(ds)}  median {med:.1f} us  min {ds[0] if ds else float('nan'):.1f} us")
    c = {k: sum(v) / len(v) for k, v in cnt.get(name, {}).items()}
    for k in sorted(c):
        print(f"   {k:28s} {c[k]:18.1f}")
    if "GRBM_GUI_ACTIVE" in c and ds:
        print(f"   -> GRBM_GUI_ACTIVE / median duration = {c['GRBM_GUI_ACTIVE'] / med:.0f} MHz")
