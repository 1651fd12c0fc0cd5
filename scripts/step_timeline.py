"""One training step's kernels in launch order from a rocprofv3 kernel trace:
duration, grid, short name -- the per-layer view the per-name summary hides.

    python scripts/step_timeline.py <trace_dir_or_csv> [--marker sgd_kernel] [--step -2]
"""
import argparse
import csv
import glob
import os
import re


def short(name):
    n = name.replace("ldnn::", "").replace("(anonymous namespace)::", "").replace("convlds::", "")
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    f = a.path if a.path.endswith(".csv") else glob.glob(os.path.join(a.path, "*kernel_trace.csv"))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo = ends[a.step - 1] + 1
    hi = ends[a.step]
    tot = gaps = 0.0
    prev_end = None
    for r in rows[lo:hi + 1]:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        us = (t1 - t0) / 1e3
        tot += us
        if prev_end is not None and t0 > prev_end:
            gaps += (t0 - prev_end) / 1e3
        prev_end = t1 if prev_end is None else max(prev_end, t1)
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{us:8.1f} {g:6d}x{r['Grid_Size_Y']:>4s}  {short(r['Kernel_Name'])}")
    span = (int(rows[hi]["End_Timestamp"]) - int(rows[lo]["Start_Timestamp"])) / 1e3
    print(f"{tot:8.1f} total ({hi - lo + 1} kernels); step span {span:.1f} us, idle gaps between kernels {gaps:.1f} us")


if __name__ == "__main__":
    main()
