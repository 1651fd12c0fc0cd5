"""One training step's kernels in launch order from a rocprofv3 kernel trace:
duration, grid, short name -- the per-layer view the per-name summary hides.

    python scripts/step_timeline.py <trace_dir_csv_or_rocpd_db> [--marker sgd_kernel] [--step -2]
"""
import argparse
import csv
import glob
import os
import re
import sqlite3


def short(name):
    n = name.replace("ldnn::", "").replace("(anonymous namespace)::", "").replace("convlds::", "")
    n = re.sub(r"\(.*$", "", n)
    n = re.sub(r"^void ", "", n)
    return n[:90]


def load(path):
    """Rows keyed like the csv trace, from a kernel_trace.csv or a rocpd .db (file or directory)."""
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    if dbs and not path.endswith(".csv"):
        q = "select name, start, end, grid_x, grid_y, workgroup_x from kernels"
        rows = [dict(Kernel_Name=n, Start_Timestamp=s, End_Timestamp=e, Grid_Size_X=gx, Grid_Size_Y=str(gy),
                     Workgroup_Size_X=wx) for n, s, e, gx, gy, wx in sqlite3.connect(dbs[0]).execute(q)]
    else:
        f = path if path.endswith(".csv") else glob.glob(os.path.join(path, "*kernel_trace.csv"))[0]
        rows = list(csv.DictReader(open(f)))
    return sorted(rows, key=lambda r: int(r["Start_Timestamp"]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--step", type=int, default=-2)
    a = ap.parse_args()
    rows = load(a.path)
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
