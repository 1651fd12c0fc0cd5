"""Per-dispatch PMC table (rocprofv3 --pmc csv): consecutive dispatches of one kernel
with one grid grouped, counters averaged -- mfma busy %, wait share, wave cycles.

    python scripts/pmc_dispatch.py gpurun_out/<dir>/micropmc_enhanced_cnn
"""
import csv
import glob
import sys
from collections import OrderedDict, defaultdict


def main():
    d = sys.argv[1]
    for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        disp = OrderedDict()
        for r in csv.DictReader(open(fn)):
            k = int(r["Dispatch_Id"])
            e = disp.setdefault(k, {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]),
                                    "wg": int(r["Workgroup_Size"]), "dur": (int(r["End_Timestamp"]) -
                                                                           int(r["Start_Timestamp"])) / 1e3})
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        groups = []
        for e in disp.values():
            key = (e["name"], e["grid"])
            if groups and groups[-1][0] == key:
                groups[-1][1].append(e)
            else:
                groups.append([key, [e]])
        print(f"{'n':>3} {'us':>7} {'WG':>6} {'mfma%':>6} {'wait%':>6} {'issue%':>6} {'active%':>7}  kernel")
        for (name, grid), es in groups:
            if not any(s in name for s in ("conv", "gemm", "bn_", "slab", "head", "pool", "xent")):
                continue
            avg = defaultdict(float)
            for e in es:
                for k, v in e.items():
                    if isinstance(v, float):
                        avg[k] += v / len(es)
            gui = avg.get("GRBM_GUI_ACTIVE", 0.0)
            wc = avg.get("SQ_WAVE_CYCLES", 0.0) or 1.0
            mf = 100.0 * avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(1.0, 1024 * gui / 8) if gui else 0.0
            print(f"{len(es):3d} {avg['dur']:7.2f} {grid // max(es[0]['wg'], 1):6d} {mf:6.1f} "
                  f"{100 * avg.get('SQ_WAIT_ANY', 0) / wc:6.1f} {100 * avg.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} "
                  f"{100 * avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.1f}  {name[:100]}")


if __name__ == "__main__":
    main()
