"""Per-dispatch kernel table from a rocprofv3 rocpd .db (or a directory holding one):
consecutive dispatches of one kernel with one grid are grouped, with the median
duration -- a microbenchmark's shapes show up as consecutive groups.

    python scripts/dispatch_table.py gpurun_out/<dir>/microprof_enhanced_cnn [min_count]
"""
import glob
import sqlite3
import sys


def main():
    d = sys.argv[1]
    min_count = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dbs = [d] if d.endswith(".db") else glob.glob(f"{d}/**/*.db", recursive=True)
    for db in dbs:
        c = sqlite3.connect(db)
        rows = list(c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, "
                              "accum_vgpr_count from kernels order by start"))
        groups = []
        for r in rows:
            key = (r[0], r[2], r[3], r[4])
            if groups and groups[-1][0] == key:
                groups[-1][1].append(r[1])
            else:
                groups.append([key, [r[1]], r[5], r[6], r[7], r[8]])
        for key, durs, wg, lds, vgpr, agpr in groups:
            if len(durs) < min_count:
                continue
            durs.sort()
            med = durs[len(durs) // 2] / 1e3
            wgs = (key[1] // max(wg, 1)) * key[2] * key[3]
            print(f"{len(durs):4d} x {med:8.2f} us  {wgs:6d} WG  lds {lds:6d}  v/a {vgpr}/{agpr}  {key[0][:110]}")


if __name__ == "__main__":
    main()
