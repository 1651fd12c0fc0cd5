"""Overlap of side-stream kernels with main-stream kernels in a rocprofv3 kernel trace
(CSV): for every kernel on the side queue, the part of its [start, end) during which
some main-queue kernel was also running.  Usage: python scripts/trace_overlap.py trace.csv [side_queue]"""
import csv
import sys
from collections import Counter


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    qs = Counter(r["Queue_Id"] for r in rows)
    main_q = qs.most_common(1)[0][0]
    side_q = sys.argv[2] if len(sys.argv) > 2 else None
    side = [r for r in rows if r["Queue_Id"] != main_q and (side_q is None or r["Queue_Id"] == side_q)]
    mains = sorted((r["s"], r["e"]) for r in rows if r["Queue_Id"] == main_q)
    tot, ov = 0, 0
    per = []
    j0 = 0
    for r in sorted(side, key=lambda r: r["s"]):
        s, e = r["s"], r["e"]
        tot += e - s
        o = 0
        while j0 < len(mains) and mains[j0][1] < s - 10_000_000:
            j0 += 1
        for ms, me in mains[j0:]:
            if ms >= e:
                break
            o += max(0, min(e, me) - max(s, ms))
        ov += min(o, e - s)
        per.append((e - s, min(o, e - s)))
    print(f"main queue {main_q}: {qs[main_q]} kernels; side kernels: {len(side)}, "
          f"busy {tot / 1e3:.1f} us, overlapped with main-queue kernels {ov / 1e3:.1f} us ({100 * ov / max(tot, 1):.1f} %)")
    if per:
        durs = sorted(d for d, _ in per)
        print(f"side kernel duration median {durs[len(durs) // 2] / 1e3:.1f} us")


if __name__ == "__main__":
    main()
