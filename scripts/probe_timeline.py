"""Comm / compute timeline of an overlap-probe run under rocprofv3 --kernel-trace: for the
last K steps of the "with stand-in" phase, how long the stand-in copies (the collectives'
stand-in, standin_copy_kernel) ran, how much of that the compute kernels covered, and
where the compute queue sat idle while a copy ran (the exposed intervals, each tagged with
the compute kernels right before / after it).

    python scripts/probe_timeline.py gpurun_out/<dir>/probe_trace [steps]
"""
import glob
import sqlite3
import sys


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def inter_len(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    db = d if d.endswith(".db") else glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    sc = [(s, e) for n, s, e in rows if "standin_copy" in n]
    if not sc:
        print("no stand-in kernels in the trace")
        return
    # the probe's --tail-steps phase: everything after the last idle gap > 10 ms
    t_end = max(r[2] for r in rows)
    t0 = rows[0][1]
    prev_end = rows[0][2]
    for n, s, e in rows[1:]:
        if s - prev_end > 10_000_000:
            t0 = s
        prev_end = max(prev_end, e)
    comp = [(n, s, e) for n, s, e in rows if "standin_copy" not in n]
    win = (t0, t_end)
    cv = union([(s, e) for _, s, e in comp if s >= win[0] and e <= win[1]])
    sv = union([(s, e) for s, e in sc if s >= win[0] and e <= win[1]])
    span = win[1] - win[0]
    s_busy = sum(e - s for s, e in sv)
    c_busy = sum(e - s for s, e in cv)
    both = inter_len(cv, sv)
    print(f"window {span / 1e3:.1f} us over {steps} steps ({span / 1e3 / steps:.1f} us per step): compute busy "
          f"{c_busy / 1e3:.1f} us, stand-in busy {s_busy / 1e3:.1f} us, overlapped {both / 1e3:.1f} us ({100 * both / max(s_busy, 1):.0f} % of the copies)")
    # exposed intervals: stand-in running, compute idle
    gaps = []
    for s, e in sv:
        cur = s
        for cs, ce in cv:
            if ce <= cur or cs >= e:
                continue
            if cs > cur:
                gaps.append((cur, cs))
            cur = max(cur, ce)
        if cur < e:
            gaps.append((cur, e))
    gaps = [g for g in gaps if g[1] - g[0] > 2_000]
    print(f"{len(gaps)} exposed intervals > 2 us, {sum(e - s for s, e in gaps) / 1e3:.1f} us total:")
    for s, e in sorted(gaps, key=lambda g: g[0] - g[1])[:25]:
        before = [n for n, cs, ce in comp if ce <= s]
        after = [n for n, cs, ce in comp if cs >= e]
        print(f"  {(s - win[0]) / 1e3:9.1f} us +{(e - s) / 1e3:7.1f} us  after {before[-1][:60] if before else '-'}"
              f"  | before {after[0][:60] if after else '-'}")


if __name__ == "__main__":
    main()
