"""Compact per-kernel PMC table from scripts/pmc_step.sh passes:
  mfma%   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
            (MFMA_BUSY sums 16 cycles per v_mfma_f32_16x16x32_bf16 over all SIMDs; GRBM_GUI_ACTIVE
             sums the 8 XCDs' busy cycles, so GRBM / 8 = the kernel's GPU cycles)
  ldsconf = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per LDS instruction)
  waitlds = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  l2hit%  = TCC_HIT / (TCC_HIT + TCC_MISS)
  usage: python scripts/pmc_util.py gpurun_out/pmc_<tag> [min_calls]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    p = f.split("/")[len(d.rstrip("/").split("/"))]
    for r in csv.DictReader(open(f)):
        cnt[r["Kernel_Name"]][(p, r["Counter_Name"])].append(float(r["Counter_Value"]))


def avg(c, k, p=None):
    vals = [v for (pp, kk), v in c.items() if kk == k and (p is None or pp == p)]
    vals = [x for v in vals for x in v]
    return sum(vals) / len(vals) if vals else float("nan")


def short(n):
    n = n.replace("void ", "").replace("ldnn::", "").replace("(anonymous namespace)::", "").split("(")[0]
    return n[:70]


rows = []
for name, c in cnt.items():
    calls = max(len(v) for v in c.values())
    g1 = avg(c, "GRBM_GUI_ACTIVE", "p1")
    g2 = avg(c, "GRBM_GUI_ACTIVE", "p2")
    mf = avg(c, "SQ_VALU_MFMA_BUSY_CYCLES") / (1024 * g1 / 8) if g1 == g1 else float("nan")
    busy = avg(c, "SQ_BUSY_CYCLES") / (g1 / 8)
    lds = avg(c, "SQ_INSTS_LDS")
    conf = avg(c, "SQ_LDS_BANK_CONFLICT") / lds if lds and lds == lds else float("nan")
    wl = avg(c, "SQ_WAIT_INST_LDS") / avg(c, "SQ_WAVE_CYCLES")
    h, m = avg(c, "TCC_HIT_sum"), avg(c, "TCC_MISS_sum")
    # HBM-side bytes (MEM=1 passes): FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts half the bytes
    # of 16-B-per-lane loads on gfx950 (MI355X_MICROARCH.md), so it is doubled here
    rd = 2 * avg(c, "FETCH_SIZE", "p3") * 1024
    wr = avg(c, "WRITE_SIZE", "p4") * 1024
    g3 = avg(c, "GRBM_GUI_ACTIVE", "p3")
    bpc = (rd + wr) / (g3 / 8) if g3 == g3 and rd == rd and wr == wr else float("nan")
    rows.append((g1, short(name), calls, mf, busy, conf, wl, h / (h + m) if h == h and m == m else float("nan"),
                 rd / 2**20, wr / 2**20, bpc))
mem = any(r[8] == r[8] for r in rows)
print(f"{'GRBM/8 cyc':>11} {'calls':>5} {'mfma%':>6} {'ldsconf':>7} {'waitlds':>7} {'l2hit%':>6}"
      + (f" {'rdMB':>8} {'wrMB':>8} {'B/cyc':>6}" if mem else "") + "  kernel")
for g1, n, calls, mf, busy, conf, wl, hit, rmb, wmb, bpc in sorted(rows, key=lambda r: -r[0] * r[2]):
    if calls < (int(sys.argv[2]) if len(sys.argv) > 2 else 1):
        continue
    extra = f" {rmb:8.1f} {wmb:8.1f} {bpc:6.0f}" if mem else ""
    print(f"{g1 / 8:11.0f} {calls:5d} {100 * mf:6.1f} {conf:7.3f} {wl:7.3f} {100 * hit:6.1f}{extra}  {n}")
if mem:
    print("# rdMB = 2 x FETCH_SIZE, wrMB = WRITE_SIZE (HBM / Infinity-Cache side), B/cyc = (rd + wr) per GPU cycle "
          "(GRBM_GUI_ACTIVE / 8); 8 TB/s at ~2.4 GHz is ~3300 B/cyc")
