#!/bin/bash
# PMC counters of every kernel of a short training run (default: the headline bench),
# two passes (SQ + GRBM, then TCC), summarised per kernel by scripts/pmc_table.py:
# MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs),
# LDS bank-conflict cycles per LDS instruction, L2 (TCC) hit rate.
#   bash scripts/pmc_step.sh <tag> [command args...]     (command defaults to bench.py)
set -e
tag=$1; shift
cmd=("$@")
[ ${#cmd[@]} -eq 0 ] && cmd=(python3 bench.py --steps 4 --warmup 3)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmc_$tag
rm -rf $d && mkdir -p $d
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $d/p1 -o run -- "${cmd[@]}" > $d/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $d/p2 -o run -- "${cmd[@]}" > $d/p2.log 2>&1
if [ -n "$MEM" ]; then   # HBM-side bytes (FETCH_SIZE reads 1/2 of 16-B-per-lane loads: doubled in the table)
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $d/p3 -o run -- "${cmd[@]}" > $d/p3.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $d/p4 -o run -- "${cmd[@]}" > $d/p4.log 2>&1
fi
python3 scripts/pmc_util.py $d > $d/table.txt
cat $d/table.txt
