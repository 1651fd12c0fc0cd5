#!/bin/bash
# PMC + kernel-trace passes over scripts/prof_pp.py; summaries in gpurun_out/pmc_pp/
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
o=gpurun_out/pmc_pp; rm -rf $o; mkdir -p $o
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/kt -o run -- python3 scripts/prof_pp.py "$@" > $o/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $o/p1 -o run -- python3 scripts/prof_pp.py "$@" > $o/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $o/p2 -o run -- python3 scripts/prof_pp.py "$@" > $o/p2.log 2>&1 || exit $?
python3 scripts/pmc_table.py $o > $o/summary.txt
