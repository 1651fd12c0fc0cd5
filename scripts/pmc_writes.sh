#!/bin/bash
# Write-path counters of the EnhancedCNN b64 step (partial-line writes to the fabric vs full lines).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
d=gpurun_out/pmc_writes; rm -rf $d && mkdir -p $d
timeout -s KILL 60 rocprofv3 -L > $d/avail.txt 2>&1
grep -o "TCC_EA0_WR[A-Z0-9_]*\|TCC_WRITE[A-Z0-9_]*\|TCC_EA_WR[A-Z0-9_]*" $d/avail.txt | sort -u > $d/names.txt
cat $d/names.txt | head -20
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE --output-format csv -d $d/p1 -o run -- python3 scripts/bench_cnn.py --model enhanced_cnn --batch 64 --steps 3 --warmup 2 --no-stock --graph > $d/p1.log 2>&1
echo "rc=$?"; tail -3 $d/p1.log
