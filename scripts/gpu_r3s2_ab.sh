#!/bin/bash
# MLP headline A/B (fused head forward on / off, alternated), kernel trace of the default step,
# conv BN-statistics epilogue probe
set -o pipefail
O=gpurun_out/r3s2ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-configs --steps 50 --warmup 10 > $O/fused_$rep.txt 2>&1 || { tail -30 $O/fused_$rep.txt; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/fused_$rep.txt
  timeout -k 10 200 python -u bench.py --no-configs --steps 50 --warmup 10 --no-fuse-head-fwd > $O/sep_$rep.txt 2>&1 || { tail -30 $O/sep_$rep.txt; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/sep_$rep.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o mlp -- python3 bench.py --no-configs --steps 30 --warmup 5 > $O/prof.txt 2>&1 || { tail -30 $O/prof.txt; exit 1; }
timeout -k 10 120 python -u scripts/conv_bn_probe.py --batch 64 > $O/conv_bn_probe64.txt 2>&1 || { tail -30 $O/conv_bn_probe64.txt; exit 1; }
cat $O/conv_bn_probe64.txt
timeout -k 10 120 python -u scripts/conv_bn_probe.py --batch 256 --iters 20 > $O/conv_bn_probe256.txt 2>&1 || { tail -30 $O/conv_bn_probe256.txt; exit 1; }
cat $O/conv_bn_probe256.txt
