#!/bin/bash
# Kernel-trace profiles of the CNN training step (ldnn path only); summaries -> gpurun_out/prof_<model>/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in ${CNN:-"resnet18 64" "enhanced_cnn 256"}; do
  set -- $spec
  d=gpurun_out/prof_$1
  rm -rf $d && mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/bench_cnn.py --model $1 --batch $2 --steps 20 --warmup 5 --no-stock ${EXTRA} > $d/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $d 25 > $d/summary.txt
  head -25 $d/summary.txt
done
