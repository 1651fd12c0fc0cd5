#!/bin/bash
# Kernel-trace profiles of the CNN training step (ldnn path only); summaries -> gpurun_out/prof_<model>_b<batch>/summary.txt
# CNN="resnet18:64,enhanced_cnn:256" (model:batch pairs), EXTRA="--graph"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS=, read -ra specs <<< "${CNN:-resnet18:64,enhanced_cnn:256}"
for spec in "${specs[@]}"; do
  model=${spec%%:*}; batch=${spec##*:}
  d=gpurun_out/prof_${model}_b${batch}
  rm -rf $d && mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/bench_cnn.py --model $model --batch $batch --steps 20 --warmup 5 --no-stock ${EXTRA} > $d/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $d 25 > $d/summary.txt
  head -30 $d/summary.txt
done
