#!/bin/bash
# Kernel-trace summaries of the final tree: headline bench and the ResNet-18 / EnhancedCNN b64 graphed steps.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
d=gpurun_out/final_prof; mkdir -p $d
p=$d/mlp3; mkdir -p $p
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 bench.py --steps 20 --warmup 5 > $p/bench.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $p 25 > $p/summary.txt; head -3 $p/summary.txt
for spec in resnet18:64 enhanced_cnn:64; do
  m=${spec%%:*}; b=${spec##*:}; p=$d/${m}_b$b
  mkdir -p $p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 20 --warmup 5 --no-stock --graph > $p/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $p 40 > $p/summary.txt
  python3 scripts/step_timeline.py $p > $p/timeline.txt
  tail -1 $p/timeline.txt
done
