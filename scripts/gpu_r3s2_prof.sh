#!/bin/bash
# kernel traces + per-step timelines of the current tree: ResNet-18 b64 / b256, EnhancedCNN b64
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
d=gpurun_out/r3s2prof; mkdir -p $d
for spec in resnet18:64 enhanced_cnn:64 resnet18:256; do
  m=${spec%%:*}; b=${spec##*:}; p=$d/${m}_b$b
  mkdir -p $p
  steps=20; [ $b = 256 ] && steps=8
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps $steps --warmup 3 --no-stock --graph > $p/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $p $((steps + 3)) > $p/summary.txt
  python3 scripts/step_timeline.py $p > $p/timeline.txt
  tail -1 $p/timeline.txt
done
