#!/bin/bash
# kernel traces + step timelines of the current tree (ResNet-18 b256, EnhancedCNN b64, LeNet-5 b256)
# and a PMC table of ResNet-18 b256 (MFMA busy, LDS conflicts, L2 hit per kernel)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
d=gpurun_out/r3s2prof2; mkdir -p $d
for spec in resnet18:256 enhanced_cnn:64 lenet5:256; do
  m=${spec%%:*}; b=${spec##*:}; p=$d/${m}_b$b
  mkdir -p $p
  steps=20; [ $m = resnet18 ] && steps=8
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps $steps --warmup 3 --no-stock --graph > $p/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $p $((steps + 3)) > $p/summary.txt
  python3 scripts/step_timeline.py $p > $p/timeline.txt
  tail -1 $p/timeline.txt
done
bash scripts/pmc_step.sh rn256 python3 scripts/bench_cnn.py --model resnet18 --batch 256 --steps 3 --warmup 2 --no-stock > $d/pmc_rn256.txt 2>&1 || { tail -20 $d/pmc_rn256.txt; exit 1; }
head -25 $d/pmc_rn256.txt
