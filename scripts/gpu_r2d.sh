#!/bin/bash
# GPU suite + CNN benches (ldnn vs stock) + kernel timelines of the ResNet-18 / EnhancedCNN b64 steps.
# OUT=gpurun_out/<name> (default r2d).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
d=${OUT:-gpurun_out/r2d}; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gputests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $d/gputests.log; [ $rc -le 1 ] || exit $rc
for spec in resnet18:64:sgd enhanced_cnn:64:sgd enhanced_cnn:64:adam lenet5:256:sgd; do
  IFS=: read m b o <<< "$spec"
  timeout -k 10 200 python scripts/bench_cnn.py --model $m --batch $b --graph --optimizer $o > $d/cnn_${m}_b${b}_$o.log 2>&1 || exit $?
  tail -1 $d/cnn_${m}_b${b}_$o.log
done
for spec in resnet18:64 enhanced_cnn:64; do
  m=${spec%%:*}; b=${spec##*:}; p=$d/prof_${m}_b$b
  mkdir -p $p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 20 --warmup 5 --no-stock --graph > $p/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $p 40 > $p/summary.txt
  python3 scripts/step_timeline.py $p > $p/timeline.txt
  tail -1 $p/timeline.txt
done
