#!/bin/bash
# Session check on a fresh box: GPU suite, smoke, headline bench, and kernel-trace timelines of the
# ResNet-18 / EnhancedCNN b64 graphed steps.  Results -> gpurun_out/r2c/.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
d=gpurun_out/r2c; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gputests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $d/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > $d/bench.log 2>&1 || exit $?
tail -1 $d/bench.log
for spec in resnet18:64 enhanced_cnn:64; do
  m=${spec%%:*}; b=${spec##*:}; p=$d/prof_${m}_b$b
  mkdir -p $p
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model $m --batch $b --steps 20 --warmup 5 --no-stock --graph > $p/bench.log 2>&1 || exit $?
  python3 scripts/kernel_summary.py $p 40 > $p/summary.txt
  python3 scripts/step_timeline.py $p > $p/timeline.txt
  tail -1 $p/bench.log
done
