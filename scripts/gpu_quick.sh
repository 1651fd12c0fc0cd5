#!/bin/bash
# GPU suite, then ldnn-only CNN bench lines (MODELS="resnet18:64 ...", default ResNet-18 + EnhancedCNN b64).
cd "${GRAFT_REPO_ROOT:-.}"; d=${OUT:-gpurun_out/quick}; mkdir -p $d
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gputests.log 2>&1
  rc=$?; tail -2 $d/gputests.log; [ $rc -le 1 ] || exit $rc; [ $rc -eq 0 ] || exit 1
fi
for spec in ${MODELS:-resnet18:64 enhanced_cnn:64}; do
  m=${spec%%:*}; b=${spec##*:}
  timeout -k 10 200 python scripts/bench_cnn.py --model $m --batch $b --graph --no-stock > $d/cnn_${m}_b$b.log 2>&1 || exit $?
  tail -1 $d/cnn_${m}_b$b.log
done
