#!/bin/bash
# One GPU call: the full GPU suite, smoke(), the headline bench, and the CNN benches
# (every BASELINE CNN config, stock PyTorch alongside).  Results -> gpurun_out/refresh/.
cd "${GRAFT_REPO_ROOT:-.}"
d=gpurun_out/refresh; mkdir -p $d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $d/gputests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --compare-stock > $d/bench.log 2>&1 || exit $?
for mb in lenet5:256 resnet18:64 enhanced_cnn:64 enhanced_cnn:256; do
  m=${mb%%:*}; b=${mb##*:}
  timeout -k 10 200 python scripts/bench_cnn.py --model $m --batch $b --graph > $d/cnn_${m}_b$b.log 2>&1 || exit $?
done
timeout -k 10 200 python scripts/bench_cnn.py --model enhanced_cnn --batch 64 --graph --optimizer adam > $d/cnn_enhanced_cnn_b64_adam.log 2>&1 || exit $?
