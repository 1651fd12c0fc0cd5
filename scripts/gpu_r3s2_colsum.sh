#!/bin/bash
# column sums with a channel-aware block geometry + fused act/colsum in the Linear / conv backward:
# kernel + layer tests, CNN step times (LeNet-5 b256, ResNet-18 b64, EnhancedCNN b64), LeNet kernel trace
set -o pipefail
O=gpurun_out/r3s2colsum
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for spec in lenet5:256 resnet18:64 enhanced_cnn:64; do
  m=${spec%%:*}; b=${spec##*:}
  timeout -k 10 300 python3 scripts/bench_cnn.py --model $m --batch $b --steps 50 --warmup 10 --no-stock --graph > $O/bench_${m}_$b.txt 2>&1 || { tail -20 $O/bench_${m}_$b.txt; exit 1; }
  tail -1 $O/bench_${m}_$b.txt
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
p=$O/lenet5_b256; mkdir -p $p
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $p -o run -- python3 scripts/bench_cnn.py --model lenet5 --batch 256 --steps 20 --warmup 3 --no-stock --graph > $p/bench.log 2>&1 || exit $?
python3 scripts/step_timeline.py $p > $p/timeline.txt
cat $p/timeline.txt
