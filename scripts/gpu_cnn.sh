#!/bin/bash
# One GPU call for the conv path: numerics tests, then CNN throughput (ldnn vs stock PyTorch).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_conv_gpu.py tests/test_kernels_gpu.py tests/test_layers_gpu.py} \
  -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/cnn.jsonl
for spec in ${CNN:-"enhanced_cnn 256" "enhanced_cnn_small 256" "resnet18 64" "lenet5 1024"}; do
  set -- $spec
  timeout -k 10 300 python scripts/bench_cnn.py --model $1 --batch $2 ${EXTRA} >> gpurun_out/cnn.jsonl 2>> gpurun_out/cnn.err
  rc=$?; echo "cnn $1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cat gpurun_out/cnn.jsonl
