#!/bin/bash
# Round-2 full check: GPU test suite, smoke(), headline bench, CNN step benches.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?
echo "gpu tests rc=$rc" >> gpurun_out/gpu_all.log
tail -3 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 200 python -u bench.py > gpurun_out/bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_final.log
for m in "enhanced_cnn 64" "resnet18 64"; do set -- $m
  timeout -k 10 200 python -u scripts/bench_cnn.py --model $1 --batch $2 --graph > gpurun_out/cnn_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/cnn_$1.log
done
