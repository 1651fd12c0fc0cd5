#!/bin/bash
# One GPU call: numerics tests, then (unless a step crashed or timed out) the benches.
# A test FAILURE (exit 1) still lets the benches run; a fault / abort / timeout ends the call.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 400 python -m pytest ${TESTS:-tests/test_kernels_gpu.py tests/test_static_mlp_gpu.py} -q -m gpu -x \
  > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; ok $rc || exit $rc
for step in ${STEPS:-gemm small bench}; do
  case $step in
    gemm) timeout -k 10 240 python scripts/bench_gemm.py > gpurun_out/gemm.log 2>&1 ;;
    small) timeout -k 10 120 python scripts/bench_small.py > gpurun_out/small.log 2>&1 ;;
    epi) timeout -k 10 120 python scripts/bench_epi.py > gpurun_out/epi.log 2>&1 ;;
    bench) timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1 ;;
    cnn) timeout -k 10 400 python scripts/bench_cnn.py > gpurun_out/cnn.log 2>&1 ;;
  esac
  rc=$?; echo "$step rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
