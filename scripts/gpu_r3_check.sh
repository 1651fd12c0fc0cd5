#!/bin/bash
# round-3 GPU check: Q4 GEMM tests + A/B, full GPU suite, headline bench (+ CNN configs), overlap probes, gloo rehearsal
set -o pipefail
mkdir -p gpurun_out/r3
O=gpurun_out/r3
export HSA_ENABLE_IPC_MODE_LEGACY=0




timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphed_dp_gpu.py tests/test_static_mlp_gpu.py tests/test_ipc_gpu.py > $O/test_dp.txt 2>&1 || { echo "dp tests failed"; tail -60 $O/test_dp.txt; exit 1; }
tail -2 $O/test_dp.txt
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/test_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -60 $O/test_gpu.txt; exit 1; }
tail -3 $O/test_gpu.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench1.txt 2> $O/bench1.err || { echo "bench failed"; tail -30 $O/bench1.err; exit 1; }
cat $O/bench1.txt
timeout -k 10 150 python -u scripts/overlap_probe.py --model resnet18 --batch 64 > $O/overlap_rn64.txt 2>&1 || { tail -30 $O/overlap_rn64.txt; exit 1; }
cat $O/overlap_rn64.txt
timeout -k 10 150 python -u scripts/overlap_probe.py --model enhanced_cnn --batch 64 > $O/overlap_ecnn64.txt 2>&1 || { tail -30 $O/overlap_ecnn64.txt; exit 1; }
cat $O/overlap_ecnn64.txt
timeout -k 10 200 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --batch 4096 > $O/bench2_gloo.txt 2> $O/bench2_gloo.err || { echo "gloo bench failed"; tail -30 $O/bench2_gloo.err; exit 1; }
cat $O/bench2_gloo.txt
