#!/bin/bash
# round-3 (session 2) re-check on the restored tree: GPU suite + default bench
set -o pipefail
O=gpurun_out/r3s2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/test_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -60 $O/test_gpu.txt; exit 1; }
tail -3 $O/test_gpu.txt
timeout -k 10 300 python -u bench.py > $O/bench1.txt 2> $O/bench1.err || { echo "bench failed"; tail -30 $O/bench1.err; exit 1; }
cat $O/bench1.txt
