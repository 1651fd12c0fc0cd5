#!/bin/bash
# full GPU suite + default bench (with the CNN configs) + smoke on the current tree
set -o pipefail
O=gpurun_out/r3s2full
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/test_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -60 $O/test_gpu.txt; exit 1; }
tail -2 $O/test_gpu.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench1.txt 2> $O/bench1.err || { echo "bench failed"; tail -30 $O/bench1.err; exit 1; }
cat $O/bench1.txt
