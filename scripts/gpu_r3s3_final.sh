#!/bin/bash
# round-3 final check: full GPU suite, smoke, default bench (+ CNN configs), headline kernel profile, 4-rank gloo rehearsal
set -o pipefail
O=gpurun_out/r3s3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/test_gpu.txt 2>&1 || { echo "gpu tests failed"; tail -60 $O/test_gpu.txt; exit 1; }
tail -3 $O/test_gpu.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -30 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench_default.txt 2> $O/bench_default.err || { echo "bench failed"; tail -30 $O/bench_default.err; exit 1; }
cat $O/bench_default.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o mlp -- python3 -u bench.py --steps 30 --warmup 5 --no-configs > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
timeout -k 10 250 python -u bench.py --gpus 4 --backend gloo --steps 5 --warmup 2 --batch 4096 --no-configs > $O/bench4_gloo.txt 2> $O/bench4_gloo.err || { echo "gloo bench failed"; tail -30 $O/bench4_gloo.err; exit 1; }
cat $O/bench4_gloo.txt
