#!/bin/bash
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_static_mlp_gpu.py > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-configs > $O/bench_$i.txt 2>/dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/bench_$i.txt')); print(d['ms_per_step'], d['gemm_kernels']['dgrad2'])"
done
