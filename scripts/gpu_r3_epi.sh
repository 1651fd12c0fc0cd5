#!/bin/bash
# register-side bf16 epilogue: GEMM / engine tests, epilogue A/B micro-bench, step bench
set -o pipefail
O=gpurun_out/r3epi
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_q_gpu.py tests/test_kernels_gpu.py tests/test_head_fused_gpu.py tests/test_static_mlp_gpu.py > $O/test.txt 2>&1 || { echo "tests failed"; tail -60 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 200 python -u scripts/bench_epi_share.py > $O/epi.txt 2>&1 || { tail -20 $O/epi.txt; exit 1; }
cat $O/epi.txt
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-configs > $O/bench.txt 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json;a=json.load(open('$O/bench.txt'));print('step ms',a['ms_per_step'])"
