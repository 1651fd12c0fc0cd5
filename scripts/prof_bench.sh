#!/bin/bash
# Kernel-trace profile of the headline bench (1 GPU); summary -> gpurun_out/prof_bench/summary.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/prof_bench && mkdir -p gpurun_out/prof_bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 50 --warmup 10 "$@" > gpurun_out/prof_bench/bench.log 2>&1 || exit $?
python3 scripts/kernel_summary.py gpurun_out/prof_bench 60 > gpurun_out/prof_bench/summary.txt
