#!/bin/bash
# smoke(), the headline bench and the CNN benches on the final tree (no test suite).
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/final_check; mkdir -p $d
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.log 2>&1 || exit $?
tail -1 $d/smoke.log
timeout -k 10 200 python bench.py > $d/bench.log 2>&1 || exit $?
tail -1 $d/bench.log
NOTESTS=1 OUT=$d MODELS="resnet18:64 enhanced_cnn:64" bash scripts/gpu_quick.sh
