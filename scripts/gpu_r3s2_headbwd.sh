#!/bin/bash
# fused MFMA head backward: tests, mlp3 A/B (fused vs stream + wgrad), kernel trace
set -o pipefail
O=gpurun_out/r3s2hb
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head_fused_gpu.py tests/test_static_mlp_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -60 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 120 python -u scripts/bench_head_bwd.py > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
grep -v amdgpu.ids $O/micro.txt
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-configs --steps 50 --warmup 10 > $O/fused_$rep.txt 2>&1 || { tail -30 $O/fused_$rep.txt; exit 1; }
  echo "fused $(grep -o '"ms_per_step": [0-9.]*' $O/fused_$rep.txt)"
  timeout -k 10 200 python -u bench.py --no-configs --steps 50 --warmup 10 --no-fuse-head-bwd > $O/sep_$rep.txt 2>&1 || { tail -30 $O/sep_$rep.txt; exit 1; }
  echo "separate $(grep -o '"ms_per_step": [0-9.]*' $O/sep_$rep.txt)"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mlp -- python3 bench.py --no-configs --steps 30 --warmup 5 > $O/prof.txt 2>&1 || { tail -30 $O/prof.txt; exit 1; }
python3 scripts/kernel_summary.py $O/prof 95 > $O/prof_summary.txt; head -12 $O/prof_summary.txt | cut -c1-150
