#!/bin/bash
# fused head forward: new tests, engine tests, A/B bench (fused vs separate head), kernel profile
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head_fused_gpu.py tests/test_static_mlp_gpu.py > $O/test.txt 2>&1 || { echo "tests failed"; tail -60 $O/test.txt; exit 1; }
timeout -k 10 120 python -u scripts/bench_head_epi.py > $O/epi.txt 2>&1 || { tail -20 $O/epi.txt; exit 1; }
cat $O/epi.txt
tail -2 $O/test.txt
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-configs > $O/bench_fused_$i.txt 2> $O/bench_fused_$i.err || { tail -30 $O/bench_fused_$i.err; exit 1; }
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 --no-configs --no-fuse-head-fwd > $O/bench_sep_$i.txt 2> $O/bench_sep_$i.err || { tail -30 $O/bench_sep_$i.err; exit 1; }
python -c "import json;a=json.load(open('$O/bench_fused_$i.txt'));b=json.load(open('$O/bench_sep_$i.txt'));print('fused',a['ms_per_step'],'sep',b['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o mlp -- python3 -u bench.py --steps 30 --warmup 5 --no-configs > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
