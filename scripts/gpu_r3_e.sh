#!/bin/bash
# headline step kernel profile + bench timing (with CNN configs) + wall time of the whole bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/mlp -o run -- python3 bench.py --steps 20 --warmup 5 --no-configs > $O/mlp.log 2>&1 || { tail -20 $O/mlp.log; exit 1; }
python3 scripts/kernel_summary.py $O/mlp 25 > $O/mlp_summary.txt
head -22 $O/mlp_summary.txt
python3 scripts/step_timeline.py $O/mlp > $O/mlp_timeline.txt
start=$(date +%s.%N)
timeout -k 10 400 python3 bench.py > $O/bench_default.txt 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
end=$(date +%s.%N)
echo "bench.py default wall: $(echo "$end - $start" | bc) s"
cat $O/bench_default.txt
