#!/bin/bash
# overlap probes with the RCCL-footprint stand-in + ResNet-18 b256 step timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphed_dp_gpu.py > $O/test_dp.txt 2>&1 || { tail -40 $O/test_dp.txt; exit 1; }
tail -1 $O/test_dp.txt
for spec in "resnet18 64 16 4" "enhanced_cnn 64 16 4" "resnet18 256 16 4" "resnet18 64 32 8"; do
  set -- $spec
  timeout -k 10 150 python -u scripts/overlap_probe.py --model $1 --batch $2 --blocks $3 --reps $4 >> $O/overlap.jsonl 2>$O/overlap.err || { tail -20 $O/overlap.err; exit 1; }
done
cat $O/overlap.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/ovtrace -o ov -- python3 scripts/overlap_probe.py --model resnet18 --batch 64 --steps 5 > $O/ovtrace.log 2>&1 || { tail -20 $O/ovtrace.log; exit 1; }
python3 scripts/trace_overlap.py $O/ovtrace/ov_kernel_trace.csv
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/rn256 -o run -- python3 scripts/bench_cnn.py --model resnet18 --batch 256 --steps 10 --warmup 3 --no-stock --graph > $O/rn256.log 2>&1 || { tail -20 $O/rn256.log; exit 1; }
python3 scripts/kernel_summary.py $O/rn256 13 > $O/rn256_summary.txt
python3 scripts/step_timeline.py $O/rn256 > $O/rn256_timeline.txt
head -25 $O/rn256_summary.txt
tail -3 $O/rn256.log
