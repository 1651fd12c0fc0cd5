#!/bin/bash
# overlap probes with the small-last-bucket plan + conv_q big tiles A/B at batch 256
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphed_dp_gpu.py > $O/test_dp.txt 2>&1 || { tail -40 $O/test_dp.txt; exit 1; }
tail -1 $O/test_dp.txt
for spec in "resnet18 64" "resnet18 256" "enhanced_cnn 64"; do
  set -- $spec
  timeout -k 10 150 python -u scripts/overlap_probe.py --model $1 --batch $2 --blocks 16 --reps 4 >> $O/overlap.jsonl 2>$O/overlap.err || { tail -20 $O/overlap.err; exit 1; }
done
cat $O/overlap.jsonl
for rep in 1 2; do
  for q in 0 1; do
    for spec in "resnet18 256" "enhanced_cnn 256" "resnet18 64"; do
      set -- $spec
      LDNN_CONV_Q=$q timeout -k 10 120 python -u scripts/bench_cnn.py --model $1 --batch $2 --graph --no-stock --steps 10 --warmup 3 | sed "s/^/{\"conv_q\": $q, /;s/{\"conv_q\": $q, {/{\"conv_q\": $q, /" >> $O/convq_ab.jsonl || exit 1
    done
  done
done
cat $O/convq_ab.jsonl
