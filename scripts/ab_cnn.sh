#!/bin/bash
# Same-box A/B of env knobs on the CNN step, alternated (A B A B ...) to cancel drift.
# Usage: bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64" "X=1" "LDNN_FUSE_BN_STATS=1" "A=1,B=2" ...
# (a comma joins several variables into one setting)
set -o pipefail
mkdir -p gpurun_out
models=$1; shift
for rep in 1 2; do
  for mb in $models; do
    m=${mb%%:*}; b=${mb##*:}
    for e in "$@"; do
      r=$(env ${e//,/ } timeout -k 10 200 python -u scripts/bench_cnn.py --model "$m" --batch "$b" --graph --no-stock 2>&1 | tail -1) || { echo "FAIL $e $m: $r"; exit 1; }
      echo "{\"rep\": $rep, \"env\": \"$e\", \"line\": $r}" | tee -a gpurun_out/ab_cnn.jsonl
    done
  done
done
