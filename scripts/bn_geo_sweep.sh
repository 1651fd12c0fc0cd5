#!/bin/bash
# BN reduce geometry sweep (LDNN_BN_RED_BLOCKS x LDNN_BN_RED_ROWS) on the CNN steps.
# Usage: bash scripts/bn_geo_sweep.sh "1024:8 512:32" "resnet18:64 enhanced_cnn:64"
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/cnn_bngeo.jsonl
for geo in $1; do
  for mb in $2; do
    m=${mb%%:*}; b=${mb##*:}
    LDNN_BN_RED_BLOCKS=${geo%%:*} LDNN_BN_RED_ROWS=${geo##*:} timeout -k 10 200 \
      python -u scripts/bench_cnn.py --model "$m" --batch "$b" --graph --no-stock > gpurun_out/bngeo_one.log 2>&1 || { cat gpurun_out/bngeo_one.log; exit 1; }
    echo "{\"geo\": \"$geo\", \"line\": $(tail -1 gpurun_out/bngeo_one.log)}" | tee -a $OUT
  done
done
