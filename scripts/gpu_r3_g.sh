#!/bin/bash
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
for i in 1 2 3; do
  for f in "" "--no-head-mask"; do
    timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --no-configs $f > $O/b.txt 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/b.txt')); print(json.dumps({'flag': '$f', 'ms': d['ms_per_step']}))" | tee -a $O/head_mask_ab.jsonl
  done
done
