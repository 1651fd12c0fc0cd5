#!/bin/bash
# HIP graph runtime knobs: do captured branches run concurrently with packet capture off?
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
for envs in "X=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4"; do
  echo "== $envs" >> $O/graph_knobs.txt
  env $envs timeout -k 10 120 python -u scripts/graph_concurrency.py >> $O/graph_knobs.txt 2>/dev/null || exit 1
  env $envs timeout -k 10 120 python -u scripts/bench_cnn.py --model enhanced_cnn --batch 64 --graph --no-stock --steps 20 --warmup 5 >> $O/graph_knobs.txt 2>/dev/null || exit 1
  env $envs timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-configs 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'mlp_ms': d['ms_per_step']}))" >> $O/graph_knobs.txt || exit 1
done
cat $O/graph_knobs.txt
