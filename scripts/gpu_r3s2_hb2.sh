#!/bin/bash
# head_bwd grid: micro sweep (256 / 384 / 512) and mlp3 step A/B, LDNN_HEAD_BWD_WGS 768 vs 512 vs 384 (alternated)
set -o pipefail
O=gpurun_out/r3s2hb2
mkdir -p $O
for w in 256 384 512; do
  echo "== wgs $w"; LDNN_HEAD_BWD_WGS=$w timeout -k 10 120 python -u scripts/bench_head_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for rep in 1 2 3; do
  for w in 768 512 384; do
    LDNN_HEAD_BWD_WGS=$w timeout -k 10 200 python -u bench.py --no-configs --steps 50 --warmup 10 > $O/w${w}_$rep.txt 2>&1 || { tail -30 $O/w${w}_$rep.txt; exit 1; }
    echo "wgs $w rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/w${w}_$rep.txt)"
  done
done
