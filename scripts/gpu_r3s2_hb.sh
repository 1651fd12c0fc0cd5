#!/bin/bash
# head_bwd grid knob sweep at the headline shape (+ a plain copy of the same bytes)
set -o pipefail
for w in 512 768 1024 1536 2048; do
  echo "== wgs $w"; LDNN_HEAD_BWD_WGS=$w timeout -k 10 120 python -u scripts/bench_head_bwd.py 2>&1 | grep -v amdgpu.ids || exit 1
done
