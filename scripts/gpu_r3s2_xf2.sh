#!/bin/bash
# conv knockouts (LDNN_CONV_XF 0 / 1 / 4) on the 128x128 fwd / dgrad / wgrad and narrow wgrad kernels
set -o pipefail
O=gpurun_out/r3s2xf2
mkdir -p $O
for b in 64 256; do
  for xf in 0 1 4; do
    LDNN_CONV_XF=$xf timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/xf${xf}_b$b.txt 2>&1 || { tail -20 $O/xf${xf}_b$b.txt; exit 1; }
    echo "== xf $xf b $b"; grep -v amdgpu.ids $O/xf${xf}_b$b.txt
  done
done
