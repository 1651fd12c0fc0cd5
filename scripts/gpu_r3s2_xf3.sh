#!/bin/bash
# fill knockouts of the 128x128 gather kernels: LDNN_CONV_XF 0 (full), 8 (no B fill), 16 (no A fill), ResNet-18 shapes b64 / b256
set -o pipefail
O=gpurun_out/r3s2xf3
mkdir -p $O
for b in 64 256; do
  for xf in 0 8 16; do
    LDNN_CONV_XF=$xf timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/xf${xf}_b$b.txt 2>&1 || { tail -20 $O/xf${xf}_b$b.txt; exit 1; }
    echo "== xf $xf b $b"; grep -v amdgpu.ids $O/xf${xf}_b$b.txt | cut -d, -f1-4
  done
done
