#!/bin/bash
# double-buffered halo at 78 KiB (W <= 27): per-shape micro A/B vs the gather kernel
set -o pipefail
O=gpurun_out/r3s2halo2
mkdir -p $O
for b in 64 256; do
  for h in 3 1; do
    LDNN_CONV_HALO=$h timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/micro_h${h}_b$b.txt 2>&1 || { tail -20 $O/micro_h${h}_b$b.txt; exit 1; }
    echo "== halo $h b $b"; grep -v amdgpu.ids $O/micro_h${h}_b$b.txt | cut -c1-130
  done
done
for h in 3 1; do
LDNN_CONV_HALO=$h timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/micro_ecnn_h$h.txt 2>&1 && grep -v amdgpu.ids $O/micro_ecnn_h$h.txt | cut -c1-130
done
