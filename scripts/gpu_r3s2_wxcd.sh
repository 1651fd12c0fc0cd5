#!/bin/bash
# wgrad split-K slices placed per XCD (LDNN_CONV_WGRAD_XCD): tests, per-shape micro, DMA-only knockout, step A/B
set -o pipefail
O=gpurun_out/r3s2wxcd
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -60 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for b in 64 256; do
  for x in 0 1; do
    LDNN_CONV_WGRAD_XCD=$x timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/micro_x${x}_b$b.txt 2>&1 || { tail -20 $O/micro_x${x}_b$b.txt; exit 1; }
    echo "== wgrad_xcd $x b $b"; grep -v amdgpu.ids $O/micro_x${x}_b$b.txt | grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*' | paste - -
  done
  LDNN_CONV_XF=4 LDNN_CONV_WGRAD_XCD=1 timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/xf4_x1_b$b.txt 2>&1 || exit 1
  echo "== DMA only, wgrad_xcd 1, b $b"; grep -v amdgpu.ids $O/xf4_x1_b$b.txt | grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*' | paste - -
done
timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/ecnn_x1.txt 2>&1 && grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*' $O/ecnn_x1.txt | paste - -
LDNN_CONV_WGRAD_XCD=0 timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/ecnn_x0.txt 2>&1 && grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*' $O/ecnn_x0.txt | paste - -
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64 resnet18:256" "LDNN_CONV_WGRAD_XCD=0" "LDNN_CONV_WGRAD_XCD=1" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
