#!/bin/bash
# 12-wave ring wgrad (2 K-tiles in flight): conv tests, per-shape micro (ring 0 / 2), step A/B (0 / 1 / 2)
set -o pipefail
O=gpurun_out/r3s2ring3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for b in 64 256; do
  for x in 0 2; do
    LDNN_CONV_WGRAD_RING=$x timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/micro_r${x}_b$b.txt 2>&1 || { tail -20 $O/micro_r${x}_b$b.txt; exit 1; }
    echo "== ring $x b $b"; grep -v amdgpu.ids $O/micro_r${x}_b$b.txt | grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*\|"wgrad_tf": [0-9.]*' | paste - - -
  done
done
for x in 0 2; do
LDNN_CONV_WGRAD_RING=$x timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/ecnn_r$x.txt 2>&1 && echo "== ecnn ring $x" && grep -o '"shape": "[^"]*"\|"wgrad_us": [0-9.]*' $O/ecnn_r$x.txt | paste - -
done
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64 resnet18:256" "LDNN_CONV_WGRAD_RING=0" "LDNN_CONV_WGRAD_RING=1" "LDNN_CONV_WGRAD_RING=2" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
