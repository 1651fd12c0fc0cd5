#!/bin/bash
# double-buffered halo conv (128x128 tiles): conv + layer GPU tests, per-shape micro A/B
# (LDNN_CONV_HALO=3 = previous default, 1 = new default), step A/B on ResNet-18 b64 / b256
# and EnhancedCNN b64
set -o pipefail
O=gpurun_out/r3s2halo
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -60 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for b in 64 256; do
  for h in 3 1; do
    LDNN_CONV_HALO=$h timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --batch $b --iters 20 > $O/micro_h${h}_b$b.txt 2>&1 || { tail -20 $O/micro_h${h}_b$b.txt; exit 1; }
    echo "== halo $h b $b"; grep -v amdgpu.ids $O/micro_h${h}_b$b.txt
  done
done
LDNN_CONV_HALO=1 timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/micro_ecnn_h1.txt 2>&1 && grep -v amdgpu.ids $O/micro_ecnn_h1.txt
LDNN_CONV_HALO=3 timeout -k 10 120 python -u scripts/conv_micro.py --no-stock --model enhanced_cnn --batch 64 --iters 20 > $O/micro_ecnn_h3.txt 2>&1 && grep -v amdgpu.ids $O/micro_ecnn_h3.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64 resnet18:256" "LDNN_CONV_HALO=3" "LDNN_CONV_HALO=1" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
