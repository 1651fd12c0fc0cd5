#!/bin/bash
# BN statistics over up to 64 accumulator copies: GPU tests, conv-epilogue probe and step A/B vs 8 copies
set -o pipefail
O=gpurun_out/r3s2bncop
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_layers_gpu.py tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -60 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for c in 8 64; do
  for b in 64 256; do
    LDNN_BN_MAX_COPIES=$c timeout -k 10 120 python -u scripts/conv_bn_probe.py --batch $b --iters 20 > $O/probe_c${c}_b$b.txt 2>&1 || { tail -20 $O/probe_c${c}_b$b.txt; exit 1; }
    echo "== copies $c b $b"; grep -v amdgpu.ids $O/probe_c${c}_b$b.txt
  done
done
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64 resnet18:256" "LDNN_BN_MAX_COPIES=8" "LDNN_BN_MAX_COPIES=64" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
