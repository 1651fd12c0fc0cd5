#!/bin/bash
# BN statistics in the conv slab epilogue: tests + step A/B (LDNN_CONV_SLAB_BN 0 / 1)
set -o pipefail
O=gpurun_out/r3s2slabbn
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_layers_gpu.py tests/test_conv_gpu.py tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "enhanced_cnn:64 resnet18:64 enhanced_cnn:256" "LDNN_CONV_SLAB_BN=0" "LDNN_CONV_SLAB_BN=1" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
