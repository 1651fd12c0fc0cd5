#!/bin/bash
# residual tail with a BN on both branches in one pass (bn_dual_*): tests, step A/B (LDNN_BN_DUAL 0 / 1)
set -o pipefail
O=gpurun_out/r3s2dual
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py tests/test_layers_gpu.py > $O/tests.txt 2>&1 || { echo "tests failed"; tail -80 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "resnet18:64 enhanced_cnn:64 resnet18:256" "LDNN_BN_DUAL=0" "LDNN_BN_DUAL=1" > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
