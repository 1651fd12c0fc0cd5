#!/bin/bash
# Conv tests, then same-box A/B of nontemporal BN apply loads (LDNN_BN_NT) on both CNNs.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/bnnt; mkdir -p $d; rm -f gpurun_out/ab_cnn.jsonl
timeout -k 10 400 python -u -m pytest tests/test_bn_pool_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -1 $d/tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_cnn.sh "enhanced_cnn:64 resnet18:64" "LDNN_BN_NT=0" "LDNN_BN_NT=1"
