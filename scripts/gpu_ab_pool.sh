#!/bin/bash
# BN / pool numerics tests, then a same-box A/B of the LDS-tiled 3x3/2 max pool on ResNet-18 b64.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/pool; mkdir -p $d; rm -f gpurun_out/ab_cnn.jsonl
timeout -k 10 400 python -u -m pytest tests/test_bn_pool_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -2 $d/tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_cnn.sh "resnet18:64" "LDNN_POOL_LDS=0" "LDNN_POOL_LDS=1"
