#!/bin/bash
# Conv tests, then same-box A/B of nontemporal slab reads (LDNN_SLAB_NT) on both CNNs.
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/slabnt; mkdir -p $d; rm -f gpurun_out/ab_cnn.jsonl
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -1 $d/tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_cnn.sh "enhanced_cnn:64 resnet18:64" "LDNN_SLAB_NT=0" "LDNN_SLAB_NT=1"
