#!/bin/bash
# Conv numerics tests, then a same-box A/B of the row-coalesced conv epilogues (knob in the A/B line).
cd "${GRAFT_REPO_ROOT:-.}"; d=gpurun_out/halfrows; mkdir -p $d; rm -f gpurun_out/ab_cnn.jsonl
LDNN_CONV_BF16_ROWS=2 timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_layers_gpu.py -x -q --timeout 120 --timeout-method thread > $d/tests.log 2>&1
rc=$?; tail -2 $d/tests.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab_cnn.sh "enhanced_cnn:64 resnet18:64" "LDNN_CONV_BF16_ROWS=1" "LDNN_CONV_BF16_ROWS=2"
