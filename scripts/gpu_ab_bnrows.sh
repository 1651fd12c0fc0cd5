#!/bin/bash
# Same-box A/B of the BN reduce geometry for small-M layers (rows per row lane, accumulator copies).
cd "${GRAFT_REPO_ROOT:-.}"; rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "enhanced_cnn:64 resnet18:64" "LDNN_BN_RED_ROWS=8" "LDNN_BN_RED_ROWS=16" "LDNN_BN_RED_ROWS=32"
