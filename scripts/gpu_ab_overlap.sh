#!/bin/bash
# Same-box A/B: optimizer overlapped with the backward (GraphedStep) off / on / narrow side-stream grids.
cd "${GRAFT_REPO_ROOT:-.}"; rm -f gpurun_out/ab_cnn.jsonl
bash scripts/ab_cnn.sh "enhanced_cnn:64" "LDNN_OVERLAP_OPT=0" "LDNN_OVERLAP_OPT_BLOCKS=32" "LDNN_OVERLAP_OPT_BLOCKS=128" "LDNN_OVERLAP_OPT_BLOCKS=32 LDNN_OVERLAP_OPT_ELEMS=16777216"
