#!/bin/bash
# the reference's default aggregation (gradients) over the six variants, full 20 x 5 schedule
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
AGG=gradients TAG=_grad bash scripts/experiment_matrix.sh || exit 1
python3 scripts/matrix_report.py gpurun_out/matrix_grad gpurun_out/matrix_grad/report || exit 1
cat gpurun_out/matrix_grad/summary.txt
