#!/bin/bash
# PMC of the ResNet-18 b256 step (config #5), then the gradients experiment matrix
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 bash scripts/pmc_cnn.sh resnet18 256 > /dev/null 2>&1 || { echo pmc failed; exit 1; }
cp gpurun_out/pmc_resnet18/summary.txt gpurun_out/pmc_rn256_summary.txt
head -40 gpurun_out/pmc_rn256_summary.txt
bash scripts/gpu_r3_matrix.sh
