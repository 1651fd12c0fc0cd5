#!/bin/bash
# ResNet-18 b64 / EnhancedCNN b64 graphed step: kernel summary + one step's timeline with idle gaps
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
CNN="resnet18:64,enhanced_cnn:64" EXTRA="--graph" bash scripts/prof_cnn.sh || exit 1
for d in gpurun_out/prof_resnet18_b64 gpurun_out/prof_enhanced_cnn_b64; do
  python3 scripts/step_timeline.py $d > $d/timeline.txt && tail -1 $d/timeline.txt
done
