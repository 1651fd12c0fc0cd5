# bucket-size sweep of the DP overlap probe (EnhancedCNN Adam sharded, ResNet-18 SGD)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for mb in ${MBS:-8 16 24 32}; do
  PROBE_ARGS="--bucket-mb $mb" bash scripts/gpu_run.sh r5bucket probe:enhanced_cnn@64@1@1@adam probe:resnet18@64@1@1@sgd || exit 4
done
echo done
