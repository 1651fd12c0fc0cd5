set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_run.sh r5probe2 probe:enhanced_cnn@64@1@1@adam probe:resnet18@64@1@1@sgd || exit 4
echo done
