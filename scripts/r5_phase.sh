set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_run.sh r5phase phase:enhanced_cnn || exit 4
echo done
