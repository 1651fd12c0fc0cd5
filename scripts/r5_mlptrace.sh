set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_run.sh r5mlptr probetrace:mlp3@16384@8@1@sgd || exit 4
echo done
