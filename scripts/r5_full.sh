set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_run.sh ${1:-r5full} suite smoke bench benchgloo || exit 4
echo done
