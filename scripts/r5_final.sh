set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=${1:-r5fin}
bash scripts/gpu_run.sh $O suite smoke bench benchgloo profmlp prof:resnet18@64 prof:resnet18@256 prof:enhanced_cnn@64 prof:lenet5@256 || exit 4
echo done
