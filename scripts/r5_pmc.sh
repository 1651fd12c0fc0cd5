set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_run.sh r5pmc pmc:resnet18_b256@resnet18@256 pmc:enhanced_cnn_b64@enhanced_cnn@64 pmc:mlp3@mlp3@0 || exit 4
echo done
