set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_NS=4 LDNN_CONV_NS=4,LDNN_CONV_SLAB_TARGET=256 LDNN_CONV_NS=3" bash scripts/gpu_run.sh r5ns ab:enhanced_cnn:64 || exit 4
echo done
