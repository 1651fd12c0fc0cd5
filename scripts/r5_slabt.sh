set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_SLAB_TILES=96 LDNN_CONV_SLAB_TILES=160" bash scripts/gpu_run.sh r5slabt ab:enhanced_cnn:64,resnet18:64 || exit 4
echo done
