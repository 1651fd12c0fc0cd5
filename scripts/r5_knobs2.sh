set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_WGRAD_MIN_KT=16 LDNN_CONV_WGRAD_MIN_KT=24 LDNN_CONV_WGRAD_MIN_KT=16,LDNN_CONV_SLAB_TARGET=256" bash scripts/gpu_run.sh r5knobs2 ab:enhanced_cnn:64,resnet18:64,resnet18:256 || exit 4
echo done
