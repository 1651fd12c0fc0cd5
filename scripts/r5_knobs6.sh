set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_SPLIT_TARGET=512 LDNN_CONV_SPLIT_TARGET=768 LDNN_CONV_WGRAD_TARGET=768" bash scripts/gpu_run.sh r5knobs6 ab:enhanced_cnn:64,resnet18:64,resnet18:256 || exit 4
echo done
