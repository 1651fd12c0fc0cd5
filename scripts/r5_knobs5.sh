set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_BN_BWD=0 LDNN_CONV_WGRAD_XCD=0 LDNN_CONV_COMBINE_LAST=0 LDNN_CONV_WGRAD_TARGET=512" bash scripts/gpu_run.sh r5knobs5 ab:enhanced_cnn:64,resnet18:64 || exit 4
echo done
