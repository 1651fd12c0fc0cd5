set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_CONV_SLAB=0" MLP_AB_ENVS="X=0 LDNN_HEAD_BWD_WGS=256 LDNN_HEAD_BWD_WGS=512" \
  bash scripts/gpu_run.sh r5ab2 ab:enhanced_cnn:64 mlpab || exit 4
echo done
