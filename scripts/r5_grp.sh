set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
AB_ENVS="X=0 LDNN_BN_GRP_ROWS=262144 LDNN_BN_GRP_ROWS=16384" bash scripts/gpu_run.sh r5grp ab:resnet18:256,resnet18:64 prof:resnet18@256 || exit 4
echo done
