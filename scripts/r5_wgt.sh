set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5wgt; mkdir -p $O
for rep in 1 2 3; do
AB_ENVS="X=0 LDNN_CONV_WGRAD_TARGET=512" bash scripts/gpu_run.sh r5wgt ab:enhanced_cnn:64,resnet18:64,resnet18:256 || exit 4
done
echo done
