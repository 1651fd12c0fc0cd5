set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_conv_gpu.py -k "big_tile" > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_ENVS="LDNN_CONV_HB=0 LDNN_CONV_HB=1" bash scripts/gpu_run.sh r5ab ab:resnet18:64,resnet18:256 || exit 4
for pr in 0 1 0 1; do
  LDNN_RCCL_HIGH_PRIO=$pr bash scripts/gpu_run.sh r5ab probe:mlp3@16384@8 || exit 5
done
LDNN_RCCL_HIGH_PRIO=1 bash scripts/gpu_run.sh r5ab probe:enhanced_cnn@64@8@1@adam probe:resnet18@64@8 || exit 6
echo done
