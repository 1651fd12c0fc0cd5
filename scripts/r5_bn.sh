set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5bn; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_bn_pool_gpu.py > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.txt
[ $rc -eq 0 ] || exit $rc
AB_ENVS="X=0 LDNN_BN_SMALL_ROWS=0" bash scripts/gpu_run.sh r5bn ab:enhanced_cnn:64 || exit 4
AB_ENVS="X=0 LDNN_BN_RED_BLOCKS=1024 LDNN_BN_RED_BLOCKS=2048 LDNN_BN_RED_ROWS=4" bash scripts/gpu_run.sh r5bn ab:resnet18:256,resnet18:64 || exit 5
echo done
